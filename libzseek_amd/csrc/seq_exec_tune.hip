// seq_exec_tune.hip — tuning builds only (libzseek_tune.so, -DZSK_TUNING;
// never in the product library): the execute's diagnostic kernel and its
// round-0 / rounds experiments, timed against the production kernel by
// scripts/kbench.py through launch_seq_exec's `version` (tuning.hip).
//
// seq_exec_diag_kernel<DIAG, OUTB, SEG, WPE> is the production kernel's loop
// with every DIAG variant (bits below) still in place; the production kernel
// (seq_exec_dev.h) carries none of them.  Round 6: the
// round-0 entry experiments copy_entries (64-byte entries, four lanes each),
// copy_entries2 (a lane per entry, literal / match / short passes),
// copy_entries3 (one mixed pass) -- all slower than the descriptor deal; the
// 32-bit descriptor adds (bit 22) and copy_entries2 for the rounds (kDiagLR)
// were kept (copy_round0, copy_ready).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "seq_exec_dev.h"

namespace zsk {

namespace {

// traffic split (tuning only): round 0's literal pieces / HBM match pieces
// not loaded (zeros staged instead: the output is not checked)
constexpr int kDiagNoLit = 1 << 23, kDiagNoMatch = 1 << 24;

__device__ unsigned long long g_xstats[12];   // DIAG 16: cycles per section, counts

// Copy, for every lane, a literal run (lit bytes of the literal source at src
// -> output op) and a match run (mn bytes from output msrc -> mb; final
// source, no overlap) into the stage.  Each lane writes one 8-byte descriptor
// per 16-byte piece (stage destination, length, kind, source) at its
// piece-prefix position in LDS — piece o of a run is base + o * (1 + 2^32),
// source and destination advancing together, a match piece's kind turning
// from HBM to stage once its source reaches `flushed`; then the wave's pieces
// are dealt one per lane per slot, four slots' flat 16-byte loads in flight
// before any write.  A literal run under 16 bytes whose 16-byte piece would
// pass the end of the literal source (the frame's last literals: 16 bytes
// from their start can pass the frame's end mark, and the last frame's the
// end of the caller's buffer) is copied by its lane first, through the
// range-checked resource `lsp` (bytes past llen read as zero), and gets no
// descriptor.
template <int DIAG>
__device__ __forceinline__ void copy_desc3(const Stage &S, const uint8_t *lbase, const Span &lsp,
                                           uint32_t llen, const uint8_t *obase, uint32_t descs,
                                           uint32_t flushed, uint32_t lane, uint32_t src, uint32_t op,
                                           uint32_t lit, uint32_t msrc, uint32_t mb, uint32_t mn)
{
    const bool ltail = lit != 0 && lit < 16 && src + 16 > llen;
    if (__ballot(ltail)) {
        if (ltail)
            lds_put(saddr(S, op), bload16(lsp.r, lsp.s0 + src), lit);
    }
    const uint32_t lpn = ltail ? 0 : npieces(lit), np = lpn + npieces(mn);
    const uint32_t inc = wave_incl_add(np);
    const uint32_t T = lane_val(inc, 63);
    if (T == 0)
        return;
    const uint32_t x = inc - np;
    const uint64_t dl = ((uint64_t)((saddr(S, op) - S.base) | (lit < 16 ? lit : 16) << 16 | K_LIT << 24) << 32) | src;
    const uint64_t dm = ((uint64_t)((saddr(S, mb) - S.base) | (mn < 16 ? mn : 16) << 16 | K_HBM << 24) << 32) | msrc;
    const uint32_t lm = lit < 16 ? 0 : lit - 16, mm = mn < 16 ? 0 : mn - 16;
    // piece i of the literal run and piece i of the match in one step: as
    // many steps as the batch's longest run, no per-piece selects between
    // the two (one step per piece of the longest literal + match cost ~22
    // VALU per step)
    const uint32_t al = descs + 8 * x;
    for (uint32_t i = 0; __ballot(i < lpn || i + lpn < np); i++) {
        if (i < lpn) {
            const uint32_t o = min(16 * i, lm);
            *lp<uint64_t>(al + 8 * i) = dl + (uint64_t)o * 0x100000001ull;
        }
        if (i + lpn < np) {
            const uint32_t o = min(16 * i, mm);
            uint64_t D = dm + (uint64_t)o * 0x100000001ull;
            if (msrc + o + 16 > flushed)
                D += (uint64_t)(K_STAGE - K_HBM) << 56;
            *lp<uint64_t>(al + 8 * (lpn + i)) = D;
        }
    }
    wave_lds_sync();
    for (uint32_t t0 = 0; t0 < T; t0 += 256) {
        u32x4 v[4];
        uint32_t dw[4], sx[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t t = t0 + 64 * j + lane;
            const bool on = t < T;
            const uint64_t D = *lp<uint64_t>(descs + 8 * (on ? t : 0));
            // an idle lane loads the literal source's first 16 bytes (its kind
            // reads as K_LIT: a stale source offset there could be a match's
            // output offset, far past a big frame's compressed bytes)
            sx[j] = on ? (uint32_t)D : 0;
            dw[j] = on ? (uint32_t)(D >> 32) : 0;
            const uint32_t kind = dw[j] >> 24;
            const uint8_t *p = kind == K_HBM ? obase + sx[j] : lbase + (kind == K_LIT ? sx[j] : 0);
            v[j] = (DIAG & 1) ? (u32x4){0, 0, 0, 0} : *reinterpret_cast<const u32x4_l *>(p);
            if (t0 + 64 * j + 64 >= T)
                break;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t n = (dw[j] >> 16) & 0xFF;
            if (n) {
                u32x4 w = v[j];
                if ((dw[j] >> 24) == K_STAGE)
                    w = lds16(saddr(S, sx[j]));
                lds_put(S.base + (dw[j] & 0xFFFF), w, n);
            }
            if (t0 + 64 * j + 64 >= T)
                break;
        }
    }
}

// Round 0 with the pieces split by size: a run of 16 bytes or more is covered
// by whole 16-byte pieces only (its last piece overlaps the one before), so
// only runs under 16 bytes need an exact-length stage write.  Whole pieces
// (descriptors [0, TF)) are dealt as in copy_desc3 and written with one
// 16-byte LDS store each, no length branches; the short ones (at most two per
// lane, descriptors [TF, TF + TS)) follow in their own deal with the exact
// write.  One DPP scan counts both (whole pieces in the low half-word).
template <int DIAG>
__device__ __forceinline__ void copy_desc4(const Stage &S, const uint8_t *lbase, const Span &lsp,
                                           uint32_t llen, const uint8_t *obase, uint32_t descs,
                                           uint32_t flushed, uint32_t lane, uint32_t src, uint32_t op,
                                           uint32_t lit, uint32_t msrc, uint32_t mb, uint32_t mn)
{
    const bool ltail = lit != 0 && lit < 16 && src + 16 > llen;
    if (__ballot(ltail)) {
        if (ltail)
            lds_put(saddr(S, op), bload16(lsp.r, lsp.s0 + src), lit);
    }
    const bool ls = lit != 0 && lit < 16 && !ltail, ms = mn != 0 && mn < 16;
    const uint32_t lpn = lit < 16 ? 0 : npieces(lit), mpn = mn < 16 ? 0 : npieces(mn);
    const uint32_t nf = lpn + mpn, ns = (uint32_t)ls + (uint32_t)ms;
    const uint32_t inc = wave_incl_add(nf | ns << 16);
    const uint32_t T = lane_val(inc, 63);
    if (T == 0)
        return;
    const uint32_t TF = T & 0xFFFF, TS = T >> 16;
    const uint32_t xf = (inc & 0xFFFF) - nf, xs = TF + (inc >> 16) - ns;
    const uint64_t dl = ((uint64_t)((saddr(S, op) - S.base) | (lit < 16 ? lit : 16) << 16 | K_LIT << 24) << 32) | src;
    const uint64_t dm = ((uint64_t)((saddr(S, mb) - S.base) | (mn < 16 ? mn : 16) << 16 | K_HBM << 24) << 32) | msrc;
    const uint64_t kst = (uint64_t)(K_STAGE - K_HBM) << 56;
    // the short pieces: one descriptor each
    if (ls)
        *lp<uint64_t>(descs + 8 * xs) = dl;
    if (ms)
        *lp<uint64_t>(descs + 8 * (xs + ls)) = msrc + 16 > flushed ? dm + kst : dm;
    const uint32_t lm = lit < 16 ? 0 : lit - 16, mm = mn < 16 ? 0 : mn - 16;
    const uint32_t al = descs + 8 * xf;
    if (DIAG & 4096) {
        // two pieces of each run per step (one 16-byte descriptor store)
        for (uint32_t i = 0; __ballot(i < lpn || i < mpn); i += 2) {
            if (i < lpn) {
                const uint32_t o0 = min(16 * i, lm), o1 = min(16 * i + 16, lm);
                const uint64_t d0 = dl + (uint64_t)o0 * 0x100000001ull, d1 = dl + (uint64_t)o1 * 0x100000001ull;
                if (i + 1 < lpn)
                    *lp<u32x4_l>(al + 8 * i) = (u32x4){(uint32_t)d0, (uint32_t)(d0 >> 32), (uint32_t)d1,
                                                       (uint32_t)(d1 >> 32)};
                else
                    *lp<uint64_t>(al + 8 * i) = d0;
            }
            if (i < mpn) {
                const uint32_t o0 = min(16 * i, mm), o1 = min(16 * i + 16, mm);
                uint64_t d0 = dm + (uint64_t)o0 * 0x100000001ull, d1 = dm + (uint64_t)o1 * 0x100000001ull;
                d0 += msrc + o0 + 16 > flushed ? kst : 0;
                d1 += msrc + o1 + 16 > flushed ? kst : 0;
                if (i + 1 < mpn)
                    *lp<u32x4_l>(al + 8 * (lpn + i)) = (u32x4){(uint32_t)d0, (uint32_t)(d0 >> 32), (uint32_t)d1,
                                                               (uint32_t)(d1 >> 32)};
                else
                    *lp<uint64_t>(al + 8 * (lpn + i)) = d0;
            }
        }
    } else if (DIAG & 32768) {
        // (tuning) runs of at most kShortRun pieces: the lane writes its own (at most
        // kShortRun steps, both descriptor halves advanced by 32-bit adds);
        // longer runs: the whole wave writes one run's pieces per step
        constexpr uint32_t kShortRun = 6;
        const uint32_t lq = lpn <= kShortRun ? lpn : 0, mq = mpn <= kShortRun ? mpn : 0;
        const uint32_t dl0 = (uint32_t)dl, dl1 = (uint32_t)(dl >> 32);
        const uint32_t dm0 = (uint32_t)dm, dm1 = (uint32_t)(dm >> 32);
        constexpr uint32_t kst1 = (K_STAGE - K_HBM) << 24;
        for (uint32_t i = 0; __ballot(i < lq || i < mq); i++) {
            if (i < lq) {
                const uint32_t o = min(16 * i, lm);
                *lp<u32x2>(al + 8 * i) = (u32x2){dl0 + o, dl1 + o};
            }
            if (i < mq) {
                const uint32_t o = min(16 * i, mm);
                *lp<u32x2>(al + 8 * (lpn + i)) = (u32x2){dm0 + o, dm1 + o + (msrc + o + 16 > flushed ? kst1 : 0)};
            }
        }
        for (uint64_t L = __ballot(lpn > kShortRun); L; L &= L - 1) {
            const int j = (int)__builtin_ctzll(L);
            const uint32_t n = lane_val(lpn, j), m = lane_val(lm, j), a = lane_val(al, j);
            const uint32_t d0 = lane_val(dl0, j), d1 = lane_val(dl1, j);
            for (uint32_t i = lane; i < n; i += 64) {
                const uint32_t o = min(16 * i, m);
                *lp<u32x2>(a + 8 * i) = (u32x2){d0 + o, d1 + o};
            }
        }
        for (uint64_t M = __ballot(mpn > kShortRun); M; M &= M - 1) {
            const int j = (int)__builtin_ctzll(M);
            const uint32_t n = lane_val(mpn, j), m = lane_val(mm, j), a = lane_val(al + 8 * lpn, j);
            const uint32_t d0 = lane_val(dm0, j), d1 = lane_val(dm1, j), sm = lane_val(msrc, j);
            for (uint32_t i = lane; i < n; i += 64) {
                const uint32_t o = min(16 * i, m);
                *lp<u32x2>(a + 8 * i) = (u32x2){d0 + o, d1 + o + (sm + o + 16 > flushed ? kst1 : 0)};
            }
        }
    } else if (DIAG & (1 << 22)) {
        // both descriptor halves advanced by 32-bit adds (the 64-bit form
        // compiles to v_mad_u64_u32, two per step)
        const uint32_t dl0 = (uint32_t)dl, dl1 = (uint32_t)(dl >> 32);
        const uint32_t dm0 = (uint32_t)dm, dm1 = (uint32_t)(dm >> 32);
        constexpr uint32_t kst1 = (K_STAGE - K_HBM) << 24;
        const uint32_t am = al + 8 * lpn;
        for (uint32_t i = 0; __ballot(i < lpn || i < mpn); i++) {
            if (i < lpn) {
                const uint32_t o = min(16 * i, lm);
                *lp<u32x2>(al + 8 * i) = (u32x2){dl0 + o, dl1 + o};
            }
            if (i < mpn) {
                const uint32_t o = min(16 * i, mm);
                *lp<u32x2>(am + 8 * i) = (u32x2){dm0 + o, dm1 + o + (msrc + o + 16 > flushed ? kst1 : 0)};
            }
        }
    } else {
        for (uint32_t i = 0; __ballot(i < lpn || i < mpn); i++) {
            if (i < lpn) {
                const uint32_t o = min(16 * i, lm);
                *lp<uint64_t>(al + 8 * i) = dl + (uint64_t)o * 0x100000001ull;
            }
            if (i < mpn) {
                const uint32_t o = min(16 * i, mm);
                uint64_t D = dm + (uint64_t)o * 0x100000001ull;
                if (msrc + o + 16 > flushed)
                    D += kst;
                *lp<uint64_t>(al + 8 * (lpn + i)) = D;
            }
        }
    }
    wave_lds_sync();
    // one deal over [0, TF + TS): four slots' loads in flight, then the
    // writes -- a slot holding short pieces (at most the last two) writes
    // exact lengths, every other slot plain 16-byte stores
    const uint32_t TT = TF + TS;
    for (uint32_t t0 = 0; t0 < TT; t0 += 256) {
        u32x4 v[4];
        uint32_t dw[4], sx[4];
        if (DIAG & 8192) {
            // the step's descriptors read together (one LDS wait), then the
            // loads: slots past the step's count are skipped uniformly
            const uint32_t ns = min(4u, (TT - t0 + 63) >> 6);
            uint64_t D[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t t = t0 + 64 * j + lane;
                D[j] = (uint32_t)j < ns ? *lp<uint64_t>(descs + 8 * (t < TT ? t : 0)) : 0;
                if (t >= TT)
                    D[j] = 0;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                sx[j] = (uint32_t)D[j];
                dw[j] = (uint32_t)(D[j] >> 32);
                if ((uint32_t)j < ns) {
                    const uint32_t kind = dw[j] >> 24;
                    const uint8_t *p = kind == K_HBM ? obase + sx[j] : lbase + (kind == K_LIT ? sx[j] : 0);
                    v[j] = (DIAG & 1) ? (u32x4){0, 0, 0, 0} : *reinterpret_cast<const u32x4_l *>(p);
                }
            }
        } else
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t t = t0 + 64 * j + lane;
            const bool on = t < TT;
            const uint64_t D = *lp<uint64_t>(descs + 8 * (on ? t : 0));
            sx[j] = on ? (uint32_t)D : 0;
            dw[j] = on ? (uint32_t)(D >> 32) : 0;
            const uint32_t kind = dw[j] >> 24;
            const uint8_t *p = kind == K_HBM ? obase + sx[j] : lbase + (kind == K_LIT ? sx[j] : 0);
            // (traffic split: kDiagNoLit / kDiagNoMatch leave one kind's pieces unloaded)
            const bool skip = (DIAG & 1) || ((DIAG & kDiagNoLit) && kind == K_LIT) ||
                              ((DIAG & kDiagNoMatch) && kind == K_HBM);
            v[j] = skip ? (u32x4){0, 0, 0, 0} : *reinterpret_cast<const u32x4_l *>(p);
            if (t0 + 64 * j + 64 >= TT)
                break;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (dw[j]) {
                u32x4 w = v[j];
                if ((dw[j] >> 24) == K_STAGE)
                    w = lds16(saddr(S, sx[j]));
                if (t0 + 64 * j + 64 <= TF)
                    *lp<u32x4_l>(S.base + (dw[j] & 0xFFFF)) = w;
                else
                    lds_put(S.base + (dw[j] & 0xFFFF), w, (dw[j] >> 16) & 0xFF);
            }
            if (t0 + 64 * j + 64 >= TT)
                break;
        }
    }
}
// ---- round 0 and the dependency rounds in 64-byte entries (round 6) ----------
// copy_desc4 gives every 16-byte piece of every run its own descriptor: the
// descriptor loop runs once per piece of the batch's longest run (11.0 steps
// per config-2 batch, measured on the LZ4 stream of the synthetic:
// scripts/exec_model.py) for ~159 pieces dealt in ~3 wave steps.  Here a run
// of L >= 16 bytes takes ceil(L / 64) entries of 8 bytes -- source, stage
// destination, min(L - 64 i, 64) bytes left, kind -- and four lanes deal one
// entry, lane k its piece at min(16 k, left - 16) (a run's last pieces overlap
// the ones before and rewrite equal bytes; left < 16 only past the run's first
// entry, so that piece starts inside the run): 3.1 loop steps and ~58 entries
// in ~4 wave steps per batch.  Runs under 16 bytes (both copy_desc4's short
// pieces) keep one lane and an exact-length write.  A match piece reads HBM
// when its 16 bytes lie below `flushed`, else the stage.

// entries [0, TE) at descs, four lanes each; then the short runs [TE, TE + TS),
// a lane each
__device__ __forceinline__ void deal_entries(const Stage &S, const uint8_t *lbase, const uint8_t *obase,
                                             uint32_t descs, uint32_t flushed, uint32_t lane, uint32_t TE,
                                             uint32_t TS)
{
    const uint32_t k16 = 16 * (lane & 3), eg = lane >> 2;
    for (uint32_t e0 = 0; e0 < TE; e0 += 64) {
        u32x4 v[4];
        uint32_t da[4], sa[4];
        bool act[4], stg[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t e = e0 + 16 * j + eg;
            const bool on = e < TE;
            const uint64_t D = *lp<uint64_t>(descs + 8 * (on ? e : 0));
            const uint32_t hi = (uint32_t)(D >> 32);
            const uint32_t left = (hi >> kEntryLeftShift) & 0x7F;
            const int32_t o = min((int32_t)k16, (int32_t)left - 16);
            const uint32_t s = (uint32_t)D + (uint32_t)o;
            const bool lit = (hi >> kEntryKindShift) == K_LIT;
            act[j] = on && k16 < left;
            stg[j] = !lit && s + 16 > flushed;
            sa[j] = s;
            da[j] = S.base + (hi & 0xFFFF) + (uint32_t)o;
            const uint8_t *p = act[j] && !stg[j] ? (lit ? lbase : obase) + s : lbase;
            v[j] = *reinterpret_cast<const u32x4_l *>(p);
            if (e0 + 16 * j + 16 >= TE)
                break;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (act[j])
                *lp<u32x4_l>(da[j]) = stg[j] ? lds16(saddr(S, sa[j])) : v[j];
            if (e0 + 16 * j + 16 >= TE)
                break;
        }
    }
    for (uint32_t t0 = 0; t0 < TS; t0 += 64) {
        const uint32_t t = t0 + lane;
        const bool on = t < TS;
        const uint64_t D = *lp<uint64_t>(descs + 8 * (TE + (on ? t : 0)));
        const uint32_t hi = (uint32_t)(D >> 32), s = (uint32_t)D;
        const bool lit = (hi >> kEntryKindShift) == K_LIT;
        const bool stg = !lit && s + 16 > flushed;
        const uint8_t *p = on && !stg ? (lit ? lbase : obase) + s : lbase;
        const u32x4 v = *reinterpret_cast<const u32x4_l *>(p);
        if (on)
            lds_put(S.base + (hi & 0xFFFF), stg ? lds16(saddr(S, s)) : v, (hi >> kEntryLeftShift) & 0x7F);
    }
}

// Entries for every lane's literal run (lit bytes of the literal source at src
// -> output op) and match (mn bytes from output msrc -> mb, final source, no
// overlap), then the deal.  A literal run under 16 bytes whose 16-byte load
// would pass llen is copied by its lane first, through the range-checked
// resource (as copy_desc4).
__device__ __forceinline__ void copy_entries(const Stage &S, const uint8_t *lbase, const Span &lsp, uint32_t llen,
                                             const uint8_t *obase, uint32_t descs, uint32_t flushed, uint32_t lane,
                                             uint32_t src, uint32_t op, uint32_t lit, uint32_t msrc, uint32_t mb,
                                             uint32_t mn)
{
    const bool ltail = lit != 0 && lit < 16 && src + 16 > llen;
    if (__ballot(ltail)) {
        if (ltail)
            lds_put(saddr(S, op), bload16(lsp.r, lsp.s0 + src), lit);
    }
    const bool ls = lit != 0 && lit < 16 && !ltail, ms = mn != 0 && mn < 16;
    const uint32_t nl = lit < 16 ? 0 : (lit + 63) >> 6, nm = mn < 16 ? 0 : (mn + 63) >> 6;
    const uint32_t ne = nl + nm, ns = (uint32_t)ls + (uint32_t)ms;
    const uint32_t inc = wave_incl_add(ne | ns << 16);
    const uint32_t T = lane_val(inc, 63);
    if (T == 0)
        return;
    const uint32_t TE = T & 0xFFFF, TS = T >> 16;
    const uint32_t xe = (inc & 0xFFFF) - ne, xs = TE + (inc >> 16) - ns;
    const uint32_t dl = (saddr(S, op) - S.base) | K_LIT << kEntryKindShift;
    const uint32_t dm = (saddr(S, mb) - S.base) | K_HBM << kEntryKindShift;
    if (ls)
        *lp<u32x2>(descs + 8 * xs) = (u32x2){src, dl | lit << kEntryLeftShift};
    if (ms)
        *lp<u32x2>(descs + 8 * (xs + ls)) = (u32x2){msrc, dm | mn << kEntryLeftShift};
    const uint32_t al = descs + 8 * xe, am = al + 8 * nl;
    for (uint32_t i = 0; __ballot(i < nl || i < nm); i++) {
        const uint32_t o = 64 * i;
        if (i < nl)
            *lp<u32x2>(al + 8 * i) = (u32x2){src + o, dl + o + (min(lit - o, 64u) << kEntryLeftShift)};
        if (i < nm)
            *lp<u32x2>(am + 8 * i) = (u32x2){msrc + o, dm + o + (min(mn - o, 64u) << kEntryLeftShift)};
    }
    wave_lds_sync();
    deal_entries(S, lbase, obase, descs, flushed, lane, TE, TS);
}
// copy_entries with one lane per entry: literal entries [0, TL), match entries
// [TL, TL + TM), short runs after them (one scan counts all three)
__device__ __forceinline__ void copy_entries2(const Stage &S, const uint8_t *lbase, const Span &lsp, uint32_t llen,
                                              const Out &O, uint32_t descs, uint32_t flushed, uint32_t lane,
                                              uint32_t src, uint32_t op, uint32_t lit, uint32_t msrc, uint32_t mb,
                                              uint32_t mn)
{
    const bool ltail = lit != 0 && lit < 16 && src + 16 > llen;
    if (__ballot(ltail)) {
        if (ltail)
            lds_put(saddr(S, op), bload16(lsp.r, lsp.s0 + src), lit);
    }
    const bool ls = lit != 0 && lit < 16 && !ltail, ms = mn != 0 && mn < 16;
    const uint32_t nl = lit < 16 ? 0 : (lit + 63) >> 6, nm = mn < 16 ? 0 : (mn + 63) >> 6;
    const uint32_t ns = (uint32_t)ls + (uint32_t)ms;
    const uint32_t inc = wave_incl_add(nl | nm << 8 | ns << 16);
    const uint32_t T = lane_val(inc, 63);
    if (T == 0)
        return;
    const uint32_t TL = T & 0xFF, TM = (T >> 8) & 0xFF, TS = T >> 16;
    const uint32_t xl = (inc & 0xFF) - nl, xm = TL + ((inc >> 8) & 0xFF) - nm, xs = TL + TM + (inc >> 16) - ns;
    const uint32_t dl = (saddr(S, op) - S.base) | K_LIT << kEntryKindShift;
    const uint32_t dm = (saddr(S, mb) - S.base) | K_HBM << kEntryKindShift;
    if (ls)
        *lp<u32x2>(descs + 8 * xs) = (u32x2){src, dl | lit << kEntryLeftShift};
    if (ms)
        *lp<u32x2>(descs + 8 * (xs + ls)) = (u32x2){msrc, dm | mn << kEntryLeftShift};
    const uint32_t al = descs + 8 * xl, am = descs + 8 * xm;
    for (uint32_t i = 0; __ballot(i < nl || i < nm); i++) {
        const uint32_t o = 64 * i;
        if (i < nl)
            *lp<u32x2>(al + 8 * i) = (u32x2){src + o, dl + o + (min(lit - o, 64u) << kEntryLeftShift)};
        if (i < nm)
            *lp<u32x2>(am + 8 * i) = (u32x2){msrc + o, dm + o + (min(mn - o, 64u) << kEntryLeftShift)};
    }
    wave_lds_sync();
    if (TL)
        deal_lane<true>(S, lsp, O, descs, flushed, lane, 0, TL);
    if (TM)
        deal_lane<false>(S, lsp, O, descs, flushed, lane, TL, TM);
    for (uint32_t t0 = 0; t0 < TS; t0 += 64) {
        const uint32_t t = t0 + lane;
        if (t < TS) {
            const uint64_t D = *lp<uint64_t>(descs + 8 * (TL + TM + t));
            const uint32_t hi = (uint32_t)(D >> 32), s = (uint32_t)D;
            u32x4 v;
            if ((hi >> kEntryKindShift) == K_LIT)
                v = bload16(lsp.r, lsp.s0 + s);
            else if (s + 16 <= flushed)
                v = bload16(O.sp.r, O.sp.s0 + s);
            else
                v = lds16(saddr(S, s));
            lds_put(S.base + (hi & 0xFFFF), v, (hi >> kEntryLeftShift) & 0x7F);
        }
    }
}
// copy_entries2 waited on the global loads three times per batch (literal
// entries, match entries, short runs; each a branch of its own): VALU per
// frame 15.8K -> 13.8K but the execute 2.41 -> 2.74 ms.  Here a lane takes
// entry t of one mixed list and short run t together, every load issued
// before any store (one wait per 64 entries), inactive pieces loading at an
// out-of-range offset (zeros, no branch).  Match pieces whose bytes reach
// `flushed` (only at the kept chunk before the batch) are copied from the
// stage after the others.
__device__ __forceinline__ void copy_entries3(const Stage &S, const uint8_t *lbase, const Span &lsp, uint32_t llen,
                                              const Out &O,
                                              uint32_t descs, uint32_t flushed, uint32_t lane, uint32_t src,
                                              uint32_t op, uint32_t lit, uint32_t msrc, uint32_t mb, uint32_t mn)
{
    const bool ltail = lit != 0 && lit < 16 && src + 16 > llen;
    if (__ballot(ltail)) {
        if (ltail)
            lds_put(saddr(S, op), bload16(lsp.r, lsp.s0 + src), lit);
    }
    const bool ls = lit != 0 && lit < 16 && !ltail, ms = mn != 0 && mn < 16;
    const uint32_t nl = lit < 16 ? 0 : (lit + 63) >> 6, nm = mn < 16 ? 0 : (mn + 63) >> 6;
    const uint32_t ne = nl + nm, ns = (uint32_t)ls + (uint32_t)ms;
    const uint32_t inc = wave_incl_add(ne | ns << 16);
    const uint32_t T = lane_val(inc, 63);
    if (T == 0)
        return;
    const uint32_t TE = T & 0xFFFF, TS = T >> 16;
    const uint32_t xe = (inc & 0xFFFF) - ne, xs = TE + (inc >> 16) - ns;
    const uint32_t dl = (saddr(S, op) - S.base) | K_LIT << kEntryKindShift;
    const uint32_t dm = (saddr(S, mb) - S.base) | K_HBM << kEntryKindShift;
    if (ls)
        *lp<u32x2>(descs + 8 * xs) = (u32x2){src, dl | lit << kEntryLeftShift};
    if (ms)
        *lp<u32x2>(descs + 8 * (xs + ls)) = (u32x2){msrc, dm | mn << kEntryLeftShift};
    const uint32_t al = descs + 8 * xe, am = al + 8 * nl;
    for (uint32_t i = 0; __ballot(i < nl || i < nm); i++) {
        const uint32_t o = 64 * i;
        if (i < nl)
            *lp<u32x2>(al + 8 * i) = (u32x2){src + o, dl + o + (min(lit - o, 64u) << kEntryLeftShift)};
        if (i < nm)
            *lp<u32x2>(am + 8 * i) = (u32x2){msrc + o, dm + o + (min(mn - o, 64u) << kEntryLeftShift)};
    }
    wave_lds_sync();
    const uint32_t TT = TE > TS ? TE : TS;
    for (uint32_t t0 = 0; t0 < TT; t0 += 64) {
        const uint32_t t = t0 + lane;
        const bool eon = t < TE, son = t < TS;
        const uint64_t D = *lp<uint64_t>(descs + 8 * (eon ? t : 0));
        const uint64_t E = *lp<uint64_t>(descs + 8 * (TE + (son ? t : 0)));
        const uint32_t hi = (uint32_t)(D >> 32), s = (uint32_t)D;
        const int32_t left = eon ? (int32_t)((hi >> kEntryLeftShift) & 0x7F) : 0;
        const bool elit = (hi >> kEntryKindShift) == K_LIT;
        int32_t r[4];
        bool act[4], stg[4];
        uint32_t off[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            r[q] = min(16 * q, left - 16);
            act[q] = 16 * q < left;
            const uint32_t x = s + (uint32_t)r[q];
            stg[q] = !elit && x + 16 > flushed;
            off[q] = act[q] && !stg[q] ? x : kBad;
        }
        // flat loads from a per-lane base (a buffer resource chosen per lane
        // compiles to a waterfall loop per load); an inactive piece loads the
        // base's first bytes
        const uint8_t *eb = elit ? lbase : O.o;
        u32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; q++)
            v[q] = *reinterpret_cast<const u32x4_l *>(eb + (off[q] == kBad ? 0u : off[q]));
        const uint32_t shi = (uint32_t)(E >> 32), ss = (uint32_t)E;
        const bool slit = (shi >> kEntryKindShift) == K_LIT;
        const bool sstg = !slit && ss + 16 > flushed;
        const u32x4 sv0 = *reinterpret_cast<const u32x4_l *>((slit ? lbase : O.o) + (son && !sstg ? ss : 0u));
        u32x4 sv = sv0;
        const uint32_t d = S.base + (hi & 0xFFFF);
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (act[q] && !stg[q])
                *lp<u32x4_l>(d + (uint32_t)r[q]) = v[q];
        if (son) {
            if (sstg)
                sv = lds16(saddr(S, ss));
            lds_put(S.base + (shi & 0xFFFF), sv, (shi >> kEntryLeftShift) & 0x7F);
        }
        if (__ballot(stg[0] || stg[1] || stg[2] || stg[3])) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (act[q] && stg[q])
                    *lp<u32x4_l>(d + (uint32_t)r[q]) = lds16(saddr(S, s + (uint32_t)r[q]));
        }
    }
}

// The first w bytes of a at LDS address d and of b at d + n - w: a run of n
// bytes (1..32) written whole-width with at most two stores (w = 16, 8, 4, 2
// or 1 by n; the two overlap below 2w bytes and rewrite equal bytes), never a
// byte outside [d, d + n).
__device__ __forceinline__ void put_ends(uint32_t d, uint32_t n, const u32x4 &a, const u32x4 &b)
{
    if (n >= 16) {
        *lp<u32x4_l>(d) = a;
        *lp<u32x4_l>(d + n - 16) = b;
    } else if (n >= 8) {
        *lp<u64_l>(d) = ((uint64_t)a.y << 32) | a.x;
        *lp<u64_l>(d + n - 8) = ((uint64_t)b.y << 32) | b.x;
    } else if (n >= 4) {
        *lp<u32_l>(d) = a.x;
        *lp<u32_l>(d + n - 4) = b.x;
    } else if (n >= 2) {
        *lp<u16_l>(d) = (uint16_t)a.x;
        *lp<u16_l>(d + n - 2) = (uint16_t)b.x;
    } else if (n) {
        *lp<uint8_t>(d) = (uint8_t)a.x;
    }
}

// Round 0, direct (round 5): every lane copies its own literal run and its
// early match (source before the batch) itself -- the run's first bytes and
// its last bytes (put_ends: all of a run of up to 32 bytes, at most two
// stores) -- and only the middle 16-byte pieces of runs longer than 32 bytes
// go through descriptors and the deal.  copy_desc4 sent every piece of every
// run through the descriptor table (one descriptor loop step per piece of the
// batch's longest run, ~3 deal slots per batch): the round cost ~300 VALU per
// 64-sequence batch, 48 % of the execute's.  Literal loads go through the
// frame's resource (the bytes a run needs lie 4+ bytes before its end: the
// end mark), match loads through the output's (below `flushed`) or the stage.
template <int DIAG>
__device__ __forceinline__ void copy_direct(const Stage &S, const uint8_t *lbase, const Span &lsp,
                                            const Out &O, uint32_t descs, uint32_t flushed, uint32_t lane,
                                            uint32_t src, uint32_t op, uint32_t lit, uint32_t msrc, uint32_t mb,
                                            uint32_t mn)
{
    const uint32_t wl = lit >= 16 ? 16 : lit >= 8 ? 8 : lit >= 4 ? 4 : lit >= 2 ? 2 : lit;
    const uint32_t wm = mn >= 16 ? 16 : mn >= 8 ? 8 : mn >= 4 ? 4 : mn;   // (matches: >= 4 bytes)
    // loads: the run's first 16 bytes and the 16 from its last w bytes' start
    const uint32_t lt = src + lit - wl;
    const u32x4 la = bload16(lsp.r, lit ? lsp.s0 + src : kBad);
    const u32x4 lb = bload16(lsp.r, lit ? lsp.s0 + lt : kBad);
    const uint32_t mt = msrc + mn - wm;
    const bool ha = mn && msrc + 16 <= flushed, hb = mn && mt + 16 <= flushed;
    const u32x4 ma_h = bload16(O.sp.r, ha ? O.sp.s0 + msrc : kBad);
    const u32x4 mb_h = bload16(O.sp.r, hb ? O.sp.s0 + mt : kBad);
    const u32x4 ma_s = lds16(mn && !ha ? saddr(S, msrc) : S.base);
    const u32x4 mb_s = lds16(mn && !hb ? saddr(S, mt) : S.base);
    // middle pieces of runs over 32 bytes: [16, n - 16) in 16-byte pieces
    const uint32_t lpn = lit > 32 ? (lit - 17) >> 4 : 0, mpn = mn > 32 ? (mn - 17) >> 4 : 0;
    const uint32_t nf = lpn + mpn;
    const uint32_t inc = wave_incl_add(nf);
    const uint32_t T = lane_val(inc, 63);
    put_ends(saddr(S, op), lit, la, lb);
    put_ends(saddr(S, mb), mn, ha ? ma_h : ma_s, hb ? mb_h : mb_s);
    if (T == 0)
        return;
    const uint64_t dl = ((uint64_t)((saddr(S, op) - S.base) | 16u << 16 | K_LIT << 24) << 32) | src;
    const uint64_t dm = ((uint64_t)((saddr(S, mb) - S.base) | 16u << 16 | K_HBM << 24) << 32) | msrc;
    const uint64_t kst = (uint64_t)(K_STAGE - K_HBM) << 56;
    const uint32_t al = descs + 8 * (inc - nf);
    for (uint32_t i = 0; __ballot(i < lpn || i < mpn); i++) {
        const uint32_t o = 16 * i + 16;
        if (i < lpn)
            *lp<uint64_t>(al + 8 * i) = dl + (uint64_t)o * 0x100000001ull;
        if (i < mpn)
            *lp<uint64_t>(al + 8 * (lpn + i)) = dm + (uint64_t)o * 0x100000001ull + (msrc + o + 16 > flushed ? kst : 0);
    }
    wave_lds_sync();
    for (uint32_t t0 = 0; t0 < T; t0 += 256) {
        u32x4 v[4];
        uint32_t dw[4], sx[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t t = t0 + 64 * j + lane;
            const bool on = t < T;
            const uint64_t D = *lp<uint64_t>(descs + 8 * (on ? t : 0));
            sx[j] = on ? (uint32_t)D : 0;
            dw[j] = on ? (uint32_t)(D >> 32) : 0;
            const uint32_t kind = dw[j] >> 24;
            const uint8_t *p = kind == K_HBM ? O.o + sx[j] : lbase + (kind == K_LIT ? sx[j] : 0);
            v[j] = *reinterpret_cast<const u32x4_l *>(p);
            if (t0 + 64 * j + 64 >= T)
                break;
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (dw[j]) {
                u32x4 w = v[j];
                if ((dw[j] >> 24) == K_STAGE)
                    w = lds16(saddr(S, sx[j]));
                *lp<u32x4_l>(S.base + (dw[j] & 0xFFFF)) = w;
            }
            if (t0 + 64 * j + 64 >= T)
                break;
        }
    }
}

// A ready match (mn bytes, msrc -> mb, no overlap) whose source lies in this
// batch: lane-owned pieces, two per step, from the stage (the HBM path only
// runs when some lane's piece lies below `flushed`).
__device__ __forceinline__ void copy_round(const Stage &S, const Out &O, uint32_t flushed,
                                           uint32_t msrc, uint32_t mb, uint32_t mn)
{
    const uint32_t mpn = npieces(mn), n0 = mn < 16 ? mn : 16;
    for (uint32_t j = 0; __ballot(j < mpn); j += 2) {
        const bool m0 = j < mpn, m1 = j + 1 < mpn;
        const uint32_t o0 = piece_off(mn, j), o1 = piece_off(mn, j + 1);
        const uint32_t s0 = msrc + o0, s1 = msrc + o1;
        const bool h0 = m0 && s0 + 16 <= flushed, h1 = m1 && s1 + 16 <= flushed;
        u32x4 v0 = lds16(m0 && !h0 ? saddr(S, s0) : S.base);
        u32x4 v1 = lds16(m1 && !h1 ? saddr(S, s1) : S.base);
        if (__ballot(h0 || h1)) {
            const u32x4 w0 = bload16(O.sp.r, h0 ? O.sp.s0 + s0 : kBad);
            const u32x4 w1 = bload16(O.sp.r, h1 ? O.sp.s0 + s1 : kBad);
            v0 = h0 ? w0 : v0;
            v1 = h1 ? w1 : v1;
        }
        if (m0)
            lds_put(saddr(S, mb + o0), v0, n0);
        if (m1)
            lds_put(saddr(S, mb + o1), v1, 16);
    }
}
// chunks [fc, end_c) -> HBM, lane-strided, four chunks' LDS reads in flight
// before their stores
template <int DIAG>
__device__ __forceinline__ void flush_chunks4d(const Stage &S, const Out &O, uint32_t fc, uint32_t end_c,
                                              uint32_t lane)
{
    // every chunk inside the frame (the usual batch: neither the frame's
    // first chunk when the output is not 16-byte aligned, nor its partial
    // last one): plain 16-byte stores through a resource based at chunk 0
    if (!(DIAG & 64) && (fc > 0 || S.a0 == 0) && 16 * end_c <= O.dlen + S.a0) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(O.o - S.a0), 0, (int)((O.dlen + S.a0 + 15) & ~15u), kRsrcDw3);
        for (uint32_t c0 = fc; c0 < end_c; c0 += 256) {
            u32x4 v[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t c = c0 + 64 * j + lane;
                v[j] = *lp<u32x4>(c < end_c ? S.base + 16u * (c - S.cb) : S.base);
                if (c0 + 64 * j + 64 >= end_c)
                    break;
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t c = c0 + 64 * j + lane;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[j]), r,
                                                       c < end_c ? 16 * c : 0x80000000u, 0, 0);
                if (c0 + 64 * j + 64 >= end_c)
                    break;
            }
        }
        return;
    }
    for (uint32_t c0 = fc; c0 < end_c; c0 += 256) {
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t c = c0 + 64 * j + lane;
            v[j] = *lp<u32x4>(c < end_c ? S.base + 16u * (c - S.cb) : S.base);
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t c = c0 + 64 * j + lane;
            if (c < end_c)
                put_chunk(O, S.a0, c, v[j]);
        }
    }
}
// DIAG (tuning builds only): 1 = no piece loads, 2 = no flush stores, 4 = no
// dependency rounds, 8 = no round 0, 16 = section timers and counters
// (g_xstats), 32 = no flush at all, 64 = round 3's flush (every chunk through
// put_chunk), 128 = round 3's round 0 (copy_desc3); inside the dependency
// rounds: 256 = no copy_round, 512 = no copy_overlap, 1024 = no readiness
// search (every pending match ready at once).  Tried and dropped in round 4:
// the pending matches one at a time in destination order over the whole wave
// (no readiness search; execute 4.23 vs 2.79 ms -- each match a serial LDS
// read-then-write), and round 0 / the rounds dealt from one table entry per
// run with a DPP max-scan (3.86 vs 2.71 ms: two dependent LDS reads per slot).
// Tried and dropped (same-box A/B, config 2): short runs'
// partial pieces dealt after the full pieces; each batch's flush deferred past
// the next batch's item decode; the rounds' readiness from an LDS bitmap; six
// waves per SIMD (80 VGPRs, spills); round 0's slot loads retired inside each
// deal step; O(1) readiness pre-tests before the binary search; a persistent
// grid with next-frame prefetch; nontemporal item / literal loads; 1, 2, 5 or
// 8 waves per workgroup instead of kXW = 4; the rounds' readiness by a
// uniform loop over the pending lanes with readlane (no compaction, no binary
// search: execute 2.886 vs 2.808 ms, more VALU per round).
[[maybe_unused]] constexpr int kDiagE0 = 1 << 17, kDiagER = 1 << 18;   // round 0 / the rounds through copy_entries
[[maybe_unused]] constexpr int kDiagEntries = kDiagE0 | kDiagER;
[[maybe_unused]] constexpr int kDiagL0 = 1 << 19, kDiagLR = 1 << 20;   // ... through copy_entries2 (a lane per entry)
[[maybe_unused]] constexpr int kDiagM0 = 1 << 21;   // round 0 through copy_entries3 (one mixed list, one wait)
template <int DIAG, uint32_t OUTB, bool SEG, int WPE = 0>
__global__ __launch_bounds__(64 * kXW) __attribute__((amdgpu_waves_per_eu(WPE ? WPE : SEG ? 4 : (OUTB <= 2560 ? 8 : OUTB <= 3072 ? 7 : OUTB <= 3584 ? 6 : 5)))) void seq_exec_diag_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ rec_base,
    const uint64_t *__restrict__ items, const uint32_t *__restrict__ nitems,
    const int32_t *__restrict__ status, const uint8_t *__restrict__ lit,
    const uint32_t *__restrict__ bfirst, const uint32_t *__restrict__ bcount,
    const BlockJob *__restrict__ jobs, const BlockRes *__restrict__ jres, uint32_t stop_last,
    uint32_t min_dsize)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[kXW * x_wave(OUTB) + (SEG ? kXW * 8 * 65 : 0)];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t f = uni(blockIdx.x * kXW + w);
    if (f >= n)
        return;
    // a frame the parse (LZ4) or the sequence kernel (zstd) failed is executed
    // over the items it emitted (every one validated; the blocks before the
    // failing one), so its bytes before fail_at are in place for partial
    // reads; hand-offs are left to the wave kernel
    const int32_t fst = (int32_t)uni((uint32_t)status[f]);
    if (fst == ST_NOT_RUN)
        return;
    const FrameDesc d = desc[f];
    if (d.d_size < min_dsize)
        return;   // seq_exec_frame_kernel's frame (the one-frame route)
    JobMap<SEG> J;
    uint32_t ispan = 0;   // item slots the resource covers (SEG)
    const uint32_t nit = SEG ? J.init(bfirst, bcount, jobs, jres, f, nitems,
                                      (uint32_t)(uintptr_t)(lds + kXW * x_wave(OUTB)) + w * 8 * 65, lane, ispan)
                             : uni(nitems[f]);
    const uint64_t *it = items + rec_base[f];
    // the frame's items as a buffer resource: loads past nit return 0
    const __amdgpu_buffer_rsrc_t irs =
        __builtin_amdgcn_make_buffer_rsrc((void *)it, 0, (int)((SEG ? ispan : nit) * 8), kRsrcDw3);
    Out O;
    O.o = out + d.d_off;
    O.dlen = d.d_size;
    O.sp = make_span(O.o, d.d_size);
    // literal source: the compressed frame (LZ4), or the frame's decoded
    // literals (zstd scratch laid out like the output, 16 bytes of slack)
    const uint32_t llen = lit ? d.d_size + 16 : d.c_size;
    const uint8_t *lbase = lit ? lit + d.d_off : comp + d.c_off;
    const Span lsp = make_span(lbase, llen);
    Stage S;
    S.base = (uint32_t)(uintptr_t)(lds + w * x_wave(OUTB));
    const uint32_t descs = S.base + x_buf(OUTB);
    S.a0 = (uint32_t)(reinterpret_cast<uintptr_t>(O.o) & 15);
    S.cb = 0xFFFFFFFFu;      // chunk -1 at index 0: chunk 0 starts at index 16
    uint32_t produced = 0;   // frame bytes decoded
    uint32_t fc = 0;         // output chunks [0, fc) are in HBM
    uint64_t cur;
    if constexpr (SEG)
        cur = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(irs, J.addr(0, lane, nit), 0, 0));
    else
        cur = lane < nit ? it[lane] : 0;
    __builtin_amdgcn_s_waitcnt(0);   // cur in registers before the loop: its waits then leave nxt in flight
    uint32_t b = 0;
    uint64_t tsec[4] = {0, 0, 0, 0};
    uint32_t cnt[6] = {0, 0, 0, 0, 0, 0};
    uint64_t tmark = (DIAG & 16) ? __builtin_readcyclecounter() : 0;
#define ZSK_T(i)                                                      \
    if (DIAG & 16) {                                                  \
        __builtin_amdgcn_s_waitcnt(0);                                \
        const uint64_t tn = __builtin_readcyclecounter();             \
        tsec[i] += tn - tmark;                                        \
        tmark = tn;                                                   \
    }
    // the batch's last frame stops once it has produced stop_last bytes (a
    // no-cache request ending inside it needs no more; its later bytes are
    // never read back)
    const uint32_t stop = f + 1 == n ? stop_last : 0xFFFFFFFFu;
    while (b < nit && produced < stop) {
        const uint64_t nxt =
            __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(irs, J.addr(b + 64, lane, nit), 0, 0));
        const uint32_t w0 = (uint32_t)cur, w1 = (uint32_t)(cur >> 32);
        const uint32_t w0n = dpp_next(w0, 0), w1n = dpp_next(w1, 0);
        const uint32_t w0p = dpp_prev(w0, 0);
        const bool act0 = b + lane < nit;
        const uint32_t src = w0 & kItemPos;
        const uint32_t off = (w0 & kItemExt) ? w1 : (w1 & 0xFFFF);   // extended: full offset
        uint32_t lit_n = 0, ml = 0;
        if (act0 && !(w0p & kItemExt)) {
            if (w0 & kItemExt) {
                lit_n = w0n;
                ml = w1n;
            } else {
                lit_n = (w1 >> 16) & 0xFF;
                const uint32_t mc = w1 >> 24;
                ml = mc ? mc + 3 : 0;
            }
        }
        // batch = the lanes before the first whose output would pass OUTB;
        // an extended item keeps its second half
        const uint32_t len = lit_n + ml;
        const uint32_t inc = wave_incl_add(len);
        const uint64_t over = __ballot(act0 && inc > OUTB);
        uint32_t nb = over ? (uint32_t)__builtin_ctzll(over) : 64;
        if (nb == 64 && (lane_val(w0, 63) & kItemExt))
            nb = 63;
        else if (nb > 0 && nb < 64 && (lane_val(w0, (int)nb - 1) & kItemExt))
            nb++;
        if (b + nb > nit)
            nb = nit - b;
        const uint32_t flushed = 16 * fc > S.a0 ? 16 * fc - S.a0 : 0;   // frame bytes < this are in HBM
        if (nb == 0) {
            // lane 0 alone is too long to stage: flush, copy in HBM, reload
            const uint32_t l0 = lane_val(lit_n, 0), m0 = lane_val(ml, 0);
            const uint32_t s0 = lane_val(src, 0), o0 = lane_val(off, 0);
            const uint32_t end_c = (produced + S.a0 + 15) >> 4;
            for (uint32_t c = fc + lane; c < end_c; c += 64)
                flush_chunk(S, O, c);
            __builtin_amdgcn_s_waitcnt(0);
            if (l0)
                hbm_run(lsp, s0, O.o + produced, l0, lane);
            __builtin_amdgcn_s_waitcnt(0);
            if (m0) {
                const uint32_t mb = produced + l0;
                if (o0 >= m0)
                    hbm_run(O.sp, mb - o0, O.o + mb, m0, lane);
                else
                    hbm_match(O, mb, o0, m0, lane);
            }
            __builtin_amdgcn_s_waitcnt(0);
            produced += l0 + m0;
            fc = (produced + S.a0) >> 4;
            S.cb = fc - 1;
            if (lane < 2) {
                const uint32_t c = fc - 1 + lane;   // chunks fc-1, fc back from HBM
                const int64_t x0 = (int64_t)16 * c - S.a0;
                if ((fc > 0 || lane == 1) && x0 >= 0)
                    *lp<u32x4>(S.base + 16 * lane) =
                        load16u(O.sp.r, (uint32_t)((int64_t)O.sp.s0 + x0));
            }
            __builtin_amdgcn_s_waitcnt(0);
            const uint32_t used = lane_val(w0, 0) & kItemExt ? 2 : 1;
            b += used;
            const uint64_t a = __shfl_down(cur, used, 64);
            const uint64_t c2 = __shfl(nxt, (int)((lane + used) & 63), 64);
            cur = lane + used < 64 ? a : c2;
            continue;
        }
        if (lane >= nb) {
            lit_n = 0;
            ml = 0;
        }
        const uint32_t bstart = produced;
        const uint32_t op = produced + inc - len;
        const uint32_t mb = op + lit_n;
        const uint32_t me = mb + ml;
        const uint32_t msrc = mb - off;
        const bool overlap = ml != 0 && off < ml;
        const uint32_t need = overlap ? mb : msrc + ml;   // end of the bytes the copy reads
        const bool early = ml != 0 && !overlap && need <= bstart;
        produced += lane_val(inc, (int)nb - 1);
        ZSK_T(0)
        // round 0: literal runs + matches whose source precedes the batch
        if ((DIAG & 8) == 0 && (DIAG & kDiagM0))
            copy_entries3(S, lbase, lsp, llen, O, descs, flushed, lane, src, op, lit_n, msrc, mb, early ? ml : 0);
        else if ((DIAG & 8) == 0 && (DIAG & kDiagL0))
            copy_entries2(S, lbase, lsp, llen, O, descs, flushed, lane, src, op, lit_n, msrc, mb, early ? ml : 0);
        else if ((DIAG & 8) == 0 && (DIAG & kDiagE0))
            copy_entries(S, lbase, lsp, llen, O.o, descs, flushed, lane, src, op, lit_n, msrc, mb, early ? ml : 0);
        else if ((DIAG & 8) == 0 && (DIAG & 65536))
            copy_direct<DIAG>(S, lbase, lsp, O, descs, flushed, lane, src, op, lit_n, msrc, mb, early ? ml : 0);
        else if ((DIAG & 8) == 0 && (DIAG & 128) == 0)
            copy_desc4<DIAG>(S, lbase, lsp, llen, O.o, descs, flushed, lane, src, op, lit_n, msrc, mb,
                             early ? ml : 0);
        else if ((DIAG & 8) == 0)
            copy_desc3<DIAG>(S, lbase, lsp, llen, O.o, descs, flushed, lane, src, op, lit_n, msrc, mb,
                             early ? ml : 0);
        wave_lds_sync();   // stage bytes of other lanes from here on
        ZSK_T(1)
        // rounds: matches reading bytes of this batch
        uint64_t pending = (DIAG & 4) ? 0 : __ballot(ml != 0 && !early);
        if (DIAG & 16) {
            cnt[0] += 1;
            cnt[1] += __builtin_popcountll(pending);
            cnt[2] += __builtin_popcountll(__ballot(ml != 0 && !early && msrc < bstart));
            cnt[3] += __builtin_popcountll(__ballot(overlap));
            cnt[4] += nb;
        }
        while (pending) {
            const bool mine = (pending >> lane) & 1;
            // pending destinations are ascending and disjoint: compact them
            // (lane order) into the descriptor area, then binary-search the
            // first one below this lane that ends after msrc; blocked iff it
            // also starts before need
            bool ready;
            if (DIAG & 16384) {
                // every pending lane's destination broadcast in turn (no LDS
                // round trips): blocked iff a lower pending destination meets
                // this lane's source range
                bool blocked = false;
                for (uint64_t pm = pending; pm; pm &= pm - 1) {
                    const int j = (int)__builtin_ctzll(pm);
                    const uint32_t mbj = lane_val(mb, j), mej = lane_val(me, j);
                    blocked |= (uint32_t)j < lane && mej > msrc && mbj < need;
                }
                ready = mine && !blocked;
            } else {
            const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(pending >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pending, 0u));
            if (mine)
                *lp<uint64_t>(descs + 8 * below) = ((uint64_t)me << 32) | mb;
            wave_lds_sync();
            uint32_t lo = 0, hi = mine ? below : 0;
            while (!(DIAG & 1024) && __ballot(lo < hi)) {
                const uint32_t mid = (lo + hi) >> 1;
                const uint32_t mem = lo < hi ? (uint32_t)(*lp<uint64_t>(descs + 8 * mid) >> 32) : 0;
                if (lo < hi) {
                    if (mem > msrc)
                        hi = mid;
                    else
                        lo = mid + 1;
                }
            }
            const uint32_t mbl = (uint32_t)*lp<uint64_t>(descs + 8 * (mine && lo < below ? lo : 0));
            ready = mine && !(lo < below && mbl < need);
            wave_lds_sync();
            }
            if (!(DIAG & 512)) {
                for (uint64_t ov = __ballot(ready && overlap); ov; ov &= ov - 1) {
                    const int i = (int)__builtin_ctzll(ov);
                    copy_overlap_wave(S, O, flushed, lane_val(mb, i), lane_val(off, i), lane_val(ml, i), lane);
                }
            }
            if (DIAG & kDiagLR)
                copy_entries2(S, lbase, lsp, llen, O, descs, flushed, lane, 0, 0, 0, msrc, mb,
                              ready && !overlap ? ml : 0);
            else if (DIAG & kDiagER)
                copy_entries(S, lbase, lsp, llen, O.o, descs, flushed, lane, 0, 0, 0, msrc, mb,
                             ready && !overlap ? ml : 0);
            else if (!(DIAG & 256))
                copy_round(S, O, flushed, msrc, mb, ready && !overlap ? ml : 0);
            pending &= ~__ballot(ready);
            wave_lds_sync();
            if (DIAG & 16)
                cnt[5] += 1;
        }
        ZSK_T(2)
        // the next batch's items before the flush: the wait for nxt (issued
        // at the top of this batch) then does not also wait for the flush's
        // stores
        {
            const uint64_t a = __shfl_down(cur, nb & 63, 64);
            const uint64_t c2 = __shfl(nxt, (int)((lane + nb) & 63), 64);
            cur = nb == 64 ? nxt : (lane + nb < 64 ? a : c2);
        }
        // flush complete chunks (the frame's last chunk exactly)
        const bool last = b + nb >= nit || produced >= stop;
        const uint32_t end_c = last ? (produced + S.a0 + 15) >> 4 : (produced + S.a0) >> 4;
        if (!(DIAG & 34))
            flush_chunks4d<DIAG>(S, O, fc, end_c, lane);
        fc = end_c;
        // keep chunks fc-1 (flushed) and fc (partial) at stage index 0
        wave_lds_sync();
        if (!last && fc - 1 != S.cb) {
            u32x4 v;
            if (lane < 2)
                v = *lp<u32x4>(S.base + 16u * (fc - 1 + lane - S.cb));
            if (lane < 2)
                *lp<u32x4>(S.base + 16 * lane) = v;
            S.cb = fc - 1;
        }
        wave_lds_sync();
        b += nb;
        ZSK_T(3)
    }
#undef ZSK_T
    if ((DIAG & 16) && lane == 0)
        for (int i = 0; i < 4; i++)
            atomicAdd(&g_xstats[i], (unsigned long long)tsec[i]);
    if ((DIAG & 16) && lane == 0)
        for (int i = 0; i < 6; i++)
            atomicAdd(&g_xstats[4 + i], (unsigned long long)cnt[i]);
}

}   // namespace

// version (tuning builds, launch_seq_exec's argument): 0x1xx / 0x3xx DIAG
// variants, 0x6.W occupancy probes (LDS padding for W waves per SIMD), 0x7xx
// the round-6 experiments.  0: the production kernel (seq_exec.hip).
int launch_seq_exec_variant(int version, const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                            uint8_t *d_out, const uint64_t *rec_base, const uint64_t *items, const uint32_t *nitems,
                            const int32_t *d_status, hipStream_t stream, uint32_t stop_last, uint32_t min_dsize)
{
    const dim3 grid((nframes + kXW - 1) / kXW), block(64 * kXW);
#define ZSK_X(D)                                                                                               \
    hipLaunchKernelGGL((seq_exec_diag_kernel<D, kExecStage, false>), grid, block, 0, stream, d_desc, nframes, d_comp, \
                       d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr, nullptr, nullptr, stop_last, \
                       min_dsize)
    switch (version) {
    case 0x100: ZSK_X(0); break;   // the round-5 production kernel (copy_desc4, copy_round)
    case 0x101: ZSK_X(1); break;
    case 0x104: ZSK_X(4); break;
    case 0x108: ZSK_X(8); break;
    case 0x122: ZSK_X(34); break;
    case 0x140: ZSK_X(64); break;
    case 0x180: ZSK_X(128); break;
    case 0x141:   // the 4,096-byte stage: five waves per SIMD
        hipLaunchKernelGGL((seq_exec_diag_kernel<0, 4096, false>), grid, block, 0, stream, d_desc, nframes, d_comp,
                           d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr, nullptr, nullptr,
                           stop_last, min_dsize);
        break;
    case 0x142:   // the 3,584-byte stage, six waves per SIMD
        hipLaunchKernelGGL((seq_exec_diag_kernel<0, 3584, false>), grid, block, 0, stream, d_desc, nframes, d_comp,
                           d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr, nullptr, nullptr,
                           stop_last, min_dsize);
        break;
    case 0x143:   // a 2,560-byte stage, eight waves per SIMD (64 VGPRs: spills)
        hipLaunchKernelGGL((seq_exec_diag_kernel<0, 2560, false>), grid, block, 0, stream, d_desc, nframes, d_comp,
                           d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr, nullptr, nullptr,
                           stop_last, min_dsize);
        break;
    case 0x1C0: ZSK_X(192); break;
    case 0x301: ZSK_X(256); break;    // rounds without copy_round
    case 0x302: ZSK_X(512); break;    // rounds without copy_overlap
    case 0x304: ZSK_X(1024); break;   // rounds without the readiness search
    case 0x307: ZSK_X(1792); break;   // rounds: compaction and ballots only
    case 0x310: ZSK_X(4096); break;   // round 0: two descriptors per step
    case 0x320: ZSK_X(8192); break;   // round 0: the deal's descriptor reads together
    case 0x340: ZSK_X(16384); break;  // rounds: readiness by broadcast instead of the LDS search
    case 0x360: ZSK_X(24576); break;  // both
    case 0x380: ZSK_X(32768); break;  // round 0: long runs' descriptors by the whole wave (-0.8 % at 6 waves, +0.5 % at 7)
    case 0x400: ZSK_X(65536); break;  // round 0 direct (copy_direct)
    case 0x810: ZSK_X(kDiagNoLit); break;     // traffic split: no literal piece loads
    case 0x811: ZSK_X(kDiagNoMatch); break;   // traffic split: no HBM match piece loads
    case 0x700: ZSK_X(kDiagEntries); break;   // round 0 and rounds in 64-byte entries
    case 0x703: ZSK_X(kDiagE0); break;        // round 0 only
    case 0x704: ZSK_X(kDiagER); break;        // the rounds only
    case 0x710: ZSK_X(kDiagL0); break;        // round 0 through copy_entries2
    case 0x711: ZSK_X(kDiagL0 | kDiagLR); break;   // round 0 and the rounds through copy_entries2
    case 0x712: ZSK_X(kDiagLR); break;        // the rounds through copy_entries2
    case 0x720: ZSK_X(kDiagM0); break;        // round 0 through copy_entries3
    case 0x721: ZSK_X(kDiagM0 | kDiagLR); break;   // ... and the rounds through copy_entries2
    case 0x722:   // copy_entries3 at six waves per SIMD (80 VGPRs: no spill)
        hipLaunchKernelGGL((seq_exec_diag_kernel<kDiagM0, kExecStage, false, 6>), grid, block, 0, stream, d_desc, nframes,
                           d_comp, d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr, nullptr,
                           nullptr, stop_last, min_dsize);
        break;
    case 0x723:
        hipLaunchKernelGGL((seq_exec_diag_kernel<kDiagM0 | kDiagLR, kExecStage, false, 6>), grid, block, 0, stream, d_desc,
                           nframes, d_comp, d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr,
                           nullptr, nullptr, stop_last, min_dsize);
        break;
    case 0x724:   // copy_entries2 (round 0 and rounds) at six waves
        hipLaunchKernelGGL((seq_exec_diag_kernel<kDiagL0 | kDiagLR, kExecStage, false, 6>), grid, block, 0, stream, d_desc,
                           nframes, d_comp, d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr,
                           nullptr, nullptr, stop_last, min_dsize);
        break;
    case 0x730: ZSK_X(1 << 22); break;        // copy_desc4's descriptors by 32-bit adds
    case 0x731: ZSK_X((1 << 22) | kDiagLR); break;   // ... and the rounds through copy_entries2
    case 0x732: ZSK_X((1 << 22) | kDiagLR | 8192); break;   // ... and the deal's descriptor reads together
    case 0x701:   // ... at six waves per SIMD (80 VGPRs)
        hipLaunchKernelGGL((seq_exec_diag_kernel<kDiagEntries, kExecStage, false, 6>), grid, block, 0, stream, d_desc,
                           nframes, d_comp, d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr,
                           nullptr, nullptr, stop_last, min_dsize);
        break;
    case 0x702:   // the production kernel at six waves per SIMD (80 VGPRs)
        hipLaunchKernelGGL((seq_exec_diag_kernel<0, kExecStage, false, 6>), grid, block, 0, stream, d_desc, nframes,
                           d_comp, d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr, nullptr,
                           nullptr, stop_last, min_dsize);
        break;
    case 0x602: case 0x603: case 0x604: case 0x605: case 0x606: {
        // occupancy probe: dynamic LDS padding so that only W = version & 0xF
        // four-wave workgroups fit a CU's 160 KiB (W waves per SIMD)
        const uint32_t W = version & 0xF, st = kXW * x_wave(kExecStage);
        const uint32_t pad = (163840 + W) / (W + 1) + 1 - st;
        hipLaunchKernelGGL((seq_exec_diag_kernel<0, kExecStage, false>), grid, block, pad, stream, d_desc, nframes,
                           d_comp, d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr, nullptr,
                           nullptr, stop_last, min_dsize);
        break;
    }
    case 0x110: {
        unsigned long long z[12] = {0};
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_xstats), z, sizeof(z), 0, hipMemcpyHostToDevice, stream);
        ZSK_X(16);
        (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_xstats), sizeof(z), 0, hipMemcpyDeviceToHost, stream);
        (void)hipStreamSynchronize(stream);
        const double t = (double)(z[0] + z[1] + z[2] + z[3]);
        fprintf(stderr, "exec sections (wave cycles): items+scan %.1f%%  round0 %.1f%%  rounds %.1f%%  flush %.1f%%  total %.3g\n",
                100 * z[0] / t, 100 * z[1] / t, 100 * z[2] / t, 100 * z[3] / t, t);
        const double nb = (double)z[4];
        fprintf(stderr, "per batch: seqs %.1f pending %.2f (src below batch %.2f) overlap %.3f rounds %.2f\n",
                z[8] / nb, z[5] / nb, z[6] / nb, z[7] / nb, z[9] / nb);
        break;
    }
    default: return -1;
    }
#undef ZSK_X
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk
