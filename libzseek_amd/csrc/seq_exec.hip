// seq_exec.hip — sequence execution for the two-phase decoders (gfx950).
//
// Input: per-sequence items (the LZ4 parse kernels lz4_lean / lz4_scan /
// lz4_chunk, or zstd_seq_kernel) = a literal run (source offset + length)
// followed by a match (offset, length).  One wave executes one frame, 64
// sequences (one per lane) per batch; the batch's output is assembled in a
// small per-wave *linear* LDS stage and leaves it as aligned 16-byte chunks,
// consecutive lanes -> consecutive chunks, so HBM sees only full coalesced
// writes of exactly the output bytes.  Per batch:
//   * item decode and the output prefix sum on DPP (row_shr / row_bcast /
//     wave_shl), no ds_bpermute chains;
//   * round 0: literal runs and matches whose source precedes the batch — one
//     8-byte descriptor per 16-byte piece from one base per run, the wave's
//     pieces dealt one per lane per slot, four slots' loads in flight;
//   * dependency rounds: a match whose source meets a lower pending match's
//     destination waits; readiness by binary search over the pending
//     destinations compacted in LDS (1.7 rounds per batch on the synthetic);
//   * flush: four chunks' stage reads in flight before their stores; the next
//     batch's items are shifted in before it.
//
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "lz4_dev.h"
#ifndef ZSK_EXEC_SEG_TU
#include "lz4_wave_dev.h"   // the one-frame execute decodes its batch's hand-offs
#endif
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4d;

constexpr uint32_t kItemExt = 0x80000000u;
constexpr uint32_t kItemPos = 0x3FFFFFFFu;
constexpr uint32_t kXW = 4;                 // waves (frames) per workgroup
// per wave, for OUTB output bytes staged per batch at most: the stage (2 kept
// chunks + read slack) and the piece descriptors (one per 16-byte piece, 8 B)
constexpr uint32_t x_buf(uint32_t outb) { return outb + 80; }
constexpr uint32_t x_pieces(uint32_t outb) { return outb / 16 + 2 * 64; }
constexpr uint32_t x_wave(uint32_t outb) { return x_buf(outb) + 8 * x_pieces(outb); }
constexpr uint32_t kBad = 0x80000000u;      // buffer offset past any range: load returns 0

typedef u32x4 u32x4_l __attribute__((aligned(1)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint64_t u64_l __attribute__((aligned(1)));
typedef uint32_t u32_l __attribute__((aligned(1)));
typedef uint16_t u16_l __attribute__((aligned(1)));

template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T *lp(uint32_t a)
{
    return (__attribute__((address_space(3))) T *)(uintptr_t)a;
}

struct Stage {
    uint32_t base;   // LDS address of stage index 0
    uint32_t a0;     // output address & 15
    uint32_t cb;     // output chunk at stage index 0 (int32 -1 at frame start)
};

// LDS address of frame output byte x
__device__ __forceinline__ uint32_t saddr(const Stage &S, uint32_t x)
{
    return S.base + x + S.a0 - 16u * S.cb;
}

__device__ __forceinline__ u32x4 lds16(uint32_t a)
{
    return *lp<u32x4_l>(a);
}

// the first n (1..16) bytes of v at LDS address a, nothing beyond
__device__ __forceinline__ void lds_put(uint32_t a, u32x4 v, uint32_t n)
{
    if (n >= 16) {
        *lp<u32x4_l>(a) = v;
        return;
    }
    if (n & 8) {
        *lp<u64_l>(a) = ((uint64_t)v.y << 32) | v.x;
        a += 8;
        v.x = v.z;
        v.y = v.w;
    }
    if (n & 4) {
        *lp<u32_l>(a) = v.x;
        a += 4;
        v.x = v.y;
    }
    if (n & 2) {
        *lp<u16_l>(a) = (uint16_t)v.x;
        a += 2;
        v.x >>= 16;
    }
    if (n & 1)
        *lp<uint8_t>(a) = (uint8_t)v.x;
}

// A run of n bytes is covered by ceil(n/16) pieces: piece i is
// [min(16 i, n - 16), +16) when n >= 16 (overlapping pieces rewrite equal
// bytes), else the single piece [0, n).
__device__ __forceinline__ uint32_t npieces(uint32_t n)
{
    return (n + 15) >> 4;
}

__device__ __forceinline__ uint32_t piece_off(uint32_t n, uint32_t i)
{
    return n < 16 ? 0 : (16 * i < n - 16 ? 16 * i : n - 16);
}

struct Out {
    uint8_t *o;      // frame output byte 0
    uint32_t dlen;
    Span sp;         // range-checked reads of the frame output
};

// 16 output bytes at frame offset s for a match piece: HBM below `flushed`
// (issued as a disabled load otherwise), else the stage
__device__ __forceinline__ u32x4 src16(const Stage &S, const Out &O, uint32_t flushed, uint32_t s,
                                       bool on)
{
    const bool h = s + 16 <= flushed;
    const u32x4 vh = load16u(O.sp.r, on && h ? O.sp.s0 + s : kBad);
    const u32x4 vl = lds16(on && !h ? saddr(S, s) : S.base);
    return h ? vh : vl;
}

// 16 bytes at byte offset x of a resource: one unaligned load.  Safe for the
// LZ4 sources because the hardware range-checks per dword and every byte a
// piece needs lies at least 4 bytes before its span's end (literal runs are
// followed by a block header / end mark; a match source ends before its
// destination, which ends at most at the frame end).
__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t x)
{
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, x, 0, 0));
}

enum : uint32_t { K_LIT = 0, K_HBM = 1, K_STAGE = 2 };

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
            v[j] = (DIAG & 1) ? (u32x4){0, 0, 0, 0} : *reinterpret_cast<const u32x4_l *>(p);
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

// Overlapping match (off < n) over the whole wave (uniform arguments; round
// 3's copy_overlap ran it on its own lane: 26 % of the execute's VALU at
// config 2 for 0.18 such matches per batch): out[mb + j] = out[mb + j - off]
// in phases of e bytes, phase p copying [p e, (p + 1) e) from the e bytes
// before it in 16-byte pieces, one per lane.  e = off when off >= 16 (the
// first phase reads the final bytes before mb); for off < 16, phase 0 writes
// the first e = off * ceil(16 / off) (16..30) bytes one byte per lane from
// the pattern out[mb - off, mb), which lies in the stage (mb - off > bstart -
// 16 >= flushed - 16, the stage's kept chunk).
__device__ __forceinline__ void copy_overlap_wave(const Stage &S, const Out &O, uint32_t flushed,
                                                  uint32_t mb, uint32_t off, uint32_t n, uint32_t lane)
{
    uint32_t e = off, done = 0;
    if (off < 16) {
        e = off * ((16 + off - 1) / off);
        done = e < n ? e : n;
        if (lane < done) {
            const uint32_t q = (lane * ((1024 + off - 1) / off)) >> 10;   // lane / off (lane < 32, off < 16)
            *lp<uint8_t>(saddr(S, mb + lane)) = *lp<uint8_t>(saddr(S, mb - off + (lane - q * off)));
        }
        wave_lds_sync();
    }
    while (done < n) {
        const uint32_t len = n - done < e ? n - done : e;
        const uint32_t np = npieces(len);
        for (uint32_t k0 = 0; k0 < np; k0 += 64) {
            const bool on = k0 + lane < np;
            const uint32_t o = piece_off(len, k0 + lane);
            const u32x4 v = src16(S, O, flushed, mb + done - e + o, on);
            if (on)
                lds_put(saddr(S, mb + done + o), v, len < 16 ? len : 16);
        }
        done += len;
        wave_lds_sync();
    }
}

// stage chunk k (output chunk cb + k) -> HBM; exact at the frame's edges
__device__ __forceinline__ void put_chunk(const Out &O, uint32_t a0, uint32_t c, const u32x4 &v)
{
    const int64_t x0 = (int64_t)16 * c - a0;
    if (x0 >= 0 && x0 + 16 <= O.dlen) {
        *reinterpret_cast<u32x4 *>(O.o + x0) = v;
    } else {
        for (int k = 0; k < 16; k++) {
            const int64_t x = x0 + k;
            if (x >= 0 && x < O.dlen)
                O.o[x] = (uint8_t)vbyte(v, k);
        }
    }
}

// chunks [fc, end_c) -> HBM, lane-strided, four chunks' LDS reads in flight
// before their stores
template <int DIAG>
__device__ __forceinline__ void flush_chunks4(const Stage &S, const Out &O, uint32_t fc, uint32_t end_c,
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

__device__ __forceinline__ void flush_chunk(const Stage &S, const Out &O, uint32_t c)
{
    const u32x4 v = *lp<u32x4>(S.base + 16u * (c - S.cb));
    const int64_t x0 = (int64_t)16 * c - S.a0;
    if (x0 >= 0 && x0 + 16 <= O.dlen) {
        *reinterpret_cast<u32x4 *>(O.o + x0) = v;
    } else {
        for (int k = 0; k < 16; k++) {
            const int64_t x = x0 + k;
            if (x >= 0 && x < O.dlen)
                O.o[x] = (uint8_t)vbyte(v, k);
        }
    }
}

// whole-wave copy in HBM for sequences too long to stage (source and
// destination do not overlap within one 1 KiB step)
__device__ __forceinline__ void hbm_run(const Span &s, uint32_t src, uint8_t *dst, uint32_t n,
                                        uint32_t lane)
{
    for (uint32_t k = 16 * lane; k < n; k += 1024) {
        const u32x4 v = load16u(s.r, s.s0 + src + k);
        store_exact(dst + k, v, n - k < 16 ? n - k : 16);
    }
}

__device__ __forceinline__ void hbm_match(const Out &O, uint32_t dst, uint32_t off, uint32_t n,
                                          uint32_t lane)
{
    uint32_t done = 0;
    while (done < n) {
        __builtin_amdgcn_s_waitcnt(0);
        const uint32_t e = off * ((done + off) / off);   // a multiple of off, <= done + off
        uint32_t step = e < 1024 ? e : 1024;
        if (step > n - done)
            step = n - done;
        if (e < 16) {
            if (lane == 0)
                for (uint32_t k = 0; k < step; k++)
                    O.o[dst + done + k] = O.o[dst + done + k - e];
        } else {
            for (uint32_t k = 16 * lane; k < step; k += 1024) {
                const uint32_t x = dst + done + k;
                const u32x4 v = load16u(O.sp.r, O.sp.s0 + x - e);
                const uint32_t r = step - k;
                store_exact(O.o + x, v, r < 16 ? r : 16);
            }
        }
        done += step;
    }
    __builtin_amdgcn_s_waitcnt(0);
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
// Item addressing of the execute: contiguous items (JobMap<false>), or the
// block route's job segments (JobMap<true>, below).
template <bool SEG>
struct JobMap {
    __device__ __forceinline__ uint32_t init(const uint32_t *, const uint32_t *, const BlockJob *,
                                             const BlockRes *, uint32_t, const uint32_t *, uint32_t, uint32_t,
                                             uint32_t &)
    {
        return 0;
    }
    __device__ __forceinline__ uint32_t addr(uint32_t i0, uint32_t lane, uint32_t) const
    {
        return 8 * (i0 + lane);
    }
};

template <>
struct JobMap<true> {
    uint32_t jtab = 0;   // LDS: entry j = {job j's first item index, its slot offset - that index}
    uint32_t nseg = 0;   // jobs (0: contiguous items)
    // cursor: the job of the window's first index, the next job's first
    // index, both offsets (uniform)
    uint32_t cs = 0, s_next = 0xFFFFFFFFu, d_cur = 0, d_next = 0;

    // the table from frame f's jobs; returns the frame's item count (their
    // total), span = the item slots its resource must cover
    __device__ __forceinline__ uint32_t init(const uint32_t *bfirst, const uint32_t *bcount, const BlockJob *jobs,
                                             const BlockRes *jres, uint32_t f, const uint32_t *nitems,
                                             uint32_t tab, uint32_t lane, uint32_t &span)
    {
        const uint32_t j0 = uni(bfirst[f]);
        if (j0 == kNoJob) {
            span = uni(nitems[f]);
            return span;
        }
        jtab = tab;
        nseg = uni(bcount[f]);
        uint32_t so = 0, nj = 0;
        if (lane < nseg) {
            so = jobs[j0 + lane].slot_off;
            nj = jres[j0 + lane].n;
        }
        const uint32_t inc = wave_incl_add(nj);
        if (lane < nseg)
            *lp<uint64_t>(jtab + 8 * lane) = ((uint64_t)(so - (inc - nj)) << 32) | (inc - nj);
        if (lane == 0)   // the end entry (index 64 for 64 jobs: no lane of its own)
            *lp<uint64_t>(jtab + 8 * nseg) = 0xFFFFFFFFull;
        span = uni(lane_val(so + nj, (int)nseg - 1));
        wave_lds_sync();
        const uint64_t e0 = *lp<uint64_t>(jtab), e1 = *lp<uint64_t>(jtab + 8);
        d_cur = uni((uint32_t)(e0 >> 32));
        s_next = uni((uint32_t)e1);
        d_next = uni((uint32_t)(e1 >> 32));
        return uni(lane_val(inc, 63));
    }

    // byte offset of item index i = i0 + lane (past nit: out of range); i0
    // never decreases
    __device__ __forceinline__ uint32_t addr(uint32_t i0, uint32_t lane, uint32_t nit)
    {
        const uint32_t i = i0 + lane;
        if (nseg == 0)
            return 8 * i;
        while (s_next <= i0) {   // the window starts in a later job
            cs++;
            d_cur = d_next;
            const uint64_t e = *lp<uint64_t>(jtab + 8 * (cs + 1));
            s_next = uni((uint32_t)e);
            d_next = uni((uint32_t)(e >> 32));
        }
        uint32_t d = d_cur;
        for (uint32_t k = cs + 1, sk = s_next, dk = d_next; sk <= i0 + 63;) {   // jobs starting inside it
            d = i >= sk ? dk : d;
            const uint64_t e = *lp<uint64_t>(jtab + 8 * (++k));
            sk = uni((uint32_t)e);
            dk = uni((uint32_t)(e >> 32));
        }
        return i < nit ? 8 * (i + d) : 0x7FFFFFF0u;
    }
};

// SEG (the LZ4 block route): a frame with a job list (bfirst[f] != kNoJob)
// has its items job by job -- job j's jres[j].n items at rec_base[f] +
// jobs[j].slot_off -- read in block order as one sequence: lane j holds job
// j's first item index in that sequence and its slot offset (a 512-byte LDS
// table per wave), and each lane maps the item index it loads onto its job's
// slots with a uniform job cursor, so batches run across jobs unchanged.
// (SEG runs at 4 waves per SIMD: its batches have <= 32,767 frames -- config
// 3's 4,096 fill 4 per SIMD -- and the job cursor's registers fit no spill)
// The LZ4 route's stage: 3,072 bytes -> 22.8 KB of LDS per 4-wave group,
// seven waves per SIMD (72 VGPRs); a batch of config 2 averages 2.7 KB, so
// the smaller stage cuts few, and the extra waves hide latency (config 2,
// execute alone, interleaved: 4,096 bytes / 5 waves 2.554 ms, 3,584 / 6
// 2.438, 3,072 / 7 2.411; 2,560 / 8 needs 64 VGPRs and spills: 2.897).
constexpr uint32_t kExecStage = 3072;

template <int DIAG, uint32_t OUTB, bool SEG>
__global__ __launch_bounds__(64 * kXW) __attribute__((amdgpu_waves_per_eu(SEG ? 4 : (OUTB <= 2560 ? 8 : OUTB <= 3072 ? 7 : OUTB <= 3584 ? 6 : 5)))) void seq_exec_kernel(
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
        if ((DIAG & 8) == 0 && (DIAG & 65536))
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
            if (!(DIAG & 256))
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
            flush_chunks4<DIAG>(S, O, fc, end_c, lane);
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

#ifndef ZSK_EXEC_SEG_TU
// ---- the one-frame route's execute: one frame per 1,024-thread workgroup ----
// A lone wave executes a 64 KiB frame in ~24 dependent batches (~67 us at a
// 4 KiB cache-0 read).  Here the frame's whole output is staged in LDS and
// every thread takes two sequences of a window of 2,048: an exclusive scan
// over the workgroup places them, literal runs are copied at once, and the
// matches resolve in passes -- a match copies once every byte it reads is
// marked done (a bit per output byte, set after the bytes are written, with
// release / acquire at workgroup scope); each wave passes over its pending
// matches on its own (a workgroup barrier per pass: 41 us per frame).  The
// earliest pending match always reads only done bytes, so the frame drains;
// the synthetic's match-dependency depth is ~18 per frame (28 at most).
// Frames of more than 64 KiB decoded go to seq_exec_kernel (min_dsize).
constexpr uint32_t kFT = 1024;
constexpr uint32_t kFMax = 65536;
// compressed bytes staged in LDS (literal source): a 64 KiB frame stored raw
// (65,551 bytes with its headers, more with checksums) still fits
constexpr uint32_t kFCStage = 65536 + 256;
constexpr uint32_t kFLong = 128;       // literal runs longer than this: copied by the whole wave

#ifdef ZSK_TUNING
// tuning builds: the one-frame execute's phase cycles (thread 0, at the
// workgroup barriers): [0] staging + init, [1] items + scans, [2] literal
// runs, [3] match passes, [4] output; [5] windows, [6] sum over waves of
// their pass counts, [7] frames; printed under ZSEEK_FRAME_TIMERS
__device__ unsigned long long g_ftime[8];
__device__ uint32_t g_fdiag;   // ZSEEK_FRAME_DIAG: 1 no literal copies, 2 no literal marks, 4 no matches
#define ZSK_FD(b) ((__builtin_amdgcn_readfirstlane(g_fdiag) & (b)) != 0)
#define ZSK_FT(i)                                                             \
    {                                                                         \
        const uint64_t tn_ = __builtin_readcyclecounter();                    \
        if (t == 0)                                                           \
            atomicAdd(&g_ftime[i], (unsigned long long)(tn_ - tmark_));       \
        tmark_ = tn_;                                                         \
    }
#else
#define ZSK_FD(b) false
#define ZSK_FT(i)
#endif

__global__ __launch_bounds__(kFT) void seq_exec_frame_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ rec_base, const uint64_t *__restrict__ items, const uint32_t *__restrict__ nitems,
    int32_t *__restrict__ status, uint32_t *__restrict__ fail_at, uint32_t stop_last, uint32_t handoff,
    const uint8_t *__restrict__ lit)
{
    __shared__ __attribute__((aligned(16))) uint8_t ob[kFMax + 80];
    __shared__ __attribute__((aligned(16))) uint8_t cs[kFCStage + 80];
    __shared__ uint32_t done[kFMax / 32 + 2];
    __shared__ uint32_t wsum[kFT / 64];
    __shared__ uint32_t hi_end;
    const uint32_t f = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (f >= n)
        return;
    const FrameDesc d = desc[f];
    if (d.d_size > kFMax)
        return;   // seq_exec_kernel's frame (its hand-off: the wave kernel)
    if (__builtin_amdgcn_readfirstlane(status[f]) == ST_NOT_RUN) {
        // the hand-off (handoff != 0): the wave decoder of lz4_wave_kernel on
        // wave 0, its ring in the stage -- the batch then launches no
        // hand-off kernel (5 us + a launch gap per one-frame miss)
        if (handoff && wv == 0)
            lz4w::wave_frame<4096>(desc, f, comp, out, status, fail_at, ob);
        return;
    }
    const uint32_t nit = nitems[f];
    const uint32_t stop = f + 1 == n ? min(stop_last, d.d_size) : d.d_size;
    const uint64_t *it = items + rec_base[f];
    // literal source: the compressed frame (LZ4), or the frame's decoded
    // literals (zstd scratch laid out like the output, 16 bytes of slack)
    const uint32_t llen = lit ? d.d_size + 16 : d.c_size;
    const Span lsp = make_span(lit ? lit + d.d_off : comp + d.c_off, llen);
    const uint32_t ob0 = (uint32_t)(uintptr_t)ob, cs0 = (uint32_t)(uintptr_t)cs;
#ifdef ZSK_TUNING
    uint64_t tmark_ = __builtin_readcyclecounter();
    if (t == 0)
        atomicAdd(&g_ftime[7], 1ull);
#endif
    // the literal source into LDS (its 16-byte loads per thread issued
    // together), so a literal run is copied LDS to LDS instead of waiting on an
    // L2 / HBM load per 16 bytes; a source too big for the stage reads HBM
    const bool staged = llen <= kFCStage;
    if (staged) {
        const uint32_t np = (llen + 15) / 16;
        constexpr uint32_t kQ = (kFCStage / 16 + kFT - 1) / kFT;
        u32x4 v[kQ];
#pragma unroll
        for (uint32_t q = 0; q < kQ; q++) {
            const uint32_t i = t + q * kFT;
            v[q] = load16u(lsp.r, i < np ? lsp.s0 + 16 * i : kBad);
        }
#pragma unroll
        for (uint32_t q = 0; q < kQ; q++) {
            const uint32_t i = t + q * kFT;
            if (i < np)
                *lp<u32x4>(cs0 + 16 * i) = v[q];
        }
    }
    for (uint32_t i = t; i < kFMax / 32 + 2; i += kFT)
        done[i] = 0;
    if (t == 0)
        hi_end = 0;
    __syncthreads();
    ZSK_FT(0)

    auto scan = [&](uint32_t v, uint32_t &total) -> uint32_t {   // exclusive, in thread order
        const uint32_t inc = wave_incl_add(v);
        if (lane == 63)
            wsum[wv] = inc;
        __syncthreads();
        uint32_t before = 0, tot = 0;
        for (uint32_t k = 0; k < kFT / 64; k++) {
            const uint32_t x = wsum[k];
            before += k < wv ? x : 0;
            tot += x;
        }
        __syncthreads();
        total = tot;
        return before + inc - v;
    };
    // one release fence, then relaxed bit sets; readiness: relaxed reads of
    // every word (no early exit, so they are in flight together), one acquire
    // fence once all are set
    auto mark = [&](uint32_t a, uint32_t len) {   // output bytes [a, a + len) written
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        for (const uint32_t e = a + len; a < e;) {
            const uint32_t b0 = a & 31, nb = min(32 - b0, e - a);
            __hip_atomic_fetch_or(&done[a >> 5], nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1) << b0, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
            a += nb;
        }
    };
    auto ready = [&](uint32_t a, uint32_t len) -> bool {
        bool all = true;
        for (const uint32_t e = a + len; a < e;) {
            const uint32_t b0 = a & 31, nb = min(32 - b0, e - a);
            const uint32_t m = nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1) << b0;
            all &= (__hip_atomic_load(&done[a >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & m) == m;
            a += nb;
        }
        if (all)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        return all;
    };
    // 1..64 bytes between disjoint LDS ranges with whole-width writes only:
    // 16-byte pieces from the start plus one ending at n (overlapping pieces
    // rewrite equal bytes), two 8- or 4-byte ones below 16 bytes -- no
    // per-piece partial-store branches (reads may run past the source: the
    // arrays have slack)
    auto scopy = [&](uint32_t dst, uint32_t src, uint32_t n) {
        if (n >= 16) {
            const u32x4 a = lds16(src), b = lds16(src + 16), c = lds16(src + 32), e = lds16(src + n - 16);
            *lp<u32x4_l>(dst) = a;
            if (n > 32)
                *lp<u32x4_l>(dst + 16) = b;
            if (n > 48)
                *lp<u32x4_l>(dst + 32) = c;
            *lp<u32x4_l>(dst + n - 16) = e;
        } else if (n >= 8) {
            const uint64_t a = *lp<u64_l>(src), e = *lp<u64_l>(src + n - 8);
            *lp<u64_l>(dst) = a;
            *lp<u64_l>(dst + n - 8) = e;
        } else if (n >= 4) {
            const uint32_t a = *lp<u32_l>(src), e = *lp<u32_l>(src + n - 4);
            *lp<u32_l>(dst) = a;
            *lp<u32_l>(dst + n - 4) = e;
        } else {
            for (uint32_t k = 0; k < n; k++)
                *lp<uint8_t>(dst + k) = *lp<uint8_t>(src + k);
        }
    };
    // n bytes from LDS src to LDS dst, dst - src >= step or the ranges apart:
    // up to four 16-byte pieces read before they are written (a piece's
    // source was written at least `step` bytes earlier)
    auto lcopy = [&](uint32_t dst, uint32_t src, uint32_t n, uint32_t step) {
        for (uint32_t k = 0; k < n; k += step) {
            u32x4 v[4];
#pragma unroll
            for (uint32_t q = 0; q < 4; q++)
                if (16 * q < step)
                    v[q] = lds16(src + k + 16 * q);
#pragma unroll
            for (uint32_t q = 0; q < 4; q++)
                if (16 * q < step && k + 16 * q < n)
                    lds_put(dst + k + 16 * q, v[q], min(16u, n - k - 16 * q));
            wave_lds_sync();
        }
    };

    uint32_t base_op = 0;
    for (uint32_t w0 = 0; w0 < nit && base_op < stop; w0 += 2 * kFT) {
        uint32_t lit[2], ml[2], off[2], src[2], op[2], tot[2];
        for (int j = 0; j < 2; j++) {
            const uint32_t i = w0 + j * kFT + t;
            lit[j] = ml[j] = off[j] = src[j] = 0;
            if (i < nit) {
                const uint64_t cur = it[i];
                const uint32_t c0 = (uint32_t)cur, c1 = (uint32_t)(cur >> 32);
                const bool second = i > 0 && ((uint32_t)it[i - 1] & kItemExt);   // an extended item's second half
                if (!second) {
                    src[j] = c0 & kItemPos;
                    if (c0 & kItemExt) {
                        const uint64_t nx = it[i + 1];
                        lit[j] = (uint32_t)nx;
                        ml[j] = (uint32_t)(nx >> 32);
                        off[j] = c1;
                    } else {
                        lit[j] = (c1 >> 16) & 0xFF;
                        const uint32_t mc = c1 >> 24;
                        ml[j] = mc ? mc + 3 : 0;
                        off[j] = c1 & 0xFFFF;
                    }
                }
            }
        }
        const uint32_t x0 = scan(lit[0] + ml[0], tot[0]);
        const uint32_t x1 = scan(lit[1] + ml[1], tot[1]);
        ZSK_FT(1)
        op[0] = base_op + x0;
        op[1] = base_op + tot[0] + x1;
        bool pend[2];
        for (int j = 0; j < 2; j++) {
            const bool on = op[j] < stop && lit[j] + ml[j] != 0;
            const uint32_t L = on ? lit[j] : 0;
            // a run longer than kFLong is copied and marked by the whole wave,
            // 1 KiB per step: one lane's serial copy of a ~1 KiB run was the
            // literal phase's critical path (and of a stored 64 KiB block, too
            // big for the stage, 4,096 dependent 16-byte loads)
            const bool coop = L > kFLong;
            if (!ZSK_FD(1)) {
                for (uint64_t lm = __ballot(coop); lm; lm &= lm - 1) {
                    const int q = (int)__builtin_ctzll(lm);
                    const uint32_t d0 = ob0 + lane_val(op[j], q), s = lane_val(src[j], q), n = lane_val(L, q);
                    if (staged)
                        for (uint32_t k = 16 * lane; k < n; k += 1024)
                            lds_put(d0 + k, lds16(cs0 + s + k), min(16u, n - k));
                    else
                        for (uint32_t k = 16 * lane; k < n; k += 1024)
                            lds_put(d0 + k, load16u(lsp.r, lsp.s0 + s + k), min(16u, n - k));
                }
            }
            if (!coop && L && !ZSK_FD(1)) {
                if (staged && L <= 2 * 64) {   // (coop takes longer runs)
                    scopy(ob0 + op[j], cs0 + src[j], min(L, 64u));
                    if (L > 64)
                        scopy(ob0 + op[j] + 64, cs0 + src[j] + 64, L - 64);
                } else if (staged)
                    lcopy(ob0 + op[j], cs0 + src[j], L, 64);
                else
                    for (uint32_t k = 0; k < L; k += 16)
                        lds_put(ob0 + op[j] + k, load16u(lsp.r, lsp.s0 + src[j] + k), min(16u, L - k));
            }
            if (!ZSK_FD(2)) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                for (uint64_t lm = __ballot(coop); lm; lm &= lm - 1) {
                    const int q = (int)__builtin_ctzll(lm);
                    const uint32_t a = lane_val(op[j], q), e = a + lane_val(L, q) - 1;
                    for (uint32_t g = (a >> 5) + lane; g <= e >> 5; g += 64) {
                        const uint32_t lo = g == a >> 5 ? a & 31 : 0, hi = g == e >> 5 ? e & 31 : 31;
                        const uint32_t m = hi - lo == 31 ? 0xFFFFFFFFu : ((1u << (hi - lo + 1)) - 1) << lo;
                        __hip_atomic_fetch_or(&done[g], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                if (!coop && L)
                    mark(op[j], L);
            }
            pend[j] = on && ml[j] != 0 && !ZSK_FD(4);
        }
        {
            // the decoded end: a wave max, one LDS atomic per wave (2,048
            // atomics on one word cost ~20K cycles per frame)
            const bool on0 = op[0] < stop && lit[0] + ml[0] != 0, on1 = op[1] < stop && lit[1] + ml[1] != 0;
            const uint32_t e = max(on0 ? op[0] + lit[0] + ml[0] : 0u, on1 ? op[1] + lit[1] + ml[1] : 0u);
            const uint32_t we = wave_incl_max(e);
            if (lane == 63 && we)
                atomicMax(&hi_end, we);
        }
        __syncthreads();
        ZSK_FT(2)
        // each wave loops on its own until its matches are copied (no
        // workgroup barrier per round: a wave whose sources are ready runs
        // ahead; one that made no progress sleeps a little)
        for (uint32_t pass = 0;; pass++) {
            bool moved = false;
            for (int j = 0; j < 2; j++) {
                if (!pend[j])
                    continue;
                const uint32_t mb = op[j] + lit[j], o = off[j], m = ml[j];
                if (!ready(mb - o, o >= m ? m : o))
                    continue;
                if (o >= m && m <= 128) {
                    scopy(ob0 + mb, ob0 + mb - o, min(m, 64u));
                    if (m > 64)
                        scopy(ob0 + mb + 64, ob0 + mb - o + 64, m - 64);
                } else if (o >= m || o >= 16) {   // apart, or trailing by >= 16: pieces ahead of their sources
                    lcopy(ob0 + mb, ob0 + mb - o, m, o >= m ? 64u : min(64u, o & ~15u));
                } else {
                    // overlapping: the first e = o * ceil(16 / o) bytes one at a
                    // time, then 16-byte pieces trailing by e (each reads bytes
                    // an earlier step of this thread wrote)
                    const uint32_t e = o >= 16 ? o : o * ((16 + o - 1) / o);
                    const uint32_t h = o >= 16 ? 0 : min(e, m);
                    for (uint32_t k = 0; k < h; k++) {
                        ob[mb + k] = ob[mb - o + k];
                        wave_lds_sync();
                    }
                    for (uint32_t k = h; k < m; k += 16) {
                        lds_put(ob0 + mb + k, lds16(ob0 + mb + k - e), min(16u, m - k));
                        wave_lds_sync();
                    }
                }
                mark(mb, m);
                pend[j] = false;
                moved = true;
            }
            // (validated items always drain; the bound only guards the GPU
            // against a malformed list)
            if (!__any(pend[0] || pend[1]) || pass > (1u << 22)) {
#ifdef ZSK_TUNING
                if (lane == 0)
                    atomicAdd(&g_ftime[6], (unsigned long long)(pass + 1));
#endif
                break;
            }
            if (!__any(moved))
                __builtin_amdgcn_s_sleep(1);
        }
        __syncthreads();
        ZSK_FT(3)
#ifdef ZSK_TUNING
        if (t == 0)
            atomicAdd(&g_ftime[5], 1ull);
#endif
        base_op += tot[0] + tot[1];
    }
    __syncthreads();
    // the decoded bytes [0, hi_end) out: a byte head to 16-byte alignment,
    // whole 16-byte stores, a byte tail
    const uint32_t E = min(hi_end, d.d_size);
    uint8_t *o = out + d.d_off;
    const uint32_t head = min(E, (uint32_t)((16 - ((uintptr_t)o & 15)) & 15));
    if (t < head)
        o[t] = ob[t];
    const uint32_t nchunks = (E - head) / 16;
    for (uint32_t c = t; c < nchunks; c += kFT)
        *reinterpret_cast<u32x4 *>(o + head + 16 * c) = lds16(ob0 + head + 16 * c);
    const uint32_t tail0 = head + 16 * nchunks;
    if (tail0 + t < E)
        o[tail0 + t] = ob[tail0 + t];
#ifdef ZSK_TUNING
    __syncthreads();
    ZSK_FT(4)
#endif
}
#undef ZSK_FT
#endif

}   // namespace

#ifdef ZSK_EXEC_SEG_TU
// seq_exec_seg.hip: the block route's instantiation, compiled on its own (in
// one module with the production kernel it cost that kernel a VGPR spill)
int launch_seq_exec_seg(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
                        const uint64_t *rec_base, const uint64_t *items, const uint32_t *nitems,
                        const int32_t *d_status, hipStream_t stream, const SplitScratch *blk)
{
    if (nframes == 0)
        return 0;
    hipLaunchKernelGGL((seq_exec_kernel<0, 4096, true>), dim3((nframes + kXW - 1) / kXW), dim3(64 * kXW), 0, stream,
                       d_desc, nframes, d_comp, d_out, rec_base, items, nitems, d_status, nullptr, blk->bfirst,
                       blk->bcount, blk->jobs, blk->jres, 0xFFFFFFFFu, 0u);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#else
// version: 0 = the production kernel; tuning builds add diagnostics
// (DIAG bits above) as 0x100 | DIAG.
int launch_seq_exec(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                    uint8_t *d_out, const uint64_t *rec_base, const uint64_t *items,
                    const uint32_t *nitems, const int32_t *d_status, hipStream_t stream,
                    int version, const SplitScratch *blk, uint32_t stop_last, uint32_t min_dsize)
{
    if (nframes == 0)
        return 0;
    if (blk)   // the block route (production kernel only)
        return launch_seq_exec_seg(d_desc, nframes, d_comp, d_out, rec_base, items, nitems, d_status, stream, blk);
    const dim3 grid((nframes + kXW - 1) / kXW), block(64 * kXW);
#define ZSK_X(D)                                                                                               \
    hipLaunchKernelGGL((seq_exec_kernel<D, kExecStage, false>), grid, block, 0, stream, d_desc, nframes, d_comp, \
                       d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr, nullptr, nullptr, stop_last, \
                       min_dsize)
#ifdef ZSK_TUNING
    switch (version) {
    case 0x101: ZSK_X(1); break;
    case 0x104: ZSK_X(4); break;
    case 0x108: ZSK_X(8); break;
    case 0x122: ZSK_X(34); break;
    case 0x140: ZSK_X(64); break;
    case 0x180: ZSK_X(128); break;
    case 0x141:   // the 4,096-byte stage: five waves per SIMD
        hipLaunchKernelGGL((seq_exec_kernel<0, 4096, false>), grid, block, 0, stream, d_desc, nframes, d_comp,
                           d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr, nullptr, nullptr,
                           stop_last, min_dsize);
        break;
    case 0x142:   // the 3,584-byte stage, six waves per SIMD
        hipLaunchKernelGGL((seq_exec_kernel<0, 3584, false>), grid, block, 0, stream, d_desc, nframes, d_comp,
                           d_out, rec_base, items, nitems, d_status, nullptr, nullptr, nullptr, nullptr, nullptr,
                           stop_last, min_dsize);
        break;
    case 0x143:   // a 2,560-byte stage, eight waves per SIMD (64 VGPRs: spills)
        hipLaunchKernelGGL((seq_exec_kernel<0, 2560, false>), grid, block, 0, stream, d_desc, nframes, d_comp,
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
    default: ZSK_X(0); break;
    }
#else
    (void)version;
    ZSK_X(0);
#endif
#undef ZSK_X
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_seq_exec_frames(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
                           const uint64_t *rec_base, const uint64_t *items, const uint32_t *nitems,
                           int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream, uint32_t stop_last,
                           bool handoff, const uint8_t *lit)
{
    if (nframes == 0)
        return 0;
#ifdef ZSK_TUNING
    // ZSEEK_FRAME_TIMERS: accumulate the phase cycles, print every 100 launches
    static const bool timers = getenv("ZSEEK_FRAME_TIMERS") != nullptr;
    static int calls = 0;
    if (timers && calls == 0) {
        unsigned long long z[8] = {0};
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_ftime), z, sizeof(z), 0, hipMemcpyHostToDevice, stream);
        const uint32_t fd = getenv("ZSEEK_FRAME_DIAG") ? (uint32_t)atoi(getenv("ZSEEK_FRAME_DIAG")) : 0u;
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_fdiag), &fd, sizeof(fd), 0, hipMemcpyHostToDevice, stream);
    }
#endif
    hipLaunchKernelGGL(seq_exec_frame_kernel, dim3(nframes), dim3(kFT), 0, stream, d_desc, nframes, d_comp, d_out,
                       rec_base, items, nitems, d_status, d_fail_at, stop_last, handoff && !lit ? 1u : 0u, lit);
#ifdef ZSK_TUNING
    if (timers && ++calls % 100 == 0) {
        unsigned long long z[8] = {0};
        (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_ftime), sizeof(z), 0, hipMemcpyDeviceToHost, stream);
        (void)hipStreamSynchronize(stream);
        const double fr = z[7] ? (double)z[7] : 1.0;
        fprintf(stderr,
                "frame execute cycles per frame: stage+init %.0f items+scan %.0f literals %.0f matches %.0f "
                "output %.0f | windows %.2f wave passes %.1f (%llu frames)\n",
                z[0] / fr, z[1] / fr, z[2] / fr, z[3] / fr, z[4] / fr, z[5] / fr, z[6] / fr / 16.0, z[7]);
    }
#endif
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_seq_exec_lit(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *lit,
                        uint8_t *d_out, const uint64_t *rec_base, const uint64_t *items,
                        const uint32_t *nitems, int32_t *d_status, hipStream_t stream, bool one,
                        uint32_t max_dsize, uint32_t stop_last)
{
    if (nframes == 0)
        return 0;
    if (one) {   // frames of <= 64 KiB a workgroup each, bigger ones a wave
        hipLaunchKernelGGL(seq_exec_frame_kernel, dim3(nframes), dim3(kFT), 0, stream, d_desc, nframes, nullptr,
                           d_out, rec_base, items, nitems, d_status, nullptr, stop_last, 0u, lit);
        if (max_dsize <= kFMax)
            return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    hipLaunchKernelGGL((seq_exec_kernel<0, 4096, false>), dim3((nframes + kXW - 1) / kXW), dim3(64 * kXW), 0,
                       stream, d_desc, nframes, nullptr, d_out, rec_base, items, nitems, d_status, lit, nullptr,
                       nullptr, nullptr, nullptr, stop_last, one ? kFMax + 1 : 0u);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#endif

}   // namespace zsk
