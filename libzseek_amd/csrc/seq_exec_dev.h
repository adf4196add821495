// seq_exec_dev.h — the execute phase's device code (gfx950): helpers and the
// production kernel seq_exec_kernel<OUTB, SEG>, shared by seq_exec.hip (the
// LZ4 / zstd launchers, OUTB = kExecStage), seq_exec_seg.hip (the block
// route's SEG instantiation, its own translation unit) and seq_exec_tune.hip
// (tuning builds: the diagnostic kernel and the round-0 experiments).
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
//     a round's ready matches one lane each, all four of its 16-byte pieces'
//     loads before their stores (copy_ready);
//   * flush: four chunks' stage reads in flight before their stores; the next
//     batch's items are shifted in before it.
#ifndef ZSK_SEQ_EXEC_DEV_H
#define ZSK_SEQ_EXEC_DEV_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4_dev.h"
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

// Round 0: a descriptor per 16-byte piece (stage destination, length, kind,
// source; a run's piece i = its base + i * (1 + 2^32), source and destination
// advancing together), the wave's pieces dealt one per lane per slot, four
// slots' loads in flight before any write.  A run of 16 bytes or more is
// covered by whole pieces only (its last piece overlaps the one before), so
// only runs under 16 bytes need an exact-length write: whole pieces
// (descriptors [0, TF)) are written with one 16-byte LDS store each, the short
// ones (at most two per lane, [TF, TF + TS)) follow in the same deal with the
// exact write; one DPP scan counts both.  A literal run under 16 bytes whose
// 16-byte load would pass the end of the literal source (the frame's last
// literals) is copied by its lane first, through the range-checked resource
// `lsp`, and gets no descriptor.  A match piece reads HBM below `flushed`,
// else the stage.  (Descriptor halves by 32-bit adds: the 64-bit form
// compiled to two v_mad_u64_u32 per step -- 2.444 -> 2.396 ms at config 2.)
__device__ __forceinline__ void copy_round0(const Stage &S, const uint8_t *lbase, const Span &lsp, uint32_t llen,
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
    const uint32_t lpn = lit < 16 ? 0 : npieces(lit), mpn = mn < 16 ? 0 : npieces(mn);
    const uint32_t nf = lpn + mpn, ns = (uint32_t)ls + (uint32_t)ms;
    const uint32_t inc = wave_incl_add(nf | ns << 16);
    const uint32_t T = lane_val(inc, 63);
    if (T == 0)
        return;
    const uint32_t TF = T & 0xFFFF, TS = T >> 16;
    const uint32_t xf = (inc & 0xFFFF) - nf, xs = TF + (inc >> 16) - ns;
    const uint32_t dl0 = src, dl1 = (saddr(S, op) - S.base) | (lit < 16 ? lit : 16) << 16 | K_LIT << 24;
    const uint32_t dm0 = msrc, dm1 = (saddr(S, mb) - S.base) | (mn < 16 ? mn : 16) << 16 | K_HBM << 24;
    constexpr uint32_t kst1 = (K_STAGE - K_HBM) << 24;
    // the short pieces: one descriptor each
    if (ls)
        *lp<u32x2>(descs + 8 * xs) = (u32x2){dl0, dl1};
    if (ms)
        *lp<u32x2>(descs + 8 * (xs + ls)) = (u32x2){dm0, msrc + 16 > flushed ? dm1 + kst1 : dm1};
    const uint32_t lm = lit < 16 ? 0 : lit - 16, mm = mn < 16 ? 0 : mn - 16;
    const uint32_t al = descs + 8 * xf, am = al + 8 * lpn;
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
    wave_lds_sync();
    // one deal over [0, TF + TS): four slots' loads in flight, then the
    // writes -- a slot holding short pieces (at most the last two) writes
    // exact lengths, every other slot plain 16-byte stores
    const uint32_t TT = TF + TS;
    for (uint32_t t0 = 0; t0 < TT; t0 += 256) {
        u32x4 v[4];
        uint32_t dw[4], sx[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t t = t0 + 64 * j + lane;
            const bool on = t < TT;
            const uint64_t D = *lp<uint64_t>(descs + 8 * (on ? t : 0));
            sx[j] = on ? (uint32_t)D : 0;
            dw[j] = on ? (uint32_t)(D >> 32) : 0;
            const uint32_t kind = dw[j] >> 24;
            const uint8_t *p = kind == K_HBM ? obase + sx[j] : lbase + (kind == K_LIT ? sx[j] : 0);
            v[j] = *reinterpret_cast<const u32x4_l *>(p);
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

// ---- the dependency rounds' copies (round 6) ---------------------------------
// A round's ready matches: one 8-byte entry per 64 bytes of a match of 16
// bytes or more (source, stage destination, bytes left from the entry capped
// at 64, kind) and one per shorter match; a lane per entry loads all four of
// its 16-byte pieces (at min(16 k, left - 16): a match's last pieces overlap
// the ones before and rewrite equal bytes; left < 16 only past the match's
// first entry, so that piece starts inside the match) before storing them.
// copy_round, the round-5 form, copied two pieces per step with each piece's
// stage read waited for before its write: the rounds through copy_ready cut
// SQ_WAIT_INST_LDS from 20 % to 12 % of the execute's wave cycles, 2.396 ->
// 2.385 ms at config 2 (scripts/gpu_kbab.sh, variants 0x730 / 0x731).
constexpr uint32_t kEntryLeftShift = 16, kEntryKindShift = 24;

template <bool LIT>
__device__ __forceinline__ void deal_lane(const Stage &S, const Span &lsp, const Out &O, uint32_t descs,
                                          uint32_t flushed, uint32_t lane, uint32_t a, uint32_t n)
{
    for (uint32_t t0 = 0; t0 < n; t0 += 64) {
        const uint32_t t = t0 + lane;
        if (t < n) {
            const uint64_t D = *lp<uint64_t>(descs + 8 * (a + t));
            const uint32_t hi = (uint32_t)(D >> 32), s = (uint32_t)D;
            const int32_t left = (int32_t)((hi >> kEntryLeftShift) & 0x7F);
            const uint32_t d = S.base + (hi & 0xFFFF);
            int32_t r[4];
            u32x4 v[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                r[q] = min(16 * q, left - 16);
                if (q == 0 || 16 * q < left) {
                    const uint32_t x = s + (uint32_t)r[q];
                    if (LIT)
                        v[q] = bload16(lsp.r, lsp.s0 + x);
                    else if (x + 16 <= flushed)
                        v[q] = bload16(O.sp.r, O.sp.s0 + x);
                    else
                        v[q] = lds16(saddr(S, x));
                }
            }
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (q == 0 || 16 * q < left)
                    *lp<u32x4_l>(d + (uint32_t)r[q]) = v[q];
        }
    }
}

// every lane's ready match (mn bytes from output msrc -> mb, no overlap;
// mn = 0 for the others): entries [0, TM), the short ones after them
__device__ __forceinline__ void copy_ready(const Stage &S, const Span &lsp, const Out &O, uint32_t descs,
                                           uint32_t flushed, uint32_t lane, uint32_t msrc, uint32_t mb, uint32_t mn)
{
    const bool ms = mn != 0 && mn < 16;
    const uint32_t nm = mn < 16 ? 0 : (mn + 63) >> 6;
    const uint32_t inc = wave_incl_add(nm | (uint32_t)ms << 16);
    const uint32_t T = lane_val(inc, 63);
    if (T == 0)
        return;
    const uint32_t TM = T & 0xFFFF, TS = T >> 16;
    const uint32_t xm = (inc & 0xFFFF) - nm, xs = TM + (inc >> 16) - ms;
    const uint32_t dm = (saddr(S, mb) - S.base) | K_HBM << kEntryKindShift;
    if (ms)
        *lp<u32x2>(descs + 8 * xs) = (u32x2){msrc, dm | mn << kEntryLeftShift};
    const uint32_t am = descs + 8 * xm;
    for (uint32_t i = 0; __ballot(i < nm); i++) {
        const uint32_t o = 64 * i;
        if (i < nm)
            *lp<u32x2>(am + 8 * i) = (u32x2){msrc + o, dm + o + (min(mn - o, 64u) << kEntryLeftShift)};
    }
    wave_lds_sync();
    deal_lane<false>(S, lsp, O, descs, flushed, lane, 0, TM);
    for (uint32_t t0 = 0; t0 < TS; t0 += 64) {
        const uint32_t t = t0 + lane;
        if (t < TS) {
            const uint64_t D = *lp<uint64_t>(descs + 8 * (TM + t));
            const uint32_t hi = (uint32_t)(D >> 32), s = (uint32_t)D;
            const u32x4 v = s + 16 <= flushed ? bload16(O.sp.r, O.sp.s0 + s) : lds16(saddr(S, s));
            lds_put(S.base + (hi & 0xFFFF), v, (hi >> kEntryLeftShift) & 0x7F);
        }
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
__device__ __forceinline__ void flush_chunks4(const Stage &S, const Out &O, uint32_t fc, uint32_t end_c, uint32_t lane)
{
    // every chunk inside the frame (the usual batch: neither the frame's
    // first chunk when the output is not 16-byte aligned, nor its partial
    // last one): plain 16-byte stores through a resource based at chunk 0
    if ((fc > 0 || S.a0 == 0) && 16 * end_c <= O.dlen + S.a0) {
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

// The production execute: one wave per frame, kXW frames per
// workgroup.
template <uint32_t OUTB, bool SEG, int WPE = 0>
__global__ __launch_bounds__(64 * kXW) __attribute__((amdgpu_waves_per_eu(WPE ? WPE : SEG ? 4 : (OUTB <= 2560 ? 8 : OUTB <= 3072 ? 7 : OUTB <= 3584 ? 6 : 5)))) void seq_exec_kernel(
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
        // round 0: literal runs + matches whose source precedes the batch
        copy_round0(S, lbase, lsp, llen, O.o, descs, flushed, lane, src, op, lit_n, msrc, mb, early ? ml : 0);
        wave_lds_sync();   // stage bytes of other lanes from here on
        // rounds: matches reading bytes of this batch
        uint64_t pending = __ballot(ml != 0 && !early);
        while (pending) {
            const bool mine = (pending >> lane) & 1;
            // pending destinations are ascending and disjoint: compact them
            // (lane order) into the descriptor area, then binary-search the
            // first one below this lane that ends after msrc; blocked iff it
            // also starts before need
            const uint32_t below = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(pending >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)pending, 0u));
            if (mine)
                *lp<uint64_t>(descs + 8 * below) = ((uint64_t)me << 32) | mb;
            wave_lds_sync();
            uint32_t lo = 0, hi = mine ? below : 0;
            while (__ballot(lo < hi)) {
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
            const bool ready = mine && !(lo < below && mbl < need);
            wave_lds_sync();
            for (uint64_t ov = __ballot(ready && overlap); ov; ov &= ov - 1) {
                const int i = (int)__builtin_ctzll(ov);
                copy_overlap_wave(S, O, flushed, lane_val(mb, i), lane_val(off, i), lane_val(ml, i), lane);
            }
            copy_ready(S, lsp, O, descs, flushed, lane, msrc, mb, ready && !overlap ? ml : 0);
            pending &= ~__ballot(ready);
            wave_lds_sync();
        }
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
        flush_chunks4(S, O, fc, end_c, lane);
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
    }
}

}   // namespace
}   // namespace zsk

#endif
