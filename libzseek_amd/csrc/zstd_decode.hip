// zstd_decode.hip — zstd frame decoding on the GPU (gfx950), the reference's
// ZSTD_decompressDCtx / ZSTD_decompressStream call (decompress.c:434-538;
// libzstd 1.4.9, restated in oracle/zstd_oracle.c).
//
// A zstd frame is serial twice over (Huffman literal streams, FSE sequence
// states), but each serial chain is short and there are many of them, so each
// gets its own lane.  Per batch, after the plan:
//
//   zstd_plan_kernel   lane per frame: walks frame and block headers and each
//   zstd_scan_kernel   block's sequence count -> item bound and block count
//                      per frame -> slot offsets (one workgroup);
//   zstd_frame_kernel  wave per frame: headers (wave-uniform, 256-byte LDS
//                      windows), raw / RLE literals into the literal scratch,
//                      Huffman and FSE tables built in LDS (rank assignment
//                      by ballots) and stored to the block's slot in HBM, one
//                      Huffman job per stream, and the frame's op list;
//   zstd_huf_kernel    lane per Huffman stream (16 blocks per wave, their
//                      tables staged in LDS) -> literal scratch, laid out like
//                      the output;
//   zstd_seq_kernel    lane per frame: replays the op list — FSE states,
//                      repeat offsets, every libzstd check in libzstd's order
//                      -> 8-byte items (LZ4 item format, full offset);
//   seq_exec_kernel    (seq_exec.hip) copies literal runs and matches;
//   zstd_check_kernel  XXH64 content checksums, for frames that carry one.
//
// Backward bitstreams are read straight from HBM: a lane holds the 16-byte
// chunk it is consuming and has the next one in flight.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "lz4_dev.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4d;

constexpr uint32_t kZMagic = 0xFD2FB528u;
constexpr uint32_t kZBlockMax = 128u << 10;
constexpr uint32_t kZW = 2;          // waves (frames) per workgroup
constexpr uint32_t kItemExt = 0x80000000u;

enum : uint32_t {
    ZE_GENERIC = 1,
    ZE_PREFIX = 10,
    ZE_FRAMEPARAM = 14,
    ZE_WINDOW = 16,
    ZE_CORRUPT = 20,
    ZE_CHECKSUM = 22,
    ZE_DICT_CORRUPT = 30,
    ZE_DICT_WRONG = 32,
    ZE_DST_SMALL = 70,
    ZE_SRC_WRONG = 72,
};

__device__ __forceinline__ int32_t zerr(uint32_t e)
{
    return (int32_t)(ST_ZSTD_FLAG | e);
}

// LDS per wave of the frame kernel
struct ZLds {
    uint32_t fse[3][512];     // LL / OF / ML cells: symbol | nbits << 8 | base << 16
    __attribute__((aligned(8))) uint8_t win[256];   // forward window: headers, table descriptions
    uint32_t wfse[64];        // FSE table of compressed Huffman weights
    int16_t norm[256];        // normalized counts
    uint16_t spr[512];        // FSE spread: symbol of each cell in spread order
    uint8_t wts[256];         // Huffman weights
    uint32_t cnt[256];        // per-symbol next-state counters
};

// literal / match length codes: base | extra bits << 24 (RFC 8878 §3.1.1.3.2.1)
__constant__ uint32_t c_ll[36] = {
    0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
    16 | 1u << 24, 18 | 1u << 24, 20 | 1u << 24, 22 | 1u << 24, 24 | 2u << 24, 28 | 2u << 24,
    32 | 3u << 24, 40 | 3u << 24, 48 | 4u << 24, 64 | 6u << 24, 128 | 7u << 24, 256 | 8u << 24,
    512 | 9u << 24, 1024 | 10u << 24, 2048 | 11u << 24, 4096 | 12u << 24, 8192 | 13u << 24,
    16384 | 14u << 24, 32768 | 15u << 24, 65536 | 16u << 24};
__constant__ uint32_t c_ml[53] = {
    3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27,
    28, 29, 30, 31, 32, 33, 34, 35 | 1u << 24, 37 | 1u << 24, 39 | 1u << 24, 41 | 1u << 24,
    43 | 2u << 24, 47 | 2u << 24, 51 | 3u << 24, 59 | 3u << 24, 67 | 4u << 24, 83 | 4u << 24,
    99 | 5u << 24, 131 | 7u << 24, 259 | 8u << 24, 515 | 9u << 24, 1027 | 10u << 24,
    2051 | 11u << 24, 4099 | 12u << 24, 8195 | 13u << 24, 16387 | 14u << 24, 32771 | 15u << 24,
    65539 | 16u << 24};
// predefined distributions (RFC 8878 §3.1.1.3.2.2)
__constant__ int8_t c_ll_def[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                    2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int8_t c_ml_def[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int8_t c_of_def[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// LDS access by byte address (pointers into LDS converted to their offset)
template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T *lp(const void *a)
{
    return (__attribute__((address_space(3))) T *)(uintptr_t)(uint32_t)(uintptr_t)a;
}

typedef u32x4 u32x4_a4 __attribute__((aligned(4)));

template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T *la(uint32_t a)
{
    return (__attribute__((address_space(3))) T *)(uintptr_t)a;
}

__device__ __forceinline__ uint32_t ldsaddr(const void *p)
{
    return (uint32_t)(uintptr_t)p;
}

__device__ __forceinline__ uint32_t lane_id()
{
    return threadIdx.x & 63;
}

__device__ __forceinline__ int32_t hibit(uint32_t v)
{
    return 31 - __builtin_clz(v);
}

#ifdef ZSK_TUNING
// tuning builds: the frame kernel's cycles, lane 0 at section ends: [0]
// kernel, [1] Huffman descriptions, [2] sequence tables (+ slot cells), [3]
// window stagings, [4] frames, [5..7] the weights description: normalized
// counts, table, walk; printed under ZSEEK_ZFRAME_TIMERS
__device__ unsigned long long g_zftime[12];
#define ZF_T0(v) const uint64_t v = __builtin_readcyclecounter();
#define ZF_ADD(i, v)                                                                                  \
    if (lane_id() == 0)                                                                               \
        atomicAdd(&g_zftime[i], (unsigned long long)(__builtin_readcyclecounter() - v));
#else
#define ZF_T0(v)
#define ZF_ADD(i, v)
#endif

// ---- compressed input: coordinates x relative to the frame's 4-aligned base
struct In {
    const uint8_t *base4;   // frame start rounded down to 4 bytes
    uint32_t s0;            // frame byte 0 is coordinate s0
    uint32_t amax;          // last dword coordinate inside the frame
};

// 256 bytes (4 per lane) from the dword coordinate a into LDS at dst,
// asynchronous (global_load_lds_dword; waited by dma_wait).  Coordinates
// outside the frame are clamped onto its last dword: those bytes are never
// interpreted.
__device__ __forceinline__ void dma256(const In &I, uint32_t a, uint32_t dst)
{
    uint32_t x = a + 4 * lane_id();
    x = x > I.amax ? I.amax : x;
    __builtin_amdgcn_global_load_lds((const void *)(I.base4 + x), la<void>(uni(dst)), 4, 0, 0);
}

// s_waitcnt vmcnt(0) through the builtin, so the compiler's wait-count pass
// knows the LDS-DMA writes have landed and adds no waits of its own before
// later LDS reads (expcnt / lgkmcnt fields left at their maximum)
__device__ __forceinline__ void dma_wait()
{
    __builtin_amdgcn_s_waitcnt(0x0F70);
    wave_lds_sync();
}

// forward window: 256 bytes from frame offset p (rounded down to 4); returns
// the coordinate of win[0]
__device__ __forceinline__ uint32_t stage_win(ZLds &L, const In &I, uint32_t p)
{
    ZF_T0(t0)
    const uint32_t a = (I.s0 + p) & ~3u;
    dma256(I, a, ldsaddr(L.win));
    dma_wait();
    ZF_ADD(3, t0)
    return a;
}

__device__ __forceinline__ uint32_t wb(const ZLds &L, uint32_t wx, const In &I, uint32_t p)
{
    return *lp<uint8_t>(L.win + (I.s0 + p - wx));
}

// ---- FSE tables -----------------------------------------------------------------
// Normalized counts from the window at bit 0 of window offset wofs,
// RFC 8878 §4.1.1 / FSE_readNCount.  Returns bytes used, or 0 on error
// (*err set).  norm[] receives nsym entries; the caller zeroes norm[0..max_sym]
// first (zero counts are not written).  The bits are read through a 64-bit
// register window W = window bits [wp, wp + 64), reloaded every 32 bits.
// Wave-uniform (every lane runs it, its state in scalar registers: the scalar
// unit has issue to spare in the VALU-bound frame kernel; lane 0 stores).
__device__ __forceinline__ uint32_t read_ncount(ZLds &L, uint32_t wofs, uint32_t avail, uint32_t max_sym,
                                                uint32_t max_log, uint32_t *tlog, uint32_t *nsym, uint32_t *err)
{
    // (uniform in the compiler's eyes: else the walk is a divergent loop,
    // every branch an exec-mask save / restore)
    wofs = uni(wofs);
    avail = uni(avail);
    uint32_t pos = 8 * wofs, wp = pos + 64;   // forces the first load
    uint64_t W = 0;
    // the window's 64 dwords one per lane: a reload is two readlanes, not an
    // LDS round trip (the walk is a lone wave's serial chain)
    const uint32_t wv = *lp<uint32_t>(L.win + 4 * lane_id());
    auto bits = [&](uint32_t n) -> uint32_t {   // n <= 16 bits at pos, not consumed
        if (pos - wp >= 32) {
            wp = pos & ~31u;
            const uint32_t d = wp >> 5;
            const uint32_t lo = d < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)wv, (int)d) : 0u;
            const uint32_t hi = d + 1 < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)wv, (int)(d + 1)) : 0u;
            W = ((uint64_t)hi << 32) | lo;
        }
        return (uint32_t)(W >> (pos - wp)) & ((1u << n) - 1);
    };
    const uint32_t tl = bits(4) + 5;
    pos += 4;
    if (tl > max_log) {
        *err = ZE_CORRUPT;
        return 0;
    }
    // (threshold = 1 << (nbits - 1) throughout: derived, not carried -- one
    // loop value fewer in the frame kernel's tight scalar register budget)
    int32_t remaining = (1 << tl) + 1;
    uint32_t nbits = tl + 1, sym = 0;
    bool prev0 = false;
    while (remaining > 1 && sym <= max_sym) {
        if (prev0) {
            uint32_t n0 = sym;
            while (bits(16) == 0xFFFF) {
                n0 += 24;
                pos += 16;
            }
            while (bits(2) == 3) {
                n0 += 3;
                pos += 2;
            }
            n0 += bits(2);
            pos += 2;
            if (n0 > max_sym) {
                *err = ZE_CORRUPT;
                return 0;
            }
            sym = n0;   // the skipped counts stay 0
        }
        const int32_t threshold = 1 << (nbits - 1);
        const int32_t mx = 2 * threshold - 1 - remaining;
        const int32_t v = (int32_t)bits(nbits);
        // (both field widths as selects, no branch per symbol)
        const bool lo = (v & (threshold - 1)) < mx;
        const int32_t wide = v & (2 * threshold - 1);
        int32_t count = lo ? v & (threshold - 1) : wide >= threshold ? wide - mx : wide;
        pos += lo ? nbits - 1 : nbits;
        count--;
        remaining -= count < 0 ? -count : count;
        // (every lane, the same value: no exec-mask branch; a zero count
        // writes the zero norm_clear left)
        *lp<int16_t>(&L.norm[sym]) = (int16_t)count;
        sym++;
        prev0 = count == 0;
        // FSE_readNCount's `while (remaining < threshold) { nbBits--;
        // threshold >>= 1; }`: remaining stays >= 1 (a count never exceeds
        // it), so the field width becomes min(nbits, log2(remaining) + 1)
        nbits = min(nbits, 32u - (uint32_t)__builtin_clz((uint32_t)remaining));
    }
    // (ran off the window -- no valid description is that long -- checked
    // once here: past it the walk reads zeros, the loop ends within max_sym
    // symbols and the description is refused as before)
    const uint32_t used = (pos + 7) / 8 - wofs;
    if (pos > 8 * 256 || remaining != 1 || used > avail) {
        *err = ZE_CORRUPT;
        return 0;
    }
    *tlog = tl;
    *nsym = sym;
    return used;
}

// norm[0..n) = 0, wave-wide (before read_ncount)
__device__ __forceinline__ void norm_clear(ZLds &L, uint32_t n)
{
    for (uint32_t i = lane_id(); i < n; i += 64)
        *lp<int16_t>(&L.norm[i]) = 0;
    wave_lds_sync();
}

// Decoding table from norm[0..nsym) with accuracy log tl (FSE_buildDTable):
// cell = symbol | nbits << 8 | base << 16.  Wave-wide.  With nsym <= 64 (every
// table zstd defines: LL 36, OF 32, ML 53, Huffman weights 13 symbols) it is
// built without serial loops: the spread visits positions (j * step) & mask
// and the valid ones (<= high) take the cells in symbol order, so a prefix
// count over j gives each position its cell and a prefix max over the symbol
// starts gives each cell its symbol; next states are ranked per 64-cell group
// by ballots, with the per-symbol counters in lane registers.
__device__ __forceinline__ void fse_build(ZLds &L, uint32_t *tab, uint32_t nsym, uint32_t tl)
{
    const uint32_t lane = lane_id();
    const uint32_t size = 1u << tl, mask = size - 1;
    const uint32_t step = (size >> 1) + (size >> 3) + 3;
    const uint64_t below = (1ull << lane) - 1;
    wave_lds_sync();   // norm[] from lane 0
    if (nsym > 64) {
        if (lane == 0) {
            uint32_t high = size - 1;
            for (uint32_t s = 0; s < nsym; s++)
                if (L.norm[s] == -1)
                    *lp<uint32_t>(tab + high--) = s;
            uint32_t pos = 0;
            for (uint32_t s = 0; s < nsym; s++) {
                for (int32_t i = 0; i < L.norm[s]; i++) {
                    *lp<uint32_t>(tab + pos) = s;
                    do
                        pos = (pos + step) & mask;
                    while (pos > high);
                }
            }
        }
        for (uint32_t s = lane; s < nsym; s += 64)
            L.cnt[s] = L.norm[s] == -1 ? 1u : (uint32_t)L.norm[s];
        wave_lds_sync();
        for (uint32_t u0 = 0; u0 < size; u0 += 64) {
            const uint32_t u = u0 + lane;
            const bool act = u < size;
            const uint32_t s = act ? (*lp<uint32_t>(tab + u) & 0xFF) : 0xFFFFu;
            uint64_t rem = __ballot(act);
            while (rem) {
                const uint32_t sj = lane_val(s, __builtin_ctzll(rem));
                const uint64_t m = __ballot(act && s == sj);
                const uint32_t base = uni(L.cnt[sj]);
                if ((m >> lane) & 1) {
                    const uint32_t ns = base + (uint32_t)__builtin_popcountll(m & below);
                    const uint32_t nb = tl - (uint32_t)hibit(ns);
                    *lp<uint32_t>(tab + u) = sj | nb << 8 | ((ns << nb) - size) << 16;
                }
                if (lane == 0)
                    L.cnt[sj] = base + (uint32_t)__builtin_popcountll(m);
                wave_lds_sync();
                rem &= ~m;
            }
        }
        return;
    }
    // lane s: symbol s
    const int32_t nc = lane < nsym ? (int32_t)*lp<int16_t>(&L.norm[lane]) : 0;
    const uint32_t c = nc > 0 ? (uint32_t)nc : 0u;
    const bool low = nc == -1;
    const uint32_t K = wave_incl_add(c) - c;   // the symbol's first cell in spread order
    const uint64_t lm = __ballot(low);
    const uint32_t high = size - 1 - (uint32_t)__builtin_popcountll(lm);
    for (uint32_t u = lane; u < size; u += 64)
        *lp<uint16_t>(&L.spr[u]) = 0;
    wave_lds_sync();
    if (c)
        *lp<uint16_t>(&L.spr[K]) = (uint16_t)(lane + 1);
    wave_lds_sync();
    uint32_t carry = 0;
    for (uint32_t k0 = 0; k0 < size; k0 += 64) {
        const uint32_t k = k0 + lane;
        const uint32_t v = k < size ? (uint32_t)*lp<uint16_t>(&L.spr[k]) : 0u;
        const uint32_t pm = max(carry, wave_incl_max(v));
        if (k < size)
            *lp<uint16_t>(&L.spr[k]) = (uint16_t)(pm - 1);
        carry = lane_val(pm, 63);
    }
    wave_lds_sync();
    uint32_t kb = 0;
    for (uint32_t j0 = 0; j0 < size; j0 += 64) {
        const uint32_t j = j0 + lane, p = (j * step) & mask;
        const bool valid = j < size && p <= high;
        const uint64_t m = __ballot(valid);
        if (valid)
            *lp<uint32_t>(tab + p) = *lp<uint16_t>(&L.spr[kb + (uint32_t)__builtin_popcountll(m & below)]);
        kb += (uint32_t)__builtin_popcountll(m);
    }
    if (low)   // low-probability symbols at the top, in symbol order from size - 1 down
        *lp<uint32_t>(tab + size - 1 - (uint32_t)__builtin_popcountll(lm & below)) = lane;
    wave_lds_sync();
    // next states: lane s holds symbol s's counter; per 64-cell group each lane
    // finds the lanes holding its symbol with six bit-sliced ballots (symbols
    // < 64), ranks itself among them, and the group's per-symbol totals come
    // back through cnt[] (one ballot loop per distinct symbol cost ~5x the
    // VALU issue of the whole kernel's other table work)
    uint32_t cntr = low ? 1u : c;
    for (uint32_t u0 = 0; u0 < size; u0 += 64) {
        const uint32_t u = u0 + lane;
        const bool act = u < size;
        const uint32_t s = act ? (*lp<uint32_t>(tab + u) & 0xFF) : 0u;
        uint64_t m = __ballot(act);
#pragma unroll
        for (int bit = 0; bit < 6; bit++) {
            const bool one = (s >> bit) & 1;
            const uint64_t bb = __ballot(one);
            m &= one ? bb : ~bb;
        }
        const uint32_t base = (uint32_t)__shfl((int)cntr, (int)s, 64);
        *lp<uint32_t>(&L.cnt[lane]) = 0;
        wave_lds_sync();
        if (act) {
            const uint32_t ns = base + (uint32_t)__builtin_popcountll(m & below);
            const uint32_t nb = tl - (uint32_t)hibit(ns);
            *lp<uint32_t>(tab + u) = s | nb << 8 | ((ns << nb) - size) << 16;
            *lp<uint32_t>(&L.cnt[s]) = (uint32_t)__builtin_popcountll(m);   // equal for every lane of s
        }
        wave_lds_sync();
        cntr += *lp<uint32_t>(&L.cnt[lane]);
        wave_lds_sync();
    }
}

// ---- Huffman tables --------------------------------------------------------------
// Tree description at frame offset p (window staged at wx); returns its size
// or 0 on error.  Writes the 2^log decoding cells (nbits | symbol << 8) to
// cells (HBM); *log receives the table log.  Wave-wide.
__device__ __forceinline__ uint32_t huf_read(ZLds &L, const In &I, uint32_t wx, uint32_t p, uint32_t avail,
                                             uint32_t *log, uint16_t *cells)
{
    const uint32_t lane = lane_id();
    const uint32_t hb = uni(wb(L, wx, I, p));
    const uint32_t wofs = uni(I.s0 + p - wx + 1);   // window offset of the description body (uniform: see read_ncount)
    uint32_t nw = 0, used = 0, err = 0;
    if (hb < 128) {
        if (1 + hb > avail || wofs + hb > 256)
            return 0;
        uint32_t tl = 0, nsym = 0;
        uint32_t hs = 0;
        ZF_T0(tq0)
        norm_clear(L, 256);
        hs = read_ncount(L, wofs, hb, 255, 6, &tl, &nsym, &err);
        ZF_ADD(5, tq0)
        hs = uni(hs);
        if (uni(err))
            return 0;
        tl = uni(tl);
        nsym = uni(nsym);
        ZF_T0(tq1)
        fse_build(L, L.wfse, nsym, tl);
        ZF_ADD(6, tq1)
        ZF_T0(tq2)
        {
            // backward stream inside the window: two interleaved states
            // (wave-uniform, as read_ncount; lane 0 stores the weights)
            const uint32_t b0 = wofs + hs, bn = hb - hs;
            const uint32_t lastb = bn ? uni(*lp<uint8_t>(L.win + b0 + bn - 1)) : 0;
            // the window's dwords and the weights' FSE cells (<= 64) one per
            // lane: the walk reads them by readlane, not LDS round trips
            const uint32_t wv = *lp<uint32_t>(L.win + 4 * lane);
            const uint32_t fv = *lp<uint32_t>(L.wfse + (lane < (1u << tl) ? lane : 0u));
            auto w32 = [&](uint32_t bit) -> uint32_t {   // win32 from the registers
                const uint32_t d = bit >> 5;
                const uint32_t lo = d < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)wv, (int)d) : 0u;
                const uint32_t hi = d + 1 < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)wv, (int)(d + 1)) : 0u;
                return (uint32_t)((((uint64_t)hi << 32) | lo) >> (bit & 31));
            };
            auto cellw = [&](uint32_t st) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)fv, (int)st); };
            if (!lastb) {
                err = 1;
            } else {
                int32_t pos = (int32_t)(8 * (bn - 1)) + hibit(lastb);
                // n backward bits ending at pos (bits below the stream read as 0)
                auto rb = [&](uint32_t n) -> uint32_t {
                    pos -= (int32_t)n;
                    const int32_t x = (int32_t)(8 * b0) + pos;
                    uint32_t v = (x >= 0 ? w32((uint32_t)x) : w32(0) << (uint32_t)(-x)) & ((1u << n) - 1);
                    if (pos < 0)
                        v = -pos >= (int32_t)n ? 0u : v & (~0u << (uint32_t)(-pos));
                    return v;
                };
                auto put = [&](uint32_t c) {
                    if (lane == 0)
                        L.wts[nw] = (uint8_t)c;
                    nw++;
                };
                uint32_t s1 = rb(tl), s2 = rb(tl);
                for (;;) {
                    if (nw > 253) {
                        err = 1;
                        break;
                    }
                    uint32_t c = cellw(s1);
                    put(c);
                    s1 = (c >> 16) + rb((c >> 8) & 0xFF);
                    if (pos < 0) {
                        put(cellw(s2));
                        break;
                    }
                    if (nw > 253) {
                        err = 1;
                        break;
                    }
                    c = cellw(s2);
                    put(c);
                    s2 = (c >> 16) + rb((c >> 8) & 0xFF);
                    if (pos < 0) {
                        put(cellw(s1));
                        break;
                    }
                }
            }
        }
        wave_lds_sync();   // lane 0's weights before every lane reads them
        ZF_ADD(7, tq2)
        used = 1 + hb;
    } else {
        nw = hb - 127;
        const uint32_t bytes = (nw + 1) / 2;
        if (1 + bytes > avail || wofs + bytes > 256)
            return 0;
        for (uint32_t i = lane; i < nw; i += 64) {
            const uint32_t by = *lp<uint8_t>(L.win + wofs + i / 2);
            L.wts[i] = (uint8_t)((i & 1) ? (by & 15) : (by >> 4));
        }
        used = 1 + bytes;
    }
    if (uni(err))
        return 0;
    nw = uni(nw);
    // weights -> table log, implied last weight, canonical cell ranges
    uint32_t total = 0, bad = 0, r1 = 0;
    for (uint32_t i = lane; i < nw; i += 64) {
        const uint32_t w = L.wts[i];
        bad |= w >= 12;
        total += (1u << w) >> 1;
        r1 += w == 1;
    }
    // wave sums (few values; DPP-free reduction through readlane is enough here)
    for (int k = 32; k >= 1; k >>= 1) {
        total += __shfl_xor(total, k, 64);
        r1 += __shfl_xor(r1, k, 64);
        bad |= __shfl_xor(bad, k, 64);
    }
    total = uni(total);
    r1 = uni(r1);
    if (uni(bad) || total == 0)
        return 0;
    const uint32_t lg = (uint32_t)hibit(total) + 1;
    if (lg > 12)
        return 0;
    const uint32_t rest = (1u << lg) - total;
    if (rest != (1u << hibit(rest)))
        return 0;
    const uint32_t lastw = (uint32_t)hibit(rest) + 1;
    if (lane == 0)
        L.wts[nw] = (uint8_t)lastw;
    wave_lds_sync();
    r1 += lastw == 1;
    if (r1 < 2 || (r1 & 1))
        return 0;
    nw++;
    // canonical cells, straight into the block's slot: class k (weight k,
    // 2^(k-1) cells per symbol) follows the lower classes, its symbols in
    // symbol order
    uint32_t wl[4];
#pragma unroll
    for (int ps = 0; ps < 4; ps++) {
        const uint32_t s = 64 * ps + lane;
        wl[ps] = s < nw ? (uint32_t)*lp<uint8_t>(&L.wts[s]) : 0u;
    }
    const uint64_t below = (1ull << lane) - 1;
    uint32_t c0 = 0;
    for (uint32_t k = 1; k <= lg; k++) {
        uint32_t n = 0;
#pragma unroll
        for (int ps = 0; ps < 4; ps++) {
            const uint64_t m = __ballot(wl[ps] == k);
            if (wl[ps] == k)
                *lp<int16_t>(&L.norm[n + (uint32_t)__builtin_popcountll(m & below)]) = (int16_t)(64 * ps + lane);
            n += (uint32_t)__builtin_popcountll(m);
        }
        if (!n)
            continue;
        wave_lds_sync();
        const uint32_t sh = k - 1, ck = n << sh, nb = lg + 1 - k;
        for (uint32_t u = lane; u < ck; u += 64)
            cells[c0 + u] = (uint16_t)((uint32_t)*lp<int16_t>(&L.norm[u >> sh]) << 8 | nb);
        c0 += ck;
        wave_lds_sync();   // before the list is rewritten
    }
    *log = lg;
    return used;
}

// ---- phase hand-off records (frame kernel -> Huffman / sequence kernels) --------------
// Per-block decoding tables, in HBM: the block's Huffman cells and its three
// FSE tables, so the lane-parallel kernels need no table building of their own.
constexpr uint32_t kZSlot = 10752;               // bytes per block slot
constexpr uint32_t kSlotFse = 8192;              // byte offset of the FSE cells (u16)
constexpr uint32_t kFseOff[3] = {0, 512, 768};   // LL / OF / ML, in u16 cells

// One Huffman stream (4 per block; len == 0: no stream).  32 bytes.
struct HufJob {
    uint64_t src;   // comp coordinate of the stream's first byte
    uint64_t dst;   // literal-scratch coordinate of its first symbol
    uint32_t len;   // stream bytes
    uint32_t cnt;   // symbols to decode
    uint32_t lim;   // symbols that may be stored (the frame's capacity)
    uint32_t tab;   // slot holding the Huffman cells | X2 decoder << 27 | table log << 28
};
constexpr uint32_t kHufSlotMask = (1u << 27) - 1;

// HUF_selectDecoder (libzstd 1.4.9): the double-symbol decoder (X2) when its
// modelled time (+1/8 for its larger table) beats X1's, per compression-ratio
// bucket q and 256-byte output units.  dst >= 1.
__device__ __forceinline__ uint32_t huf_select_x2(uint32_t dst, uint32_t csrc)
{
    constexpr uint16_t kT[16][4] = {
        {0, 0, 1, 1},          {0, 0, 1, 1},          {38, 130, 1313, 74},   {448, 128, 1353, 74},
        {556, 128, 1353, 74},  {714, 128, 1418, 74},  {883, 128, 1437, 74},  {897, 128, 1515, 75},
        {926, 128, 1613, 75},  {947, 128, 1729, 77},  {1107, 128, 2083, 81}, {1177, 128, 2379, 87},
        {1242, 128, 2415, 93}, {1349, 128, 2644, 106}, {1455, 128, 2422, 124}, {722, 128, 1891, 145},
    };
    const uint32_t q = csrc >= dst ? 15u : csrc * 16u / dst, d256 = dst >> 8;
    const uint32_t t0 = kT[q][0] + kT[q][1] * d256;
    uint32_t t1 = kT[q][2] + kT[q][3] * d256;
    t1 += t1 >> 3;
    return t1 < t0 ? 1u : 0u;
}
static_assert(sizeof(HufJob) == 32, "HufJob");

// Per-frame op list, in decode order.  The frame kernel stops at its first
// error (OP_ERR); the sequence kernel replays the list and reports the first
// failure in libzstd's order, interleaving the Huffman kernel's stream
// results (OP_LIT) with the frame kernel's header checks.
enum : uint32_t {
    OP_LIT = 1,   // a: block -> the block's Huffman streams must have decoded cleanly
    OP_SEQ,       // a: nseq, b: stream (frame offset), c: stream bytes, d: literal start,
                  // e: literal count, f: block, g: table logs LL | OF << 4 | ML << 8
    OP_RUN,       // a: literal start, b: bytes (raw / RLE block)
    OP_FBEGIN,    // zstd frame starts: repeat offsets reset
    OP_FEND,      // a: 1 = content size present, 2 = checksum; b/c: size lo/hi; d: checksum
    OP_ERR,       // a: status
    OP_DONE,
};
struct ZOp {
    uint32_t k, a, b, c, d, e, f, g;
};
static_assert(sizeof(ZOp) == 32, "ZOp");

__device__ __forceinline__ uint64_t op_base(const uint64_t *blk_base, uint32_t f)
{
    return 4 * blk_base[f] + 4ull * f;
}

// ---- frame kernel state ------------------------------------------------------------------
struct Frame {
    In I;
    uint32_t clen;     // compressed entry bytes
    uint64_t c_abs;    // comp coordinate of the entry
    uint64_t d_abs;    // literal-scratch coordinate of the entry
    uint8_t *lit;      // literal scratch of this frame (laid out like its output)
    uint32_t cap;      // output capacity (seek-table dSize)
    uint32_t lo;       // literal bytes placed in the scratch
    uint32_t huf_log;  // 0: no Huffman table yet
    uint32_t huf_slot; // block slot holding the current Huffman cells
    uint32_t tlog[3];  // LL / OF / ML table logs (valid flags below)
    uint32_t tvalid;   // bit t: table t valid
    ZOp *ops;          // this frame's op list
    uint32_t nop, op_cap;
    uint64_t blk0;     // first block slot of the frame
    uint32_t nblk, blk_cap;
    uint8_t *slots;
    HufJob *jobs;
    // the one-frame route's helper wave (HelpBox below): a posted Huffman
    // description (its block's jobs and table log completed at the block's end)
    struct HelpBox *help = nullptr;
    bool posted = false;
    uint32_t post_ns = 0;
};

// The one-frame route's frame kernel runs a second wave beside the frame's:
// a block's Huffman description (a serial walk of its weights, ~60K cycles)
// is decoded there while the frame's wave parses the block's sequence
// section (the FSE tables, ~90K) -- the description's size is known from its
// first byte, so nothing after it waits for its decode.  One box in LDS per
// workgroup; the waves meet at two barriers per posted description (A: posted
// or done, B: decoded).
struct HelpBox {
    uint32_t kind;   // 1 = decode the description at q (qn bytes) into slot g; 0 = done
    uint32_t q, qn;
    uint32_t g;
    uint32_t hs, lg;   // result: bytes used (0 = corrupt), table log
};

// append an op (wave-uniform; lane 0 writes).  The last slot is kept for the
// error that ends a list which would overflow.
__device__ __forceinline__ bool put_op(Frame &F, uint32_t k, uint32_t a = 0, uint32_t b = 0, uint32_t c = 0,
                                       uint32_t d = 0, uint32_t e = 0, uint32_t f = 0, uint32_t g = 0)
{
    if (F.nop + 1 >= F.op_cap && k != OP_ERR && k != OP_DONE)
        return false;
    if (lane_id() == 0)
        F.ops[F.nop] = ZOp{k, a, b, c, d, e, f, g};
    F.nop++;
    return true;
}

// write bytes [p, p + n) of v (16 bytes) into the literal scratch, clamped at
// the frame's capacity (corrupt frames may announce more literals)
__device__ __forceinline__ void lit_put(Frame &F, uint32_t p, u32x4 v, uint32_t n)
{
    if (p >= F.cap)
        return;
    if (p + n > F.cap)
        n = F.cap - p;
    store_exact(F.lit + p, v, n);
}

// Literals section at frame offset p (block bytes [p, p + n)) of the block
// with slot g; *used, *litn, *huf (Huffman streams queued).  Returns 0 or a
// zstd error.  Wave-wide.
__device__ __forceinline__ uint32_t literals(ZLds &L, Frame &F, uint64_t g, uint32_t p, uint32_t n,
                                             uint32_t *used, uint32_t *litn, bool *huf)
{
    const uint32_t lane = lane_id();
    *huf = false;
    if (n < 3)
        return ZE_CORRUPT;
    const uint32_t wx = stage_win(L, F.I, p);
    auto B = [&](uint32_t i) { return uni(wb(L, wx, F.I, p + i)); };
    const uint32_t b0 = B(0), type = b0 & 3, sf = (b0 >> 2) & 3;
    if (type <= 1) {
        uint32_t lh, size;
        if (sf == 1) {
            lh = 2;
            size = (b0 | B(1) << 8) >> 4;
        } else if (sf == 3) {
            lh = 3;
            size = (b0 | B(1) << 8 | B(2) << 16) >> 4;
        } else {
            lh = 1;
            size = b0 >> 3;
        }
        if (type == 0) {
            if (lh + size > n)
                return ZE_CORRUPT;
            // raw literals: wave copy compressed -> scratch
            const Span sp = make_span(F.I.base4 + F.I.s0, F.clen);
            for (uint32_t k = 16 * lane; k < size; k += 1024) {
                const u32x4 v = load16u(sp.r, sp.s0 + p + lh + k);
                lit_put(F, F.lo + k, v, size - k < 16 ? size - k : 16);
            }
            *used = lh + size;
        } else {
            if (lh + 1 > n || size > kZBlockMax)
                return ZE_CORRUPT;
            const uint32_t bv = B(lh) * 0x01010101u;
            for (uint32_t k = 16 * lane; k < size; k += 1024)
                lit_put(F, F.lo + k, (u32x4){bv, bv, bv, bv}, size - k < 16 ? size - k : 16);
            *used = lh + 1;
        }
        *litn = size;
        return 0;
    }
    if (n < 5)
        return ZE_CORRUPT;
    const uint32_t lhc = b0 | B(1) << 8 | B(2) << 16 | B(3) << 24;
    uint32_t lh, size, csize, ns = 4;
    if (sf <= 1) {
        ns = sf == 0 ? 1 : 4;
        lh = 3;
        size = (lhc >> 4) & 0x3FF;
        csize = (lhc >> 14) & 0x3FF;
    } else if (sf == 2) {
        lh = 4;
        size = (lhc >> 4) & 0x3FFF;
        csize = lhc >> 18;
    } else {
        lh = 5;
        size = (lhc >> 4) & 0x3FFFF;
        csize = (lhc >> 22) + (B(4) << 10);
    }
    if (size > kZBlockMax || csize + lh > n)
        return ZE_CORRUPT;
    uint32_t q = p + lh, qn = csize;
    if (type == 2) {
        // libzstd's decoder choice (ZSTD_decodeLiteralsBlock): one stream ->
        // X1; four -> HUF_decompress4X_hufOnly: no literals is an error, then
        // X1 or X2 by HUF_selectDecoder.  A treeless section reuses the
        // table's decoder (the X2 flag rides in huf_slot).
        if (ns == 4 && size == 0)
            return ZE_CORRUPT;
        const uint32_t x2 = ns == 4 ? huf_select_x2(size, csize) : 0u;
        uint32_t lg = 0, hs = 0;
        if (F.help) {
            // the helper wave decodes it; its size from its first byte (the
            // size checks huf_read makes before decoding)
            const uint32_t h0 = uni(wb(L, wx, F.I, q));
            if (h0 < 128) {
                if (1 + h0 > qn)
                    return ZE_CORRUPT;
                hs = 1 + h0;
            } else {
                const uint32_t bytes = (h0 - 127 + 1) / 2;
                if (1 + bytes > qn)
                    return ZE_CORRUPT;
                hs = 1 + bytes;
            }
            if (lane == 0) {
                F.help->kind = 1;
                F.help->q = q;
                F.help->qn = qn;
                F.help->g = (uint32_t)g;
            }
            __syncthreads();   // A: posted
            F.posted = true;
            lg = 1;   // (placeholder: the log arrives at the block's end)
        } else {
            ZF_T0(t0)
            hs = huf_read(L, F.I, wx, q, qn, &lg, reinterpret_cast<uint16_t *>(F.slots + g * kZSlot));
            ZF_ADD(1, t0)
            if (!hs)
                return ZE_CORRUPT;
        }
        F.huf_log = lg;
        F.huf_slot = (uint32_t)g | x2 << 27;
        q += hs;
        qn -= hs;
    } else if (!F.huf_log) {
        return ZE_DICT_CORRUPT;
    }
    uint32_t len[4] = {0, 0, 0, 0};
    if (ns == 1) {
        len[0] = qn;
    } else {
        if (qn < 10)
            return ZE_CORRUPT;
        const uint32_t wx2 = stage_win(L, F.I, q);
        auto C = [&](uint32_t i) { return uni(wb(L, wx2, F.I, q + i)); };
        len[0] = C(0) | C(1) << 8;
        len[1] = C(2) | C(3) << 8;
        len[2] = C(4) | C(5) << 8;
        if (len[0] + len[1] + len[2] + 6 > qn)
            return ZE_CORRUPT;
        len[3] = qn - 6 - len[0] - len[1] - len[2];
        if (3 * ((size + 3) / 4) > size)
            return ZE_CORRUPT;
        q += 6;
    }
    for (uint32_t k = 0; k < ns; k++)
        if (len[k] == 0)
            return ZE_CORRUPT;   // a stream without its end mark
    // one job per stream; the cells are in the slot of the block that sent the
    // table (this one, or an earlier one for a treeless literals section)
    const uint32_t lg = F.huf_log;
    if (lane < ns) {
        const uint32_t seg = ns == 1 ? size : (size + 3) / 4;
        const uint32_t off = q + (lane > 0 ? len[0] : 0) + (lane > 1 ? len[1] : 0) + (lane > 2 ? len[2] : 0);
        const uint32_t dst = F.lo + lane * seg;
        const uint32_t cnt = lane + 1 < ns ? seg : size - lane * seg;
        const uint32_t room = dst < F.cap ? F.cap - dst : 0;
        HufJob J;
        J.src = F.c_abs + off;
        J.dst = F.d_abs + dst;
        J.len = lane == 0 ? len[0] : lane == 1 ? len[1] : lane == 2 ? len[2] : len[3];
        J.cnt = cnt;
        J.lim = cnt < room ? cnt : room;
        J.tab = F.huf_slot | (F.posted ? 0u : lg << 28);   // (posted: the log is or-ed in later)
        F.jobs[4 * g + lane] = J;
    }
    F.post_ns = ns;
    *huf = true;
    *used = lh + csize;
    *litn = size;
    return 0;
}

// one of the sequence tables; returns bytes used, or ~0u with *err
__device__ __forceinline__ uint32_t seq_table(ZLds &L, Frame &F, uint32_t t, uint32_t mode, uint32_t p,
                              uint32_t avail, uint32_t *err)
{
    const uint32_t lane = lane_id();
    uint32_t *tab = L.fse[t];
    const uint32_t max_sym = t == 0 ? 35 : t == 1 ? 31 : 52, max_log = t == 1 ? 8 : 9;
    if (mode == 0) {
        const int8_t *def = t == 0 ? c_ll_def : t == 1 ? c_of_def : c_ml_def;
        const uint32_t nsym = t == 0 ? 36 : t == 1 ? 29 : 53, lg = t == 1 ? 5 : 6;
        for (uint32_t s = lane; s < nsym; s += 64)
            L.norm[s] = def[s];
        fse_build(L, tab, nsym, lg);
        F.tlog[t] = lg;
        F.tvalid |= 1u << t;
        return 0;
    }
    if (mode == 1) {
        if (avail == 0) {
            *err = ZE_SRC_WRONG;
            return ~0u;
        }
        const uint32_t wx = stage_win(L, F.I, p);
        const uint32_t sym = uni(wb(L, wx, F.I, p));
        if (sym > max_sym) {
            *err = ZE_CORRUPT;
            return ~0u;
        }
        if (lane == 0)
            *lp<uint32_t>(tab) = sym;
        F.tlog[t] = 0;
        F.tvalid |= 1u << t;
        return 1;
    }
    if (mode == 2) {
        const uint32_t wx = stage_win(L, F.I, p);
        uint32_t tl = 0, nsym = 0, e = 0, used = 0;
        norm_clear(L, max_sym + 1);
        ZF_T0(tn0)
        used = read_ncount(L, F.I.s0 + p - wx, avail, max_sym, max_log, &tl, &nsym, &e);
        ZF_ADD(8, tn0)
        if (uni(e) || uni(used) == 0) {
            *err = ZE_CORRUPT;
            return ~0u;
        }
        ZF_T0(tn1)
        fse_build(L, tab, uni(nsym), uni(tl));
        ZF_ADD(9, tn1)
        F.tlog[t] = uni(tl);
        F.tvalid |= 1u << t;
        return uni(used);
    }
    if (!((F.tvalid >> t) & 1)) {
        *err = ZE_CORRUPT;
        return ~0u;
    }
    return 0;
}

// One compressed block [p, p + n): literals, then the sequence section's
// header and tables -> the block's slot and ops.  Returns 0 or a zstd error.
// Wave-wide.
__device__ __forceinline__ uint32_t block_body(ZLds &L, Frame &F, uint32_t p, uint32_t n)
{
    const uint32_t lane = lane_id();
    if (n >= kZBlockMax)
        return ZE_SRC_WRONG;
    if (F.nblk >= F.blk_cap)
        return ZE_GENERIC;
    const uint64_t g = F.blk0 + F.nblk++;
    uint32_t lused = 0, litn = 0;
    bool huf = false;
    uint32_t e = literals(L, F, g, p, n, &lused, &litn, &huf);
    if (e)
        return e;
    if (huf && !put_op(F, OP_LIT, (uint32_t)g))
        return ZE_GENERIC;
    uint32_t q = p + lused;
    const uint32_t qe = p + n;
    if (q >= qe)
        return ZE_SRC_WRONG;
    const uint32_t wx = stage_win(L, F.I, q);
    auto B = [&](uint32_t i) { return uni(wb(L, wx, F.I, q + i)); };
    uint32_t nseq = B(0);
    if (nseq == 0) {
        if (qe - q != 1)
            return ZE_SRC_WRONG;
        q += 1;
    } else if (nseq == 255) {
        if (q + 3 > qe)
            return ZE_SRC_WRONG;
        nseq = (B(1) | B(2) << 8) + 0x7F00;
        q += 3;
    } else if (nseq > 127) {
        if (q + 2 > qe)
            return ZE_SRC_WRONG;
        nseq = ((nseq - 128) << 8) + B(1);
        q += 2;
    } else {
        q += 1;
    }
    uint32_t tl = 0;
    if (nseq) {
        if (q + 1 > qe)
            return ZE_SRC_WRONG;
        const uint32_t modes = uni(wb(L, wx, F.I, q));
        q++;
        const uint32_t mode[3] = {modes >> 6, (modes >> 4) & 3, (modes >> 2) & 3};
        ZF_T0(t0)
#pragma unroll
        for (uint32_t t = 0; t < 3; t++) {
            uint32_t err = 0;
            const uint32_t u = seq_table(L, F, t, mode[t], q, qe - q, &err);
            if (u == ~0u)
                return err;
            q += u;
        }
        // the three tables -> the block's slot as u16 cells: symbol | next-state
        // rank ns << 6 (nbits and base follow from ns and the table log)
        uint16_t *dst = reinterpret_cast<uint16_t *>(F.slots + g * kZSlot + kSlotFse);
        ZF_T0(tn2)
        wave_lds_sync();
#pragma unroll
        for (uint32_t t = 0; t < 3; t++) {
            const uint32_t size = 1u << F.tlog[t];
            for (uint32_t u = lane; u < size; u += 64) {
                const uint32_t c = *lp<uint32_t>(&L.fse[t][u]);
                const uint32_t ns = ((c >> 16) + size) >> ((c >> 8) & 0xFF);
                dst[kFseOff[t] + u] = (uint16_t)((c & 0xFF) | ns << 6);
            }
        }
        tl = F.tlog[0] | F.tlog[1] << 4 | F.tlog[2] << 8;
        ZF_ADD(10, tn2)
        ZF_ADD(2, t0)
    }
    if (!put_op(F, OP_SEQ, nseq, q, qe > q ? qe - q : 0, F.lo, litn, (uint32_t)g, tl))
        return ZE_GENERIC;
    F.lo += litn;
    return 0;
}

// A block; with the helper wave, its posted Huffman description joined at the
// end: a corrupt description is the block's error (libzstd decodes the
// literals before the sequences), its ops dropped and its jobs cleared, else
// the table log goes into the block's jobs.
__device__ __forceinline__ uint32_t block(ZLds &L, Frame &F, uint32_t p, uint32_t n)
{
    const uint32_t nop0 = F.nop;
    const uint32_t e = block_body(L, F, p, n);
    if (!F.posted)
        return e;
    __syncthreads();   // B: decoded
    F.posted = false;
    const uint32_t lane = lane_id(), hs = F.help->hs, lg = F.help->lg, g = F.help->g;
    if (!hs) {
        if (lane < 4)
            F.jobs[4 * g + lane] = HufJob{0, 0, 0, 0, 0, 0};
        F.nop = nop0;
        F.huf_log = 0;
        return ZE_CORRUPT;
    }
    F.huf_log = lg;
    if (lane < F.post_ns)
        F.jobs[4 * g + lane].tab |= lg << 28;
    return e;
}

// One seek-table entry: every zstd frame in it (ZSTD_decompressDCtx) -> ops.
// Returns 0, or the zstd error at which the op list ends.
__device__ __forceinline__ uint32_t decode_entry(ZLds &L, Frame &F, uint32_t clen)
{
    const uint32_t lane = lane_id();
    uint32_t ip = 0, frames = 0;
    bool summed = false;   // a checksummed frame was decoded: it must be the entry's last
    while (clen - ip >= 5) {
        if (summed)
            return ZE_GENERIC;
        uint32_t wx = stage_win(L, F.I, ip);
        auto B = [&](uint32_t i) { return uni(wb(L, wx, F.I, ip + i)); };
        const uint32_t magic = B(0) | B(1) << 8 | B(2) << 16 | B(3) << 24;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            if (clen - ip < 8)
                return ZE_SRC_WRONG;
            const uint64_t sk = 8 + (uint64_t)(B(4) | B(5) << 8 | B(6) << 16 | B(7) << 24);
            if (sk > clen - ip)
                return ZE_SRC_WRONG;
            ip += (uint32_t)sk;
            continue;
        }
        if (magic != kZMagic)
            return frames ? ZE_SRC_WRONG : ZE_PREFIX;
        frames++;
        const uint32_t n = clen - ip;
        if (n < 9)
            return ZE_SRC_WRONG;
        const uint32_t fhd = B(4);
        const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, csum = (fhd >> 2) & 1,
                       did = fhd & 3;
        const uint32_t dsz = did == 3 ? 4 : did;
        const uint32_t hsize = 5 + !single + dsz + (fcs_flag == 0 ? single : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8);
        if (n < hsize + 3)
            return ZE_SRC_WRONG;
        if (fhd & 0x08)
            return ZE_FRAMEPARAM;
        uint32_t h = 5;
        if (!single) {
            if ((B(h) >> 3) + 10 > 31)
                return ZE_WINDOW;
            h++;
        }
        uint32_t dict = 0;
        for (uint32_t i = 0; i < dsz; i++)
            dict |= B(h + i) << (8 * i);
        h += dsz;
        uint64_t fcs = ~0ull;
        if (fcs_flag == 0 && single)
            fcs = B(h);
        else if (fcs_flag == 1)
            fcs = (B(h) | B(h + 1) << 8) + 256;
        else if (fcs_flag == 2)
            fcs = B(h) | B(h + 1) << 8 | B(h + 2) << 16 | (uint64_t)B(h + 3) << 24;
        else if (fcs_flag == 3)
            fcs = (uint64_t)(B(h) | B(h + 1) << 8 | B(h + 2) << 16 | B(h + 3) << 24) |
                  ((uint64_t)(B(h + 4) | B(h + 5) << 8 | B(h + 6) << 16 | B(h + 7) << 24) << 32);
        if (dict)
            return ZE_DICT_WRONG;
        ip += hsize;
        // frame state
        F.huf_log = 0;
        F.tvalid = 0;
        if (!put_op(F, OP_FBEGIN))
            return ZE_GENERIC;
        for (;;) {
            if (clen - ip < 3)
                return ZE_SRC_WRONG;
            wx = stage_win(L, F.I, ip);
            const uint32_t bh = B(0) | B(1) << 8 | B(2) << 16;
            const uint32_t lastb = bh & 1, type = (bh >> 1) & 3, bsize = bh >> 3;
            const uint32_t csz = type == 1 ? 1 : bsize;
            if (type == 3)
                return ZE_CORRUPT;
            ip += 3;
            if (csz > clen - ip)
                return ZE_SRC_WRONG;
            if (type == 0 || type == 1) {
                // into the scratch (clamped at the capacity); the sequence
                // kernel checks the output room in order
                if (type == 0) {
                    const Span sp = make_span(F.I.base4 + F.I.s0, F.clen);
                    for (uint32_t k = 16 * lane; k < bsize; k += 1024) {
                        const u32x4 v = load16u(sp.r, sp.s0 + ip + k);
                        lit_put(F, F.lo + k, v, bsize - k < 16 ? bsize - k : 16);
                    }
                } else {
                    const uint32_t bv = uni(wb(L, wx, F.I, ip)) * 0x01010101u;
                    for (uint32_t k = 16 * lane; k < bsize; k += 1024)
                        lit_put(F, F.lo + k, (u32x4){bv, bv, bv, bv}, bsize - k < 16 ? bsize - k : 16);
                }
                if (!put_op(F, OP_RUN, F.lo, bsize))
                    return ZE_GENERIC;
                F.lo += bsize;
            } else {
                const uint32_t e = block(L, F, ip, bsize);
                if (e)
                    return e;
            }
            ip += csz;
            if (lastb)
                break;
        }
        uint32_t fl = fcs != ~0ull ? 1u : 0u, want = 0;
        bool trunc = false;
        if (csum) {
            if (clen - ip < 4) {
                trunc = true;
            } else {
                wx = stage_win(L, F.I, ip);
                want = B(0) | B(1) << 8 | B(2) << 16 | B(3) << 24;
                fl |= 2;
                summed = true;
                ip += 4;
            }
        }
        if (!put_op(F, OP_FEND, fl, (uint32_t)fcs, (uint32_t)(fcs >> 32), want))
            return ZE_GENERIC;
        if (trunc)
            return ZE_CHECKSUM;
    }
    if (clen != ip)
        return ZE_SRC_WRONG;
    return 0;
}


// ---- kernels -------------------------------------------------------------------------------

// item bound per frame (lane per frame): 2 items per sequence + padding + 4 per
// block; and the frame's block count (its table slots and op list)
__global__ __launch_bounds__(256) void zstd_plan_kernel(const FrameDesc *__restrict__ desc, uint32_t n,
                                                        const uint8_t *__restrict__ comp,
                                                        uint32_t *__restrict__ bound,
                                                        uint32_t *__restrict__ bblk,
                                                        unsigned long long *__restrict__ extent)
{
    const uint32_t f = blockIdx.x * 256 + threadIdx.x;
    FrameDesc d = {0, 0, 0, 0};
    if (f < n)
        d = desc[f];
    // the output extent max(d_off + d_size), a wave at a time (the scan then
    // reads no descriptors)
    // (and the largest frame, extent[2]: whether the one-frame route's
    // execute needs a wave kernel beside its workgroups)
    const uint64_t wx = wave_max64(f < n ? d.d_off + d.d_size : 0ull);
    const uint64_t wd = wave_max64(f < n ? d.d_size : 0ull);
    if ((threadIdx.x & 63) == 0 && wx)
        atomicMax(extent, (unsigned long long)wx);
    if ((threadIdx.x & 63) == 0 && wd)
        atomicMax(extent + 2, (unsigned long long)wd);
    if (f >= n)
        return;
    const Span sp = make_span(comp + d.c_off, d.c_size);
    auto B = [&](uint32_t p) -> uint32_t {
        return p < d.c_size ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(sp.r, sp.s0 + p, 0, 0) : 0u;
    };
    const uint32_t clen = d.c_size;
    uint64_t items = 8;
    uint32_t ip = 0, blocks = 0;
    while (clen - ip >= 9 && items < (1u << 30)) {
        const uint32_t magic = B(ip) | B(ip + 1) << 8 | B(ip + 2) << 16 | B(ip + 3) << 24;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            ip += 8 + (B(ip + 4) | B(ip + 5) << 8 | B(ip + 6) << 16 | B(ip + 7) << 24);
            continue;
        }
        if (magic != kZMagic)
            break;
        const uint32_t fhd = B(ip + 4);
        const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, did = fhd & 3;
        ip += 5 + !single + (did == 3 ? 4 : did) + (fcs_flag == 0 ? single : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8);
        for (;;) {
            if (clen < ip + 3)
                break;
            const uint32_t bh = B(ip) | B(ip + 1) << 8 | B(ip + 2) << 16;
            const uint32_t type = (bh >> 1) & 3, bsize = bh >> 3;
            ip += 3;
            items += 4;
            blocks++;
            if (type == 2 && bsize >= 3) {
                const uint32_t b0 = B(ip), lt = b0 & 3, sf = (b0 >> 2) & 3;
                uint32_t sec;
                if (lt <= 1) {
                    const uint32_t lh = sf == 1 ? 2 : sf == 3 ? 3 : 1;
                    const uint32_t sz = sf == 1 ? (b0 | B(ip + 1) << 8) >> 4
                                      : sf == 3 ? (b0 | B(ip + 1) << 8 | B(ip + 2) << 16) >> 4
                                                : b0 >> 3;
                    sec = lt == 0 ? lh + sz : lh + 1;
                } else {
                    const uint32_t lhc = b0 | B(ip + 1) << 8 | B(ip + 2) << 16 | B(ip + 3) << 24;
                    sec = sf <= 1 ? 3 + ((lhc >> 14) & 0x3FF) : sf == 2 ? 4 + (lhc >> 18)
                                                                      : 5 + (lhc >> 22) + (B(ip + 4) << 10);
                }
                if (sec < bsize) {
                    const uint32_t q = ip + sec, s0 = B(q);
                    const uint32_t nseq = s0 < 128 ? s0 : s0 < 255 ? ((s0 - 128) << 8) + B(q + 1)
                                                                   : (B(q + 1) | B(q + 2) << 8) + 0x7F00;
                    items += 2ull * nseq + (2ull * nseq + 62) / 63;
                }
            }
            ip += type == 1 ? 1 : bsize;
            if ((bh & 1) || ip > clen)
                break;
        }
        if (ip > clen)
            break;
        if ((fhd >> 2) & 1)
            ip += 4;
    }
    bound[f] = (uint32_t)((items + 3) & ~3ull);
    bblk[f] = blocks;
}

// exclusive scans of the per-frame item bounds and block counts ->
// rec_base[0..n], blk_base[0..n]; item total, output extent max(d_off +
// d_size) and block total into total[0..2] (device memory, copied to the host
// by the launcher; one workgroup)
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(1024) void zstd_scan_kernel(const uint32_t *__restrict__ bound,
                                                         const uint32_t *__restrict__ bblk, uint32_t n,
                                                         uint64_t *__restrict__ rec_base,
                                                         uint64_t *__restrict__ blk_base,
                                                         uint64_t *__restrict__ total)
{
    // tiles of 4096 frames, four per thread, loaded 16 bytes at a time
    // (coalesced) and scanned a wave at a time; a thread per frame chunk with
    // a dependent load per element cost ~0.3 ms at 65,536 frames
    __shared__ uint64_t wsum[16], wsumb[16];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint64_t carry = 0, carryb = 0;
    auto load4 = [&](const uint32_t *a, uint32_t x) -> u32x4 {
        if (x + 4 <= n)
            return *reinterpret_cast<const u32x4 *>(a + x);
        u32x4 v = {0, 0, 0, 0};
        for (uint32_t q = 0; q < 4; q++)
            if (x + q < n)
                v[q] = a[x + q];
        return v;
    };
    const uint32_t x0 = 4 * t;
    u32x4 a = load4(bound, x0), c = load4(bblk, x0);
    for (uint32_t b = 0; b < n; b += 4096) {
        const uint32_t x = b + x0;
        const u32x4 ca = a, cc = c;
        if (b + 4096 < n) {   // the next tile's loads in flight during this one's scan
            a = load4(bound, x + 4096);
            c = load4(bblk, x + 4096);
        }
        const uint64_t s = (uint64_t)ca.x + ca.y + ca.z + ca.w;
        const uint64_t sb = (uint64_t)cc.x + cc.y + cc.z + cc.w;
        uint64_t is = s, isb = sb;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint64_t v = __shfl_up(is, d, 64), vb = __shfl_up(isb, d, 64);
            if (lane >= d) {
                is += v;
                isb += vb;
            }
        }
        if (lane == 63) {
            wsum[w] = is;
            wsumb[w] = isb;
        }
        __syncthreads();
        uint64_t pre = carry, preb = carryb, tot = carry, totb = carryb;
        for (uint32_t k = 0; k < 16; k++) {
            pre += k < w ? wsum[k] : 0;
            preb += k < w ? wsumb[k] : 0;
            tot += wsum[k];
            totb += wsumb[k];
        }
        __syncthreads();   // wsum free for the next tile
        uint64_t r = pre + is - s, rb = preb + isb - sb;
        if (x < n) {
            const uint64_t r1 = r + ca.x, r2 = r1 + ca.y, r3 = r2 + ca.z;
            const uint64_t q1 = rb + cc.x, q2 = q1 + cc.y, q3 = q2 + cc.z;
            if (x + 4 <= n) {
                *reinterpret_cast<u64x2 *>(rec_base + x) = (u64x2){r, r1};
                *reinterpret_cast<u64x2 *>(rec_base + x + 2) = (u64x2){r2, r3};
                *reinterpret_cast<u64x2 *>(blk_base + x) = (u64x2){rb, q1};
                *reinterpret_cast<u64x2 *>(blk_base + x + 2) = (u64x2){q2, q3};
            } else {
                const uint64_t rr[4] = {r, r1, r2, r3}, qq[4] = {rb, q1, q2, q3};
                for (uint32_t q = 0; x + q < n; q++) {
                    rec_base[x + q] = rr[q];
                    blk_base[x + q] = qq[q];
                }
            }
        }
        carry = tot;
        carryb = totb;
    }
    if (t == 0) {
        rec_base[n] = carry;
        blk_base[n] = carryb;
        total[0] = carry;
        total[2] = carryb;
    }
}

// Frame kernel: one wave per seek-table entry.  Headers, literal sections
// (raw / RLE literals straight into the scratch), Huffman and FSE tables
// (built in LDS, stored to the block's slot), Huffman stream jobs and the op
// list the sequence kernel replays.
// HELP: one frame per workgroup, wave 1 the helper wave (HelpBox above);
// else kZW frames per workgroup, one per wave.
template <bool HELP>
__global__ __launch_bounds__(64 * kZW) __attribute__((amdgpu_waves_per_eu(4))) void zstd_frame_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    uint8_t *__restrict__ lit, uint64_t lit_cap, const uint64_t *__restrict__ rec_base,
    uint64_t capacity, const uint64_t *__restrict__ blk_base, uint8_t *__restrict__ ops,
    uint8_t *__restrict__ slots, uint8_t *__restrict__ jobs, uint32_t f0)
{
    static_assert(kZW >= 2, "the helper wave needs a second ZLds");
    __shared__ ZLds lds[kZW];
    __shared__ HelpBox box;
    ZF_T0(tk)
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t f = HELP ? uni(f0 + blockIdx.x) : uni(f0 + blockIdx.x * kZW + w);   // frames [f0, n)
    if (f >= n)
        return;   // (HELP: the whole workgroup)
    ZLds &L = lds[w];
    const FrameDesc d = desc[f];
    Frame F;
    if (HELP && w == 1) {
        // helper: the frame's In, then the posted descriptions until done
        const uintptr_t fa = reinterpret_cast<uintptr_t>(comp + d.c_off);
        F.I.base4 = reinterpret_cast<const uint8_t *>(fa & ~(uintptr_t)3);
        F.I.s0 = (uint32_t)(fa & 3);
        F.I.amax = d.c_size ? (F.I.s0 + d.c_size - 1) & ~3u : 0;
        for (;;) {
            __syncthreads();   // A
            if (uni(box.kind) == 0)
                break;
            const uint32_t q = uni(box.q), qn = uni(box.qn), g = uni(box.g);
            const uint32_t wx = stage_win(L, F.I, q);
            uint32_t lg = 0;
            ZF_T0(t0)
            const uint32_t hs = huf_read(L, F.I, wx, q, qn, &lg, reinterpret_cast<uint16_t *>(slots + (uint64_t)g * kZSlot));
            ZF_ADD(1, t0)
            if (lane_id() == 0) {
                box.hs = hs;
                box.lg = lg;
            }
            __syncthreads();   // B
        }
        return;
    }
    if (HELP)
        F.help = &box;
    const uintptr_t fa = reinterpret_cast<uintptr_t>(comp + d.c_off);
    F.I.base4 = reinterpret_cast<const uint8_t *>(fa & ~(uintptr_t)3);
    F.I.s0 = (uint32_t)(fa & 3);
    F.I.amax = d.c_size ? (F.I.s0 + d.c_size - 1) & ~3u : 0;
    F.c_abs = d.c_off;
    F.d_abs = d.d_off;
    F.lit = lit + d.d_off;
    F.clen = d.c_size;
    F.cap = d.d_size;
    F.lo = 0;
    F.huf_log = 0;
    F.tvalid = 0;
    F.tlog[0] = F.tlog[1] = F.tlog[2] = 0;
    const uint64_t ob = op_base(blk_base, f);
    F.ops = reinterpret_cast<ZOp *>(ops) + ob;
    F.nop = 0;
    F.op_cap = (uint32_t)(op_base(blk_base, f + 1) - ob);
    F.blk0 = blk_base[f];
    F.nblk = 0;
    F.blk_cap = (uint32_t)(blk_base[f + 1] - F.blk0);
    F.slots = slots;
    F.jobs = reinterpret_cast<HufJob *>(jobs);
    // this frame's Huffman jobs zeroed (a block without Huffman literals, or
    // one the frame never reaches, has no streams) -- no memset of the whole
    // job array per launch; ordered before the jobs literals() writes
    for (uint32_t i = lane_id(); i < 4 * F.blk_cap; i += 64)
        F.jobs[4 * F.blk0 + i] = HufJob{0, 0, 0, 0, 0, 0};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    uint32_t e;
    // scratch sized by the plan: a frame that would not fit is refused, never
    // written out of bounds
    if (rec_base[f + 1] > capacity || d.c_size >= 0x7FFFFF00u ||
        d.d_off + (uint64_t)d.d_size + 16 > lit_cap)
        e = ZE_GENERIC;
    else
        e = decode_entry(L, F, d.c_size);
    if (e)
        put_op(F, OP_ERR, (uint32_t)zerr(e));
    else
        put_op(F, OP_DONE);
    if (HELP) {
        if (lane_id() == 0)
            box.kind = 0;
        __syncthreads();   // A: done
    }
    ZF_ADD(0, tk)
#ifdef ZSK_TUNING
    if (lane_id() == 0)
        atomicAdd(&g_zftime[4], 1ull);
#endif
}

// ---- backward bitstreams, lane per stream -------------------------------------------
// Bits of one stream of comp, read from its end: C holds stream bits
// [pos, pos + nb) (coordinates in bits from the stream's 16-aligned chunk
// base x0; bits below the stream's first byte read as 0).  The lane's stream
// bytes pass through a ring of kRS 16-byte slots in LDS (dword k of slot s of
// lane l at ring base + s * 1024 + k * 256 + 4 * l: a wave's ring reads hit 64
// different banks whatever dword each lane reads): br_step, once per decode step at a fixed
// place in the loop, commits the chunk loaded one step earlier and issues the
// next load — unconditionally, re-fetching the last chunk when the ring is
// full — so no load result is ever waited for in the step that issued it and
// no load sits in a divergent branch.  br_fill refills C from the ring.  The
// buffer resource is wave-uniform (a span of comp covering the wave's
// streams); x0 is the lane's offset in it.
constexpr int32_t kRS = 4;

struct BRd {
    __amdgpu_buffer_rsrc_t r;
    uint64_t C;
    u32x4 P, P2;     // chunks `pend`, `pend2`, committed to the ring at the next step
    uint32_t x0;
    uint32_t ring;   // LDS address of this lane's dword 0 of slot 0
    int32_t nb, pos, xs;
    int32_t pq;      // next chunk to fetch (decreasing; < 0 reads zeros)
    int32_t pend, pend2;
};

constexpr uint32_t kOOR = 0x80000000u;   // out-of-range buffer offset: loads 0
constexpr uint64_t kMaxSpan = 0x7FFFFF00ull;   // largest span one resource covers

__device__ __forceinline__ u32x4 chunk16(const BRd &b, int32_t q)
{
    return __builtin_bit_cast(
        u32x4, __builtin_amdgcn_raw_buffer_load_b128(b.r, q >= 0 ? b.x0 + 16u * (uint32_t)q : kOOR, 0, 0));
}

__device__ __forceinline__ uint32_t slot_addr(const BRd &b, int32_t q)
{
    return b.ring + (uint32_t)(q & (kRS - 1)) * 1024u;
}

__device__ __forceinline__ void slot_put(const BRd &b, int32_t q, u32x4 v)
{
    const uint32_t a = slot_addr(b, q);
    *la<uint32_t>(a) = v.x;
    *la<uint32_t>(a + 256) = v.y;
    *la<uint32_t>(a + 512) = v.z;
    *la<uint32_t>(a + 768) = v.w;
}

// mask of the bits of the dword at bit coordinate p that lie at or above xs
__device__ __forceinline__ uint32_t above(int32_t xs, int32_t p)
{
    const int32_t sh = xs - p;
    return sh <= 0 ? ~0u : sh >= 32 ? 0u : ~0u << sh;
}

// A span [base, base + len) of comp as a buffer resource (len < 2^31 - 256;
// rounded up to whole dwords: the hardware range-checks each dword).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t span_rsrc(const uint8_t *comp, uint64_t base, uint64_t len)
{
    return __builtin_amdgcn_make_buffer_rsrc((void *)(comp + base), 0, (int)(uint32_t)((len + 3) & ~3ull),
                                             kRsrcDw3);
}

// The stream at offset x (len >= 1 bytes) of resource r, ring at LDS address
// ring.  False when its last byte (the end mark) is 0.
__device__ __forceinline__ bool br_init(BRd &b, __amdgpu_buffer_rsrc_t r, uint32_t x, uint32_t len, uint32_t ring,
                                        bool d2 = false)
{
    b.r = r;
    b.ring = ring;
    b.x0 = x & ~15u;
    const uint32_t rel = (x & 15u) + len;   // bytes from x0 to the stream's end
    b.xs = 8 * (int32_t)(x & 15u);
    const uint32_t last = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, b.x0 + rel - 1, 0, 0);
    const int32_t xm = 8 * (int32_t)(rel - 1) + (last ? 31 - __builtin_clz(last) : 0);
    const int32_t D = xm >> 5, i = D & 3, q = D >> 2;
    u32x4 c[kRS - 1];
#pragma unroll
    for (int k = 0; k < kRS - 1; k++)
        c[k] = chunk16(b, q - k);
#pragma unroll
    for (int k = 0; k < kRS - 1; k++)
        slot_put(b, q - k, c[k]);
    b.pq = q - (kRS - 1);
    b.P = chunk16(b, b.pq);
    b.P2 = b.P;
    b.pend = b.pend2 = b.pq;
    b.pq--;
    const uint32_t top = i == 3 ? c[0].w : i == 2 ? c[0].z : i == 1 ? c[0].y : c[0].x;
    b.pos = 32 * D;
    b.C = top & ((1u << (xm & 31)) - 1) & above(b.xs, b.pos);
    b.nb = xm & 31;
    if (d2) {   // a second chunk in flight (br_step<1, 2>), room permitting
        const int32_t qcur = (b.pos - 32) >> 7;
        const bool room = b.pq >= qcur - (kRS - 1);
        const int32_t t = room ? b.pq : b.pq + 1;
        b.P2 = chunk16(b, t);
        b.pend2 = t;
        b.pq = room ? b.pq - 1 : b.pq;
    }
    return last != 0;
}

// Once per decode step: commit the pending chunk(s), fetch the next one(s)
// (F = 1 or 2 chunks per step).  D = 2 (with F = 1): two chunks in flight,
// each committed two steps after its load, so the load's wait never waits
// on the literal store of the step just before it (vmcnt retires in issue
// order): a store has two steps to land instead of one.  A room check at
// issue suffices: the slot it fills held a chunk above the one then in use.
template <int F = 1, int D = 1>
__device__ __forceinline__ void br_step(BRd &b)
{
    if (D == 2) {
        slot_put(b, b.pend, b.P);
        b.P = b.P2;
        b.pend = b.pend2;
        const int32_t qcur = (b.pos - 32) >> 7;
        const bool room = b.pq >= qcur - (kRS - 1);
        const int32_t t = room ? b.pq : b.pq + 1;
        b.P2 = chunk16(b, t);
        b.pend2 = t;
        b.pq = room ? b.pq - 1 : b.pq;
        return;
    }
    slot_put(b, b.pend, b.P);
    if (F == 2)
        slot_put(b, b.pend2, b.P2);
    const int32_t qcur = (b.pos - 32) >> 7;   // chunk of the next dword to absorb
    bool room = b.pq >= qcur - (kRS - 1);
    int32_t t = room ? b.pq : b.pq + 1;
    b.P = chunk16(b, t);
    b.pend = t;
    b.pq = room ? b.pq - 1 : b.pq;
    if (F == 2) {
        room = b.pq >= qcur - (kRS - 1);
        t = room ? b.pq : b.pq + 1;
        b.P2 = chunk16(b, t);
        b.pend2 = t;
        b.pq = room ? b.pq - 1 : b.pq;
    }
}

// refill C to >= 32 bits when below (branch-free)
__device__ __forceinline__ void br_fill(BRd &b)
{
    const int32_t p2 = b.pos - 32, dw = p2 >> 5;
    const uint32_t v = *la<uint32_t>(slot_addr(b, dw >> 2) + 256u * (uint32_t)(dw & 3)) & above(b.xs, p2);
    const bool need = b.nb < 32;
    b.C = need ? (b.C << 32) | v : b.C;
    b.nb = need ? b.nb + 32 : b.nb;
    b.pos = need ? p2 : b.pos;
}

// stream bits not consumed yet (< 0 once read past the start)
__device__ __forceinline__ int32_t br_left(const BRd &b)
{
    return b.pos + b.nb - b.xs;
}

// ---- Huffman literals: one lane per stream -------------------------------------------
// 16 blocks (64 streams) per wave; their tables packed into LDS when they fit
// (else read from the slots).  Cells are nbits | symbol << 8.  In the main
// loop a lane refills its bit container every G symbols (G * lg <= 32) and
// decodes those G symbols from a 32-bit MSB-first window w of the
// container's top bits: index = w >> (32 - lg), consume = w <<= cell (the
// shift takes the cell's low 5 bits, nbits).  16 decoded bytes are stored at
// a time, aligned.
constexpr uint32_t kHufLdsCells = 2048;

template <int G, int F, int DIAG, int B = 4, typename Tab>
__device__ __forceinline__ void huf_stream(BRd &b, Tab T, uint32_t lg, uint8_t *out, uint64_t dst, uint32_t cnt,
                                           uint32_t lim)
{
    const uint32_t mask = (1u << lg) - 1, sh = 32 - lg;
    auto one = [&]() -> uint32_t {
        const uint32_t e = T((uint32_t)(b.C >> (uint32_t)(b.nb - (int32_t)lg)) & mask);
        b.nb -= (int32_t)(e & 0xFF);
        return e >> 8;
    };
    uint32_t i = 0;
    // head (< 16 symbols, <= 180 bits): the ring holds kRS - 1 chunks after br_init
    while (i < cnt && ((dst + i) & 15)) {
        br_fill(b);
        const uint32_t s = one();
        if (i < lim)
            out[i] = (uint8_t)s;
        i++;
    }
    // 16 symbols per step
    auto step16 = [&]() -> u32x4 {
        if (!(DIAG & 2))
            br_step<F, F == 1 ? 2 : 1>(b);
        u32x4 acc = {0, 0, 0, 0};
        uint32_t w = 0, used = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            if (k % G == 0) {
                b.nb -= (int32_t)used;
                br_fill(b);
                w = (uint32_t)(b.C >> (uint32_t)(b.nb - 32));
                used = 0;
            }
            const uint32_t e = (DIAG & 4) ? (w >> 26) << 8 | 6u : T(w >> sh);
            w <<= (e & 31);   // nbits
            used += e & 0xFF;
            if ((k & 3) == 0)
                acc[k >> 2] = e >> 8;
            else
                acc[k >> 2] |= (e >> 8) << (8 * (k & 3));
        }
        b.nb -= (int32_t)used;
        return acc;
    };
    auto put16 = [&](uint32_t at, const u32x4 &v) {
        if (!(DIAG & 1))
            *reinterpret_cast<u32x4 *>(out + at) = v;
    };
    // to a 128-byte boundary of the output, a step at a time
    while (i + 16 <= lim && ((dst + i) & (16 * B - 1))) {
        const u32x4 v = step16();
        put16(i, v);
        i += 16;
    }
    // then 4 steps per iteration and their 64 bytes stored back to back: a
    // line arrives in two halves, where 16-byte stores a step apart left
    // partial lines in L2 to be evicted (and merged in HBM) under this
    // kernel's write load (5.2 -> 3.9 ms; no stores at all: 1.9 ms; 8 steps
    // need more than the 128 VGPRs four waves per SIMD leave: spills).
    // Round 3, config 5 (6-bit codes, kernels serialized): 2.90 ms; without
    // the stores 1.85, also without the ring refills 1.33, also without the
    // lookups 0.58.  Neither 128-byte bursts (three waves per SIMD) nor
    // keeping the second step's chunk wait clear of the stores just issued
    // (the loop head's wait-count merge made it wait for them) moved it;
    // nontemporal stores doubled it (6.03 ms: L2 write-combining is doing
    // real work here).
    while (i + 16 * B <= lim) {
        u32x4 v[B];
#pragma unroll
        for (int k = 0; k < B; k++)
            v[k] = step16();
#pragma unroll
        for (int k = 0; k < B; k++)
            put16(i + 16 * k, v[k]);
        i += 16 * B;
    }
    while (i + 16 <= lim) {
        const u32x4 v = step16();
        put16(i, v);
        i += 16;
    }
    while (i < cnt) {
        br_step<F, F == 1 ? 2 : 1>(b);
        br_fill(b);
        const uint32_t s = one();
        if (i < lim)
            out[i] = (uint8_t)s;
        i++;
    }
}

// ---- libzstd's X2 decoder on a stream X1 rejects --------------------------------------
// On a valid stream X1 and X2 decode the same bytes; they differ only on
// streams X1 rejects (HUF_decodeLastSymbolX2: at a stream's last output byte a
// two-symbol cell consumes both codes' bits, clamped at the stream's start,
// and a read with no bits left looks at the bit container's top bits).  So a
// lane keeps the fast X1 walk and, for an X2 stream it rejected, re-walks it
// here in X2 cells (tests/test_zstd_oracle.py pins the rule the oracle and
// this walk share against libzstd 1.4.9).  The re-walk reads one cell at a
// time; only streams that failed X1 -- corrupt ones -- pay for it.

// the stream at byte x of resource r, read backward through a 64-bit window
// (two dwords, reloaded when a read leaves it: one load per ~4 cells)
struct X2Bits {
    __amdgpu_buffer_rsrc_t r;
    uint32_t x;
    uint32_t wlo;   // absolute bit of the window's bit 0 (a multiple of 32)
    uint64_t w;
    // bits [q - n, q) (bit q - 1 most significant), bits below the stream's
    // first byte 0; n <= 12
    __device__ uint32_t get(int32_t q, uint32_t n)
    {
        if (q <= 0)
            return 0;
        const int32_t lo = q - (int32_t)n, l0 = lo > 0 ? lo : 0;
        const uint32_t a = 8 * x + (uint32_t)l0, e = 8 * x + (uint32_t)q;
        if (a < wlo || e > wlo + 64) {
            const uint32_t d = a >> 5;
            w = (uint64_t)(uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, 4 * d, 0, 0) |
                (uint64_t)(uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, 4 * d + 4, 0, 0) << 32;
            wlo = 32 * d;
        }
        const uint32_t bits = (uint32_t)(w >> (a - wlo)) & ((1u << (uint32_t)(q - l0)) - 1);
        return lo < 0 ? bits << (uint32_t)(-lo) : bits;
    }
};

// X2 result of the stream (len bytes at x, cnt symbols, cells tab of table
// log lg): bit 0 ok; bit 16: the last byte is bits 8..15 (a read with no
// bits left), else the X1 walk's bytes stand.
__device__ __attribute__((noinline)) uint32_t x2_rescue(__amdgpu_buffer_rsrc_t r, uint32_t x, uint32_t len,
                                                        uint32_t cnt, const uint16_t *tab, uint32_t lg)
{
    const uint32_t last = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, x + len - 1, 0, 0);
    if (!last || !cnt)
        return 0;
    int32_t rr = 8 * (int32_t)(len - 1) + (31 - __builtin_clz(last));   // bits below the end mark
    X2Bits B{r, x, 0xFFFFFFC0u, 0};
    auto Z = [&](int32_t q) -> uint32_t { return tab[B.get(q, lg)]; };
    uint32_t p = 0;
    while (p + 2 <= cnt) {   // HUF_decodeStreamX2's cells before the last byte
        if (rr <= 0)
            return 0;
        const uint32_t nb1 = Z(rr) & 0xFF, nb2 = Z(rr - (int32_t)nb1) & 0xFF;
        const bool two = nb1 + nb2 <= 12;
        p += two ? 2 : 1;
        rr -= (int32_t)(two ? nb1 + nb2 : nb1);
    }
    if (p == cnt)
        return rr == 0 ? 1u : 0u;
    if (rr > 0) {   // HUF_decodeLastSymbolX2
        const uint32_t nb1 = Z(rr) & 0xFF, nb2 = Z(rr - (int32_t)nb1) & 0xFF;
        if (nb1 + nb2 <= 12)
            return rr <= (int32_t)(nb1 + nb2) ? 1u : 0u;
        return rr == (int32_t)nb1 ? 1u : 0u;
    }
    if (rr < 0)
        return 0;
    // no bits left: the cell at the container's top 12 bits (the stream's
    // first 8 bytes, zero past its end); only a two-symbol cell leaves it
    // consumed exactly
    uint64_t c = 0;
    for (uint32_t i = 0; i < 8 && i < len; i++)
        c |= (uint64_t)(uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, x + i, 0, 0) << (8 * i);
    const uint32_t v = (uint32_t)(c >> 52);
    const uint32_t g1 = tab[v >> (12 - lg)], nb1 = g1 & 0xFF;
    const uint32_t nb2 = tab[((v << nb1) & 0xFFF) >> (12 - lg)] & 0xFF;
    if (nb1 + nb2 > 12)
        return 0;
    return 1u | 0x10000u | (g1 >> 8) << 8;
}

__device__ unsigned int g_hdiag[32];   // diagnostic builds: waves per lgmax, LDS / global path

// B: steps per store burst (4 = 64 bytes)
template <int DIAG, int B = 4>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void zstd_huf_kernel(const uint8_t *__restrict__ jobs, uint32_t nj,
                                                      const uint8_t *__restrict__ comp,
                                                      const uint8_t *__restrict__ slots,
                                                      uint8_t *__restrict__ lit, uint8_t *__restrict__ hbad)
{
    __shared__ __attribute__((aligned(16))) uint16_t tabs[kHufLdsCells];
    __shared__ __attribute__((aligned(16))) uint8_t rings[kRS * 1024];
    const uint32_t lane = threadIdx.x;
    const uint32_t j = blockIdx.x * 64 + lane;
    HufJob J = {0, 0, 0, 0, 0, 0};
    if (j < nj)
        J = reinterpret_cast<const HufJob *>(jobs)[j];
    const bool act = J.len != 0;
    const uint32_t jlg = J.tab >> 28, jslot = J.tab & kHufSlotMask, jx2 = (J.tab >> 27) & 1;
    const uint32_t lgmax = lane_val(wave_incl_max(act ? jlg : 0u), 63);
    // cells of each block's table (stream 0's lane), packed in block order
    const uint32_t cells = (lane & 3) == 0 && act ? ((1u << jlg) < 8 ? 8u : 1u << jlg) : 0u;
    const uint32_t incl = wave_incl_add(cells);
    const uint32_t first = (uint32_t)__shfl((int)(incl - cells), (int)(lane & ~3u), 64);
    const bool in_lds = lane_val(incl, 63) <= kHufLdsCells;
    // the longest streams (a literal-only 64 KiB block: 16 Ki symbols each,
    // ~2.5x the usual) bound the kernel: their waves issue first
    if (lane_val(wave_incl_max(act ? J.cnt : 0u), 63) > 12000)
        __builtin_amdgcn_s_setprio(3);
    if (in_lds) {
        for (uint32_t b = 0; b < 16; b++) {
            const uint32_t nc = lane_val(cells, 4 * b);
            if (!nc)
                continue;
            const uint32_t c0 = lane_val(incl, 4 * b) - nc;
            const uint8_t *src = slots + (uint64_t)lane_val(jslot, 4 * b) * kZSlot;
            for (uint32_t c = lane; c < nc / 8; c += 64)
                *lp<u32x4>(&tabs[c0 + 8 * c]) = *reinterpret_cast<const u32x4 *>(src + 16 * c);
        }
        __syncthreads();
    }
    // one resource over the wave's streams (else lane by lane, each its own)
    const uint64_t lo = uni64(wave_min64(act ? J.src : ~0ull)) & ~15ull;
    const uint64_t hi = uni64(wave_max64(act ? J.src + J.len : 0ull));
    if (DIAG && lane == 0) {
        atomicAdd(&g_hdiag[lgmax & 15], 1u);
        atomicAdd(&g_hdiag[16 + (in_lds ? 1 : 0)], 1u);
    }
    if (j >= nj)
        return;
    bool bad = false;
    auto run = [&](__amdgpu_buffer_rsrc_t r, uint64_t base) {
        BRd b;
        bad = !br_init(b, r, (uint32_t)(J.src - base), J.len, (uint32_t)(uintptr_t)lp<uint8_t>(rings) + 4 * lane,
                       in_lds && lgmax <= 8);   // huf_stream<4, 1>: two chunks in flight
        uint8_t *out = lit + J.dst;
        if (in_lds) {
            const uint32_t tb = (uint32_t)(uintptr_t)lp<uint16_t>(&tabs[first]);
            auto T = [&](uint32_t i) -> uint32_t { return *la<uint16_t>(tb + 2 * i); };
            if (lgmax <= 8)
                huf_stream<4, 1, DIAG, B>(b, T, jlg, out, J.dst, J.cnt, J.lim);
            else
                huf_stream<2, 2, DIAG, B>(b, T, jlg, out, J.dst, J.cnt, J.lim);
        } else {
            const uint16_t *gt = reinterpret_cast<const uint16_t *>(slots + (uint64_t)jslot * kZSlot);
            auto T = [&](uint32_t i) -> uint32_t { return gt[i]; };
            huf_stream<2, 2, DIAG, B>(b, T, jlg, out, J.dst, J.cnt, J.lim);
        }
        bad = bad || br_left(b) != 0;
    };
    if (hi > lo && hi - lo < kMaxSpan) {
        if (act)
            run(span_rsrc(comp, lo, hi - lo), lo);
    } else {
        for (uint64_t m = __ballot(act); m; m &= m - 1) {
            const int l = __builtin_ctzll(m);
            const uint64_t s0 = uni64(__shfl(J.src, l, 64)) & ~15ull;
            const uint64_t s1 = uni64(__shfl(J.src + J.len, l, 64));
            if ((int)lane == l)
                run(span_rsrc(comp, s0, s1 - s0), s0);
        }
    }
    if (bad && jx2) {   // libzstd's X2 decoder may still accept the stream
        const uint16_t *tp =
            in_lds ? &tabs[first] : reinterpret_cast<const uint16_t *>(slots + (uint64_t)jslot * kZSlot);
        const uint64_t s0 = J.src & ~15ull;
        const uint32_t x = x2_rescue(span_rsrc(comp, s0, J.src + J.len - s0), (uint32_t)(J.src - s0), J.len, J.cnt,
                                     tp, jlg);
        bad = !(x & 1);
        if ((x & 0x10000) && J.cnt - 1 < J.lim)
            lit[J.dst + J.cnt - 1] = (uint8_t)(x >> 8);
    }
    hbad[j] = bad ? 1 : 0;
}

// ---- Huffman literals, the one-frame route: a workgroup per stream ----------------------
// A lone frame's four streams on four lanes were a 366 us serial chain (~130
// cycles a symbol: an LDS lookup per symbol).  Here 256 threads split the
// stream's bits into chunks and decode them at once.  A symbol boundary at a
// chunk's top is unknown until the chunks above are decoded, but it lies in
// the top lg bits of the chunk (no code is longer than lg): so each thread
// decodes its chunk from every one of those lg entry bits (lockstep, ILP over
// the entries), recording for each entry where the walk leaves the chunk and
// how many symbols it took.  One thread then follows the true entries from
// the stream's end mark chunk by chunk (the exit of one chunk is the next
// one's entry), giving each chunk its entry and output base; a second pass
// decodes each chunk from its true entry into an LDS copy of the output,
// written out in 16-byte stores.  Identical bytes to the serial walk (the
// same cells and bit reads, bits below the stream read as 0): a stream is
// valid iff the followed walk makes exactly cnt symbols and ends at bit 0.
// Anything else -- a stream the walk rejects (X2 rescue), too long for the
// stage, an empty end mark -- is decoded by thread 0 exactly as
// zstd_huf_kernel's lane does.
constexpr uint32_t kHufOneT = 256;
constexpr uint32_t kHufOneStage = 65536;    // stream bytes staged (else the serial walk)
constexpr uint32_t kHufOneOut = 32768;      // symbols staged (else the serial walk)
constexpr uint32_t kHufOneMaxLg = 12;

// its LDS (a struct: the one-frame decode kernel below shares it with the
// sequence replay's, as a union)
struct HufOneLds {
    __attribute__((aligned(16))) uint8_t sst[16 + kHufOneStage + 32];
    __attribute__((aligned(16))) uint8_t obuf[kHufOneOut + 16];
    __attribute__((aligned(16))) uint16_t tab[1u << kHufOneMaxLg];
    uint32_t cand[kHufOneT * kHufOneMaxLg];   // exit offset | symbols << 8, per chunk and entry
    uint32_t ent[kHufOneT];                   // true entry | output base << 4
    uint32_t verdict;
    __attribute__((aligned(16))) uint8_t rings[kRS * 1024];   // the serial walk's ring
};

// job j by the workgroup's kHufOneT threads (t = thread index)
__device__ __forceinline__ void huf_one_body(HufOneLds &H, uint32_t j, uint32_t t, const uint8_t *__restrict__ jobs,
                                             const uint8_t *__restrict__ comp, const uint8_t *__restrict__ slots,
                                             uint8_t *__restrict__ lit, uint8_t *__restrict__ hbad)
{
    auto &sst = H.sst;
    auto &obuf = H.obuf;
    auto &tab = H.tab;
    auto &cand = H.cand;
    auto &ent = H.ent;
    auto &verdict = H.verdict;
    auto &rings = H.rings;
    const HufJob J = reinterpret_cast<const HufJob *>(jobs)[j];
    if (J.len == 0) {
        if (t == 0)
            hbad[j] = 0;
        return;
    }
    const uint32_t lg = J.tab >> 28, jslot = J.tab & kHufSlotMask, jx2 = (J.tab >> 27) & 1;
    const uint16_t *gt = reinterpret_cast<const uint16_t *>(slots + (uint64_t)jslot * kZSlot);
    const uint64_t s0 = J.src & ~15ull;
    const __amdgpu_buffer_rsrc_t r = span_rsrc(comp, s0, J.src + J.len - s0);
    const uint32_t x = (uint32_t)(J.src - s0);
    const uint32_t sl = ldsaddr(sst) + 16;
    bool par = J.len <= kHufOneStage && J.cnt <= kHufOneOut && lg >= 1 && lg <= kHufOneMaxLg;
    if (par) {
        // the stream's bytes (16 zero bytes below them), the cells
        if (t < 4)
            *la<uint32_t>(sl - 16 + 4 * t) = 0;
        for (uint32_t q = 16 * t; q < J.len; q += 16 * kHufOneT)
            *la<u32x4>(sl + q) = load16u(r, x + q);
        for (uint32_t c = t; c < (1u << lg); c += kHufOneT)
            tab[c] = gt[c];
        __syncthreads();
    }
    const uint32_t last = par ? (uint32_t)*la<uint8_t>(sl + J.len - 1) : 0u;
    par = par && last != 0;
    if (par) {
        const int32_t S = 8 * (int32_t)(J.len - 1) + (31 - __builtin_clz(last));   // bits below the end mark
        const uint32_t mask = (1u << lg) - 1;
        // lg bits below bit p (bit p - 1 most significant); bits below 0 read 0
        auto cell = [&](int32_t p) -> uint32_t {
            const int32_t lo = p - (int32_t)lg;
            const int32_t d = lo >> 5;   // >= -1: the zero bytes below
            const uint32_t a = (uint32_t)((int32_t)sl + 4 * d);
            const uint64_t w = (uint64_t)*la<uint32_t>(a) | (uint64_t)*la<uint32_t>(a + 4) << 32;
            return tab[(uint32_t)(w >> (uint32_t)(lo - 32 * d)) & mask];
        };
        // chunks of C >= 16 bits (> lg), at most kHufOneT of them, each with
        // bits: hi > 0
        const int32_t C = max<int32_t>(16, (S + (int32_t)kHufOneT - 1) / (int32_t)kHufOneT);
        const uint32_t T = (uint32_t)max<int32_t>(1, (S + C - 1) / C);
        const int32_t hi = S - (int32_t)t * C, lo = max(hi - C, 0);
        if (t < T) {
            const uint32_t ne = t == 0 ? 1u : lg;
            int32_t pc[kHufOneMaxLg];
            uint32_t nc[kHufOneMaxLg];
#pragma unroll
            for (uint32_t c = 0; c < kHufOneMaxLg; c++) {
                pc[c] = hi - (int32_t)c;
                nc[c] = 0;
            }
            for (bool any = true; any;) {
                any = false;
#pragma unroll
                for (uint32_t c = 0; c < kHufOneMaxLg; c++) {
                    if (c < ne && pc[c] > lo) {
                        const uint32_t e = cell(pc[c]);
                        pc[c] -= (int32_t)max(e & 0xFFu, 1u);
                        nc[c]++;
                        any = true;
                    }
                }
            }
#pragma unroll
            for (uint32_t c = 0; c < kHufOneMaxLg; c++)
                if (c < ne)
                    cand[t * kHufOneMaxLg + c] = (uint32_t)(lo - pc[c]) | nc[c] << 8;
        }
        __syncthreads();
        if (t == 0) {
            uint32_t c = 0, base = 0;
            for (uint32_t k = 0; k < T; k++) {
                ent[k] = c | base << 4;
                const uint32_t v = cand[k * kHufOneMaxLg + c];
                base += v >> 8;
                c = v & 0xFF;
            }
            verdict = c == 0 && base == J.cnt ? 1u : 0u;
        }
        __syncthreads();
        par = verdict != 0;
        if (par) {
            if (t < T) {
                const uint32_t e0 = ent[t];
                int32_t p = hi - (int32_t)(e0 & 15);
                for (uint32_t i = e0 >> 4; p > lo; i++) {
                    const uint32_t e = cell(p);
                    obuf[i] = (uint8_t)(e >> 8);
                    p -= (int32_t)max(e & 0xFFu, 1u);
                }
            }
            __syncthreads();
            // out: [0, lim) of the decoded symbols, 16-byte stores where aligned
            uint8_t *out = lit + J.dst;
            const uint32_t n = J.lim, head = min(n, (uint32_t)((16 - ((uintptr_t)out & 15)) & 15));
            if (t < head)
                out[t] = obuf[t];
            const uint32_t nq = (n - head) / 16;
            for (uint32_t q = t; q < nq; q += kHufOneT)
                *reinterpret_cast<u32x4 *>(out + head + 16 * q) = *la<u32x4_u>(ldsaddr(obuf) + head + 16 * q);
            const uint32_t tail = head + 16 * nq;
            if (tail + t < n)
                out[tail + t] = obuf[tail + t];
            if (t == 0)
                hbad[j] = 0;
            return;
        }
    }
    // the serial walk (zstd_huf_kernel's lane), thread 0
    if (t != 0)
        return;
    BRd b;
    bool bad = !br_init(b, r, x, J.len, ldsaddr(rings));
    auto Tg = [&](uint32_t i) -> uint32_t { return gt[i]; };
    huf_stream<2, 2, 0, 4>(b, Tg, lg, lit + J.dst, J.dst, J.cnt, J.lim);
    bad = bad || br_left(b) != 0;
    if (bad && jx2) {
        const uint32_t xr = x2_rescue(r, x, J.len, J.cnt, gt, lg);
        bad = !(xr & 1);
        if ((xr & 0x10000) && J.cnt - 1 < J.lim)
            lit[J.dst + J.cnt - 1] = (uint8_t)(xr >> 8);
    }
    hbad[j] = bad ? 1 : 0;
}

__global__ __launch_bounds__(kHufOneT) void zstd_huf_one_kernel(const uint8_t *__restrict__ jobs,
                                                                const uint8_t *__restrict__ comp,
                                                                const uint8_t *__restrict__ slots,
                                                                uint8_t *__restrict__ lit,
                                                                uint8_t *__restrict__ hbad)
{
    __shared__ HufOneLds H;
    huf_one_body(H, blockIdx.x, threadIdx.x, jobs, comp, slots, lit, hbad);
}

// ---- sequences: one lane per seek-table entry ------------------------------------------
// Replays the frame's op list: FSE states (tables from the block slots),
// repeat offsets, every libzstd check, items in the LZ4 item format with the
// full offset; then the final status, item count and checksum request.
// Items go straight from registers to the frame's slots: every emit issues
// exactly three 8-byte buffer stores (the ones it does not need are disabled
// by an out-of-range offset), so the compiler's vmcnt waits for the next
// sequence's bitstream window -- loaded before the stores -- never wait on
// them.  Consecutive 8-byte stores of a lane fill its lines in L2.
struct LSink {
    __amdgpu_buffer_rsrc_t r;   // the wave's item slots (one resource per replay)
    uint32_t ib;                // this frame's slot 0 in r (items)
    uint32_t k, cap;
};

typedef uint32_t u32x2s __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void lput3(const LSink &S, uint32_t n, uint64_t v0, uint64_t v1, uint64_t v2)
{
    const uint32_t a = 8u * (S.ib + S.k);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2s, v0), S.r, n >= 1 ? a : kOOR, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2s, v1), S.r, n >= 2 ? a + 8 : kOOR + 8, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2s, v2), S.r, n >= 3 ? a + 16 : kOOR + 16, 0, 0);
}

// the 8-byte item format of lz4_split.hip (Sink), with the full offset in
// extended items (an extended pair never starts in slot 63 of a 64-slot
// group: a zero item pads it)
// (ONE: every lane runs the emit in step; lane 0's stores land)
template <bool ONE = false>
__device__ __forceinline__ bool lemit(LSink &S, uint32_t src, uint32_t lit, uint32_t off, uint32_t ml)
{
    const bool ext = lit > 255 || ml > 258 || (ml != 0 && ml < 4) || off > 0xFFFF;
    const uint32_t pad = ext && (S.k & 63) == 63 ? 1u : 0u;
    const uint32_t n = ext ? 2 + pad : 1;
    const bool ok = S.k + n <= S.cap;
    const uint64_t e0 = ((uint64_t)off << 32) | src | kItemExt, e1 = ((uint64_t)ml << 32) | lit;
    const uint64_t sh = ((uint64_t)(off | lit << 16 | (ml ? ml - 3 : 0) << 24) << 32) | src;
    // (ONE: thread 0's -- lane 0 of the first wave -- land)
    lput3(S, ok && (!ONE || threadIdx.x == 0) ? n : 0, ext ? (pad ? 0 : e0) : sh, pad ? e0 : e1, e1);
    S.k += ok ? n : 0;
    return ok;
}

// Sequence bitstream reader, no ring: at each sequence the lane loads the 16
// bytes (4 dwords) just below its cursor together with the sequence's table
// cells — one wait covers both — and consumes from registers: C = the top
// two dwords, two reserve dwords shifted in by fills.  A sequence reads at
// most 89 bits; the window holds at least 97 below the cursor.  Coordinates
// are bits from the stream's dword-aligned base x0; bits below the stream's
// first byte (xs) read as 0.
struct SRd {
    __amdgpu_buffer_rsrc_t r;
    uint32_t x0;
    int32_t xs;
    int32_t cur;        // stream bits below cur are unread
    uint64_t C;         // bits [base, base + 64)
    int32_t base, nb;   // nb = cur - base valid bits at the bottom of C
    uint32_t r1, r0;    // the two dwords below C
    u32x4 L;            // the window in flight (sr_issue -> sr_use)
    int32_t D;
    uint32_t sl;        // the one-frame route: the stream's dwords staged at this LDS address (0: not)
    uint32_t zv;        // (ONE) an opaque per-lane zero added to LDS addresses (below)
};

// len >= 1.  False when the stream's last byte (its end mark) is 0.
__device__ __forceinline__ bool sr_init(SRd &b, __amdgpu_buffer_rsrc_t r, uint32_t x, uint32_t len)
{
    b.r = r;
    b.x0 = x & ~3u;
    b.xs = 8 * (int32_t)(x & 3u);
    const uint32_t rel = (x & 3u) + len;
    const uint32_t last = b.sl ? (uint32_t)*la<uint8_t>(b.sl + rel - 1)
                               : (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, b.x0 + rel - 1, 0, 0);
    b.cur = 8 * (int32_t)(rel - 1) + (last ? 31 - __builtin_clz(last) : 0);
    return last != 0;
}

// the window below the cursor in two halves: sr_issue loads it (one 16-byte
// load on every path, so the compiler's vmcnt counts stay exact; near the
// stream's base it loads dwords [0, 4) and sr_use shifts them up by -k0,
// dwords below the base reading as 0), sr_use unpacks it where it is first
// needed -- a sequence's window is issued at the end of the one before,
// ahead of that one's item stores
template <bool ONE>
__device__ __forceinline__ void sr_issue(SRd &b)
{
    const int32_t D = (b.cur + 31) >> 5, k0 = D - 4;   // dwords [k0, D) hold bits [32 k0, 32 D)
    // (ONE: the staged stream has 16 zero bytes below it, bits [-128, 0): a
    // window wholly below the stream -- a corrupt stream read past its start,
    // which libzstd 1.4.9 reads as zeros -- is those bytes too)
    if (ONE)
        b.L = *la<u32x4_a4>(b.sl + 4u * (uint32_t)(k0 > -4 ? k0 : -4) + b.zv);
    else
        b.L = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(b.r, b.x0 + 4u * (uint32_t)(k0 > 0 ? k0 : 0), 0, 0));
    b.D = D;
}

template <bool ONE = false>
__device__ __forceinline__ void sr_use(SRd &b)
{
    const int32_t D = b.D, k0 = D - 4;
    u32x4 w = b.L;
    // the window reaches the stream's first dword only at a block's last few
    // sequences: a branch the wave skips, not selects on every sequence (ONE:
    // the staged copy reads zeros there itself)
    if (!ONE && k0 <= 0) {
        const u32x4 L = b.L;
        const int32_t sft = -k0;
        w.x = sft == 0 ? L.x : 0u;
        w.y = sft == 0 ? L.y : sft == 1 ? L.x : 0u;
        w.z = sft == 0 ? L.z : sft == 1 ? L.y : sft == 2 ? L.x : 0u;
        w.w = sft == 0 ? L.w : sft == 1 ? L.z : sft == 2 ? L.y : sft == 3 ? L.x : 0u;
        // dword 0 holds the stream's first byte: clear the bits below it
        w.x &= above(b.xs, 32 * k0);
        w.y &= above(b.xs, 32 * k0 + 32);
        w.z &= above(b.xs, 32 * k0 + 64);
        w.w &= above(b.xs, 32 * k0 + 96);
    }
    b.C = (uint64_t)w.w << 32 | w.z;
    b.base = 32 * (D - 2);
    b.nb = b.cur - b.base;   // 33..64
    b.r1 = w.y;
    b.r0 = w.x;
}

template <bool ONE>
__device__ __forceinline__ void sr_load(SRd &b)
{
    sr_issue<ONE>(b);
    sr_use<ONE>(b);
}

__device__ __forceinline__ void sr_fill(SRd &b)
{
    const bool need = b.nb < 32;
    b.C = need ? (b.C << 32) | b.r1 : b.C;
    b.r1 = need ? b.r0 : b.r1;
    b.nb = need ? b.nb + 32 : b.nb;
    b.base = need ? b.base - 32 : b.base;
}

// n (<= 31) bits; nb >= n (a bitfield extract: width 0 reads 0)
__device__ __forceinline__ uint32_t sr_take(SRd &b, uint32_t n)
{
    const uint32_t v =
        __builtin_amdgcn_ubfe((uint32_t)(b.C >> ((uint32_t)(b.nb - (int32_t)n) & 63)), 0u, n);
    b.nb -= (int32_t)n;
    return v;
}

// close the sequence: the cursor moves past what was consumed
__device__ __forceinline__ void sr_done(SRd &b)
{
    b.cur = b.base + b.nb;
}


// 32 frames per wave (lanes 32..63 idle), one wave per workgroup: each
// frame's three FSE tables are copied into 1600 bytes of LDS when they fit
// (else read from the slot), so the per-sequence lookups stay on chip; with
// three such workgroups per CU the LDS, not the lanes, sets how many frames
// are in flight.  Same-box A/B at config 5 (sequence kernel alone in the
// profile, beside the Huffman kernel): 5.6 ms as here; tables read from the
// slot only, 64 or 32 frames per wave, 9.3 ms; 408 or 544 cells per frame
// (more workgroups per CU, more blocks' tables read from the slot) 8.2 and
// 6.6 ms; 1,056 or 1,312 cells (more blocks' tables in LDS, fewer frames per
// CU) 11.4 and 12.8 ms per launch against 10.6; the LL / ML code tables
// computed (packed constants and selects) instead of read from LDS, 11.05;
// 24 or 20 frames per wave (four or five single-wave workgroups per CU, one
// per SIMD) the same as 32.  Round 3, under the 4-chunk pipeline (other
// chunks' kernels beside it): tables from the slot (no LDS) 10.96 ms per
// launch at 32 frames per wave, 11.42 at 64, against 10.34 as here; the
// sequence loop made branch-free (repeat offsets, checks, window unpack)
// 11 % more wave cycles (its window wait no longer clear of the stores).
// OFG: only the LL and ML tables in LDS (544 cells: four workgroups per CU,
// 128 frames in flight instead of 96); the OF cell of the next sequence is
// loaded from the slot right after its state is known, just ahead of the
// next window load, so the one wait for the window covers it.  Same-box A/B
// at config 5: kernel alone 2.42 ms against 2.79 with all three tables in
// LDS (800 cells); the 4-chunk pipeline 9.25 / 9.27 against 9.43 / 9.40 ms
// per launch.
// GM generalizes it: bit t set = table t (LL, OF, ML) read from the slot, its
// cell loaded one sequence ahead; the others are staged in LDS.  More tables
// from the slot lose: OF + ML (288 cells, eight workgroups per CU) 4.71 ms
// alone, all three 6.45 ms, against 2.43 (pipeline 9.70 / 10.15 vs 9.26).
// Round 4: the bitstream through a per-lane LDS ring (64 dwords, refilled 4
// per sequence two sequences ahead, so the window is an LDS read and no load
// is waited on per sequence) loses -- the loop is issue-bound, not waiting on
// the window: same-box config 5, 3 chunks, 8.52 ms as here against 9.18 / 9.45
// with the ring beside these tables, 10.9 with the ring and all three tables in
// LDS (11.2 at 64 frames per wave); 4 chunks 8.85 against 9.05 / 10.6
// (profiles/r04_zstd_ring_ab.txt; the variant since removed).
constexpr uint32_t kSeqLanes = 32;
constexpr uint32_t kSeqCells = 544;   // u16 cells per frame (LL + ML 512 + copy slack)
constexpr uint32_t kSeqGm = 2;        // OF from the slot
// ONE (the one-frame route, a request's few frames): a wave per frame, every
// lane replaying the same frame in step (one lane's item stores land), with
// all three tables (up to 512 + 256 + 512 cells) and each block's sequence
// bitstream (up to kSeqStage bytes) staged in LDS by the whole wave.  A lone
// frame's replay is one dependent chain: with the window and the OF cell read
// from L2 / HBM per sequence it ran at ~0.8 us per sequence (853 us for a
// 64 KiB frame); from LDS the chain waits on LDS latency only.
constexpr uint32_t kSeqOneCells = 1312;
constexpr uint32_t kSeqStage = 131072 + 64;   // > a block's largest sequences section
#ifdef ZSK_TUNING
// tuning builds, ONE: [0] kernel cycles, [1] sequence-loop cycles, [2]
// sequences, [3] kernel real-time ticks (100 MHz), [4] frames; printed under
// ZSEEK_SEQ_TIMERS
__device__ unsigned long long g_sdiag[8];
#endif

// its LDS (a struct: the one-frame decode kernel below shares it with the
// Huffman job's, as a union)
template <uint32_t LANES, uint32_t CELLS, bool ONE>
struct SeqLds {
    uint32_t codes[89];
    __attribute__((aligned(16))) uint16_t ftab[CELLS && !ONE ? LANES * CELLS : 8];
    __attribute__((aligned(16))) uint8_t sstage[ONE ? kSeqStage + 32 : 16];
    uint64_t xtab[ONE ? kSeqOneCells : 1];                 // ONE: the expanded cells (below)
    __attribute__((aligned(16))) uint32_t srec[ONE ? 2 * 64 * 8 : 4];   // ONE: a batch's records (two buffers)
    uint32_t xflag;     // (two waves) a failure: stop
    uint32_t xst[8];    // (two waves) the replay state handed over
};

// the replay of workgroup bid (one wave: threads 0-63; TWO: two, the
// one-frame replay's chain on wave 0 and its vector phase on wave 1)
template <uint32_t LANES, uint32_t CELLS, uint32_t GM = 0, bool ONE = false, bool TWO = false>
__device__ __forceinline__ void seq_body(
    SeqLds<LANES, CELLS, ONE> &SH, uint32_t bid, const FrameDesc *__restrict__ desc, uint32_t n,
    const uint8_t *__restrict__ comp, uint8_t *__restrict__ ops, const uint64_t *__restrict__ blk_base,
    const uint8_t *__restrict__ slots, uint32_t *__restrict__ stop,
    const uint64_t *__restrict__ rec_base, uint64_t *__restrict__ items, uint32_t *__restrict__ nitems,
    int32_t *__restrict__ status, uint64_t *__restrict__ ck, uint32_t *__restrict__ fail_at, uint32_t f0)
{
    auto &codes = SH.codes;
    auto &ftab = SH.ftab;
    auto &sstage = SH.sstage;
    auto &xtab = SH.xtab;
    auto &srec = SH.srec;
#ifdef ZSK_TUNING
    const uint64_t tk0 = __builtin_readcyclecounter(), rt0 = __builtin_amdgcn_s_memrealtime();
    uint64_t tloop = 0, nseqs = 0, tchain = 0;
#endif
    for (uint32_t i = threadIdx.x; i < 89; i += 64)
        codes[i] = i < 36 ? c_ll[i] : c_ml[i - 36];
    if (threadIdx.x == 0)
        SH.xflag = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t f = ONE ? f0 + bid : f0 + bid * LANES + lane;   // frames [f0, n)
    const bool act = (ONE || lane < LANES) && f < n;
    FrameDesc d = {0, 0, 0, 0};
    if (act)
        d = desc[f];
    // one resource over the wave's frames (else lane by lane, each its own)
    const uint64_t lo = uni64(wave_min64(act ? d.c_off : ~0ull)) & ~15ull;
    const uint64_t hi = uni64(wave_max64(act ? d.c_off + d.c_size : 0ull));
    // the wave's item slots as one resource (else lane by lane, as comp);
    // reduced over the active lanes with every lane still present (an idle
    // lane's registers are not a value)
    uint64_t rb = 0;
    uint32_t icap = 0;
    if (act) {
        rb = rec_base[f];
        icap = (uint32_t)(rec_base[f + 1] - rb);
    }
    const uint64_t ilo = uni64(wave_min64(act ? rb : ~0ull)), ihi = uni64(wave_max64(act ? rb + icap : 0ull));
    if (!act)
        return;
    const uint64_t ob = op_base(blk_base, f);
    const uint32_t opn = (uint32_t)(op_base(blk_base, f + 1) - ob);
    ZOp *op = reinterpret_cast<ZOp *>(ops) + ob;
    LSink S;
    S.k = 0;
    S.cap = icap;
    uint16_t *const mytab = &ftab[CELLS && !ONE ? lane * CELLS : 0];
    const uint32_t cap = d.d_size;
    uint32_t o = 0, o0 = 0, rep0 = 1, rep1 = 4, rep2 = 8;
    uint64_t c = 0;
    int32_t st = zerr(ZE_GENERIC);
    // output offset where a failure is met: the start of the failing block
    // (every op of a block starts at its output start: literals advance
    // nothing, sequences and runs advance o), the frame's end for its
    // end-of-frame checks -- what libzstd's streaming decoder has produced
    // when it meets the failure (decompress.c:414-454)
    uint32_t fa = 0;
    uint32_t kstop = opn;   // the op the replay stopped at
    auto replay = [&](__amdgpu_buffer_rsrc_t r, uint64_t base, __amdgpu_buffer_rsrc_t ir, uint64_t i0) {
        S.r = ir;
        S.ib = (uint32_t)(rb - i0);
        for (uint32_t k = 0; k < opn; k++) {
            const ZOp P = op[k];
            uint32_t err = 0;
            fa = o;
            kstop = k;
            if (P.k == OP_LIT) {
                // the Huffman kernel runs beside this one: whether this
                // block's literals decoded is settled by zstd_lit_fix_kernel,
                // from the item count and output offset kept here
                op[k].b = S.k;
                op[k].c = o;
            } else if (P.k == OP_SEQ) {
                const uint32_t nseq = P.a;
                uint32_t lp_ = P.d;
                const uint32_t le = P.d + P.e;
                if (nseq) {
                    SRd b;
                    b.sl = 0;
                    b.zv = 0;
                    const uint32_t sx = (uint32_t)(d.c_off - base) + P.b;
                    bool staged = !ONE;
                    if (ONE && P.c != 0 && (sx & 3u) + P.c + 16 <= kSeqStage) {
                        // the stream's dwords into LDS, 16 bytes per lane per
                        // step, after 16 zero bytes; the bytes of its first dword
                        // below the stream zeroed too (the window's "bits below
                        // the stream read as 0" without a branch per sequence)
                        const uint32_t x0 = sx & ~3u, nb = (sx & 3u) + P.c, sl = ldsaddr(sstage) + 16;
                        // (TWO: wave 0 stages, then a barrier -- wave 1 reads
                        // the same bytes, so both waves take the same branches)
                        const bool stager = !TWO || threadIdx.x < 64;
                        if constexpr (TWO)
                            __syncthreads();   // (the last block's stage read by both)
                        wave_lds_sync();
                        if (stager)
                            for (uint32_t q = 16 * lane; q < nb; q += 1024)
                                *la<u32x4_a4>(sl + q) =
                                    __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, x0 + q, 0, 0));
                        wave_lds_sync();
                        if (stager && lane == 0) {
                            *la<u32x4>(sl - 16) = (u32x4){0, 0, 0, 0};
                            *la<uint32_t>(sl) &= above(8 * (int32_t)(sx & 3u), 0);
                        }
                        wave_lds_sync();
                        if constexpr (TWO)
                            __syncthreads();
                        b.sl = sl;
                        staged = true;
                    }
                    if (!staged) {   // (ONE: a block's sequences always fit the stage)
                        err = ZE_GENERIC;
                    } else if (P.c == 0 || !sr_init(b, r, sx, P.c)) {
                        err = ZE_CORRUPT;
                    } else {
                        const uint32_t tll = P.g & 15, tof = (P.g >> 4) & 15, tml = (P.g >> 8) & 15;
                        // the block's tables into this lane's LDS cells when they
                        // fit: LL, OF, ML back to back (16-byte copies)
                        const uint16_t *gt = reinterpret_cast<const uint16_t *>(slots + (uint64_t)P.f * kZSlot + kSlotFse);
                        const uint32_t nll = 1u << tll, nof = 1u << tof, nml = 1u << tml;
                        const uint16_t *TL = gt + kFseOff[0], *TO = gt + kFseOff[1], *TM = gt + kFseOff[2];
                      if constexpr (ONE) {
                        // the one-frame replay: every cell expanded once by the
                        // wave into 8 bytes -- lo: the LDS address of its next
                        // state's base cell; hi: the state's bit count (bits
                        // 0-3, bit 4 clear: a bitfield extract's width or offset
                        // operand as it is), the value's extra bits (8-12), a
                        // bad-symbol flag (13), the symbol (16-21), the cell's
                        // whole bit count (value + state, 24-29) -- so a
                        // sequence's chain is one LDS read per table and its next
                        // cells' addresses two ops away from the bits (no
                        // code-table read, no next-state arithmetic).  Same bit
                        // order, values and checks as the loop below.
                        const uint32_t xb = ldsaddr(xtab), ncell = nll + nof + nml;
                        wave_lds_sync();
                        for (uint32_t cix = lane; cix < ((!TWO || threadIdx.x < 64) ? ncell : 0u); cix += 64) {
                            const uint32_t t = cix < nll ? 0u : cix < nll + nof ? 1u : 2u;
                            const uint32_t toff = t == 0 ? 0u : t == 1 ? nll : nll + nof;
                            const uint32_t x = cix - toff;
                            const uint32_t e = t == 0 ? TL[x] : t == 1 ? TO[x] : TM[x];
                            const uint32_t tl = t == 0 ? tll : t == 1 ? tof : tml;
                            const uint32_t sym = e & 63, ns = e >> 6;
                            const uint32_t nbits = tl + (uint32_t)__builtin_clz(ns) - 31;
                            const uint32_t nbase = (ns << nbits) - (1u << tl);
                            const bool bad = sym > (t == 0 ? 35u : t == 1 ? 31u : 52u);
                            // OF: value 2^code + code extra bits; LL / ML: the code table
                            const uint32_t code = bad || t == 1 ? 0u : codes[t == 0 ? sym : 36 + sym];
                            const uint32_t add = bad ? 0u : t == 1 ? sym : code >> 24;
                            const uint32_t hi32 = nbits | add << 8 | (bad ? 1u : 0u) << 13 | (bad ? 0u : sym) << 16 |
                                                  (add + nbits) << 24;
                            *la<uint64_t>(xb + 8 * cix) = (uint64_t)hi32 << 32 | (xb + 8 * (toff + nbase));
                        }
                        wave_lds_sync();
                        if constexpr (TWO)
                            __syncthreads();   // (wave 0's cells, seen by both)
                        // (an opaque per-lane zero in the addresses keeps the chain
                        // in VGPRs: scalarized, each LDS result waited for and
                        // copied to SGPRs at once -- the window's and the cells'
                        // reads no longer in flight together)
                        uint32_t zv;
                        asm volatile("v_mov_b32 %0, 0" : "=v"(zv));
                        b.zv = zv;
                        auto XL = [&](uint32_t x) { return *la<uint64_t>(xb + 8 * x + zv); };
                        auto XO = [&](uint32_t x) { return *la<uint64_t>(xb + 8 * (nll + x) + zv); };
                        auto XM = [&](uint32_t x) { return *la<uint64_t>(xb + 8 * (nll + nof + x) + zv); };
                        sr_load<ONE>(b);
                        uint64_t cl, co, cm;
                        {
                            const uint32_t sll = sr_take(b, tll), sof = sr_take(b, tof), sml = sr_take(b, tml);
                            sr_done(b);
                            cl = XL(sll);
                            co = XO(sof);
                            cm = XM(sml);
                        }
                        // the window: stream dwords [(cur >> 5) - 3, + 4), the
                        // staged zeros below the stream for a cursor past its start
                        const uint32_t sl = b.sl;
                        auto win = [&](int32_t cur) {
                            const int32_t k0 = (cur >> 5) - 3;
                            return *la<u32x4_a4>(sl + 4u * (uint32_t)(k0 > -4 ? k0 : -4) + zv);
                        };
                        int32_t cur = b.cur;
                        u32x4 W = win(cur);
#ifdef ZSK_TUNING
                        const uint64_t tl0 = __builtin_readcyclecounter();
                        nseqs += nseq;
#endif
                        // batches of up to 64 sequences: (1) the chain, wave-
                        // uniform -- cells, state bits, next states -> one 32-byte
                        // record per sequence in LDS: its 64 value bits and its
                        // three cells (a bad cell goes on: its state fields are
                        // valid); (2) lane q takes record q: the values,
                        // repeat offsets, item slots, the output / literal prefix
                        // sums, the replay's
                        // checks in its order (a bad cell first), the first
                        // failing sequence by ballot, and the items of the
                        // sequences before it (a lane's own stores).  Everything
                        // the serial loop below leaves -- items, o, lp_, S.k,
                        // err -- is the same.
                        const uint32_t rec = ldsaddr(srec);
                        // the chain of a batch of nb sequences: records at rb
                        auto chain = [&](uint32_t rb, uint32_t nb) {
                                if (lane == 0)
                                for (uint32_t q = 0; q < nb; q++) {
                                    // the 96 stream bits below cur, top-aligned: bit
                                    // 95 of N3:N2:N1 is stream bit cur - 1 (the
                                    // align takes the shift's low five bits)
                                    const uint32_t N3 = __builtin_amdgcn_alignbit(W.w, W.z, (uint32_t)cur),
                                                   N2 = __builtin_amdgcn_alignbit(W.z, W.y, (uint32_t)cur),
                                                   N1 = __builtin_amdgcn_alignbit(W.y, W.x, (uint32_t)cur);
                                    const uint64_t H = (uint64_t)N3 << 32 | N2;
                                    const uint32_t hl = (uint32_t)(cl >> 32), hm = (uint32_t)(cm >> 32), ho = (uint32_t)(co >> 32);
                                    // the sequence's bits: OF, ML, LL values, then the
                                    // LL, ML, OF states (T <= 31 + 16 + 16 + 26 = 89)
                                    // (byte-select adds: the three counts are the cells' top bytes)
                                    uint32_t T;
                                    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:BYTE_3\n\t"
                                        "v_add_u32_sdwa %0, %0, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
                                        : "=&v"(T)
                                        : "v"(hl), "v"(hm), "v"(ho));
                                    // (T <= 64: from N3:N2; else at bit 96 - T < 32 of N2:N1)
                                    const uint32_t yH = (uint32_t)(H >> ((64 - T) & 63)),
                                                   yM = __builtin_amdgcn_alignbit(N2, N1, 0u - T);
                                    // (a select in asm: the compiler made the choice an
                                    // if / else over the exec mask, twice the ops)
                                    uint32_t Y;
                                    asm("v_cmp_ge_u32 vcc, 64, %1\n\tv_cndmask_b32 %0, %2, %3, vcc"
                                        : "=v"(Y)
                                        : "v"(T), "v"(yM), "v"(yH)
                                        : "vcc");
                                    // (the extract takes offset and width from the low
                                    // five bits: the state counts straight from hi)
                                    const uint32_t ao = (uint32_t)co + (__builtin_amdgcn_ubfe(Y, 0, ho) << 3),
                                                   am = (uint32_t)cm + (__builtin_amdgcn_ubfe(Y, ho, hm) << 3),
                                                   al = (uint32_t)cl + (__builtin_amdgcn_ubfe(Y, ho + hm, hl) << 3);
                                    const int32_t cur2 = cur - (int32_t)T;
                                    // the record (this sequence's values are the
                                    // vector phase's, from H and the cells), stored
                                    // ahead of the next sequence's reads: after them,
                                    // the wait for them would wait for it too
                                    // (two paired stores in asm: the compiler's own
                                    // choice varied with the kernel it sat in, up to
                                    // four stores and four address moves)
                                    asm volatile("ds_write2_b64 %0, %1, %2 offset1:1\n\t"
                                                 "ds_write2_b64 %0, %3, %4 offset0:2 offset1:3"
                                                 :
                                                 : "v"(rb + 32 * q), "v"(H), "v"(cl), "v"(cm), "v"(co)
                                                 : "memory");
                                    const u32x4 W2 = win(cur2);
                                    const uint64_t cl2 = *la<uint64_t>(al), cm2 = *la<uint64_t>(am), co2 = *la<uint64_t>(ao);
                                    cl = cl2;
                                    cm = cm2;
                                    co = co2;
                                    W = W2;
                                    cur = cur2;
                                }
                        };
                        // the vector phase of a batch of nd records at rb
                        auto vphase = [&](uint32_t rb, uint32_t nd) {
                                const bool on = lane < nd;
                                uint32_t ofv = 0, ml = 0, ll = 0, bad = 0;
                                if (on) {
                                    const u32x4 R = *la<u32x4>(rb + 32 * lane), R2 = *la<u32x4>(rb + 32 * lane + 16);
                                    const uint32_t hl = R.w, hm = R2.y, ho = R2.w;
                                    const uint32_t ob = __builtin_amdgcn_ubfe(ho, 8, 5), mb = __builtin_amdgcn_ubfe(hm, 8, 5),
                                                   lb = __builtin_amdgcn_ubfe(hl, 8, 5), vb = ob + mb + lb;
                                    const uint64_t H = (uint64_t)R.y << 32 | R.x;
                                    const uint32_t X = (uint32_t)(H >> ((64 - vb) & 63));
                                    ofv = (1u << ob) + __builtin_amdgcn_ubfe(R.y, 32 - ob, ob);
                                    ll = (codes[__builtin_amdgcn_ubfe(hl, 16, 6)] & 0xFFFFFF) + __builtin_amdgcn_ubfe(X, 0, lb);
                                    ml = (codes[36 + __builtin_amdgcn_ubfe(hm, 16, 6)] & 0xFFFFFF) + __builtin_amdgcn_ubfe(X, lb, mb);
                                    bad = ((ho | hm | hl) >> 13) & 1;
                                }
                                // repeat offsets (RFC 8878 §3.1.2.5) by a scan: each
                                // sequence maps the history (a, b, c) = (rep0, rep1,
                                // rep2) to a new one -- a new offset v: (v, a, b);
                                // index 0: (a, b, c); 1: (b, a, c); 2: (c, a, b); 3:
                                // (a - 1 but >= 1, a, b) -- and its offset is the new
                                // first entry.  A composed map keeps, per entry,
                                // either a value (tag 3) or "old entry t less d"
                                // (tag t, d decrements: max(x - d, 1), as repeated
                                // decrements of values >= 1 compose).  Six shuffle
                                // steps compose each lane's prefix; applied to the
                                // batch's starting history they give every offset.
                                uint32_t tg[3], vl[3];
                                {
                                    const bool fresh = ofv > 3;
                                    const uint32_t idx = fresh ? 0u : ofv - 1 + (ll == 0);
                                    tg[0] = fresh ? 3u : idx == 3 ? 0u : idx;
                                    vl[0] = fresh ? ofv - 3 : idx == 3 ? 1u : 0u;
                                    tg[1] = !fresh && idx == 0 ? 1u : 0u;
                                    tg[2] = !fresh && idx <= 1 ? 2u : 1u;
                                    vl[1] = vl[2] = 0;
                                    if (!on) {   // identity
                                        tg[0] = 0;
                                        tg[1] = 1;
                                        tg[2] = 2;
                                        vl[0] = 0;
                                    }
                                }
    #pragma unroll
                                for (uint32_t sft = 1; sft < 64; sft <<= 1) {
                                    uint32_t pt[3], pv[3];
    #pragma unroll
                                    for (int q = 0; q < 3; q++) {
                                        pt[q] = (uint32_t)__shfl_up((int)tg[q], sft, 64);
                                        pv[q] = (uint32_t)__shfl_up((int)vl[q], sft, 64);
                                    }
                                    if (lane >= sft) {
    #pragma unroll
                                        for (int q = 0; q < 3; q++) {   // mine after the earlier prefix
                                            const uint32_t t = tg[q], v = vl[q];
                                            const uint32_t et = t == 0 ? pt[0] : t == 1 ? pt[1] : pt[2];
                                            const uint32_t ev = t == 0 ? pv[0] : t == 1 ? pv[1] : pv[2];
                                            tg[q] = t == 3 ? 3u : et;
                                            vl[q] = t == 3 ? v : et == 3 ? (ev > v ? ev - v : 1u) : ev + v;
                                        }
                                    }
                                }
                                auto apply = [&](uint32_t t, uint32_t v) -> uint32_t {
                                    if (t == 3)
                                        return v;
                                    const uint32_t x = t == 0 ? rep0 : t == 1 ? rep1 : rep2;
                                    return x > v ? x - v : 1u;
                                };
                                const uint32_t off = apply(tg[0], vl[0]);
                                if (nd) {
                                    const uint32_t n0 = lane_val(off, (int)nd - 1),
                                                   n1v = lane_val(apply(tg[1], vl[1]), (int)nd - 1),
                                                   n2v = lane_val(apply(tg[2], vl[2]), (int)nd - 1);
                                    rep0 = n0;
                                    rep1 = n1v;
                                    rep2 = n2v;
                                }
                                // item slots (lemit's rule: an extended pair never
                                // starts in slot 63 of a 64-slot group, a zero item
                                // pads it): a scan without pads, then, only if some
                                // extended pair lands on slot 63, the slots again
                                // sequence by sequence
                                const bool ext = on && (ll > 255 || ml > 258 || (ml != 0 && ml < 4) || off > 0xFFFF);
                                const uint32_t n1 = on ? (ext ? 2u : 1u) : 0u;
                                uint32_t kq = S.k + wave_incl_add(n1) - n1, pad = 0;
                                if (__ballot(ext && (kq & 63) == 63)) {
                                    uint32_t k = S.k;
                                    for (uint32_t q = 0; q < nd; q++) {
                                        const bool eq = lane_val(ext ? 1u : 0u, (int)q) != 0;
                                        const uint32_t pq = eq && (k & 63) == 63 ? 1u : 0u;
                                        if (lane == q) {
                                            kq = k;
                                            pad = pq;
                                        }
                                        k += eq ? 2 + pq : 1;
                                    }
                                }
                                const uint32_t ni = ext ? 2 + pad : 1;
                                const uint32_t ill = wave_incl_add(ll), iol = wave_incl_add(ll + ml);
                                const uint32_t lpq = lp_ + ill - ll, oq = o + iol - (ll + ml);
                                const uint32_t kind = bad                ? (uint32_t)ZE_CORRUPT
                                                      : ll + ml > cap - oq ? (uint32_t)ZE_DST_SMALL
                                                      : le - lpq < ll    ? (uint32_t)ZE_CORRUPT
                                                      : off > oq + ll    ? (uint32_t)ZE_CORRUPT
                                                      : kq + ni > S.cap  ? (uint32_t)ZE_GENERIC
                                                                         : 0u;
                                const uint64_t em = __ballot(on && kind != 0);
                                const uint32_t e = em ? (uint32_t)__builtin_ctzll(em) : nd;
                                if (lane < e) {
                                    const uint64_t e0 = ((uint64_t)off << 32) | lpq | kItemExt, e1 = ((uint64_t)ml << 32) | ll;
                                    const uint64_t sh = ((uint64_t)(off | ll << 16 | (ml ? ml - 3 : 0) << 24) << 32) | lpq;
                                    LSink Q = S;
                                    Q.k = kq;
                                    lput3(Q, ni, ext ? (pad ? 0 : e0) : sh, pad ? e0 : e1, e1);
                                }
                                if (e > 0) {
                                    lp_ += lane_val(ill, (int)e - 1);
                                    o += lane_val(iol, (int)e - 1);
                                }
                                if (e < nd) {
                                    err = lane_val(kind, (int)e);
                                    S.k = lane_val(kq, (int)e);
                                } else {
                                    if (nd)
                                        S.k = lane_val(kq + ni, (int)nd - 1);
                                }
                        };
                        if constexpr (TWO) {
                            // two waves (the fused launch's first two): wave 0
                            // runs batch k's chain while wave 1 runs batch k - 1's
                            // vector phase -- records double-buffered, one
                            // barrier per step; a failure found by wave 1 stops
                            // both after the step; then wave 1's replay state and
                            // wave 0's cursor are exchanged, so both waves go on
                            // with the same values
                            const uint32_t wv = threadIdx.x >> 6, nbat = (nseq + 63) / 64;
                            for (uint32_t kb = 0; kb <= nbat; kb++) {
                                if (wv == 0 && kb < nbat) {
#ifdef ZSK_TUNING
                                    const uint64_t tc0 = __builtin_readcyclecounter();
#endif
                                    chain(rec + 2048 * (kb & 1), min(64u, nseq - 64 * kb));
#ifdef ZSK_TUNING
                                    tchain += __builtin_readcyclecounter() - tc0;
#endif
                                }
                                if (wv == 1 && kb >= 1) {
                                    vphase(rec + 2048 * ((kb - 1) & 1), min(64u, nseq - 64 * (kb - 1)));
                                    if (err && lane == 0)
                                        SH.xflag = 1;
                                }
                                __syncthreads();
                                if (uni(*lp<uint32_t>(&SH.xflag)))
                                    break;
                            }
                            if (wv == 1 && lane == 0) {
                                SH.xst[0] = o;
                                SH.xst[1] = lp_;
                                SH.xst[2] = S.k;
                                SH.xst[3] = err;
                                SH.xst[4] = rep0;
                                SH.xst[5] = rep1;
                                SH.xst[6] = rep2;
                            }
                            if (wv == 0 && lane == 0)
                                SH.xst[7] = (uint32_t)cur;
                            __syncthreads();
                            o = uni(*lp<uint32_t>(&SH.xst[0]));
                            lp_ = uni(*lp<uint32_t>(&SH.xst[1]));
                            S.k = uni(*lp<uint32_t>(&SH.xst[2]));
                            err = uni(*lp<uint32_t>(&SH.xst[3]));
                            rep0 = uni(*lp<uint32_t>(&SH.xst[4]));
                            rep1 = uni(*lp<uint32_t>(&SH.xst[5]));
                            rep2 = uni(*lp<uint32_t>(&SH.xst[6]));
                            cur = (int32_t)uni(*lp<uint32_t>(&SH.xst[7]));
                            __syncthreads();   // (everyone has read; the flag reset for the next block)
                            if (threadIdx.x == 0)
                                SH.xflag = 0;
                            __syncthreads();
                        } else {
                            for (uint32_t i = 0; i < nseq && !err;) {
                                const uint32_t nb = min(64u, nseq - i);
                                wave_lds_sync();   // the last batch's records read
#ifdef ZSK_TUNING
                                const uint64_t tc0 = __builtin_readcyclecounter();
#endif
                                chain(rec, nb);
                                wave_lds_sync();
#ifdef ZSK_TUNING
                                tchain += __builtin_readcyclecounter() - tc0;
#endif
                                vphase(rec, nb);
                                i += nb;
                            }
                        }
                        b.cur = __builtin_amdgcn_readlane(cur, 0);
#ifdef ZSK_TUNING
                        tloop += __builtin_readcyclecounter() - tl0;
#endif
                      } else {
                        // cells staged in LDS per table (0: read from the slot)
                        const uint32_t nlll = (GM & 1) ? 0u : nll, nofl = (GM & 2) ? 0u : nof,
                                       nmll = (GM & 4) ? 0u : nml;
                        const bool fit = nlll + nofl + nmll == 0 || (CELLS && nlll + nofl + nmll + 32 <= CELLS);
                        if (fit) {
                            // (ONE: the whole wave copies, 8 cells per lane per step)
                            auto cp = [&](const uint16_t *src, uint32_t at, uint32_t cells) {
                                for (uint32_t c = ONE ? 8 * lane : 0; c < cells; c += ONE ? 512 : 8)
                                    *reinterpret_cast<u32x4 *>(mytab + at + c) = *reinterpret_cast<const u32x4 *>(src + c);
                            };
                            if (ONE)
                                wave_lds_sync();
                            cp(TL, 0, nlll);
                            cp(TO, nlll, nofl);
                            cp(TM, nlll + nofl, nmll);
                            if (ONE)
                                wave_lds_sync();
                        }
                        // the sequence loop, over tables in LDS (ds_read: the
                        // lookups' waits stay off vmcnt) or in the slot
                        auto seqs = [&](auto TLf, auto TOf, auto TMf) {
                            sr_load<ONE>(b);

                            uint32_t sll = sr_take(b, tll), sof = sr_take(b, tof), sml = sr_take(b, tml);
                            sr_done(b);
                            sr_issue<ONE>(b);
                            // three disabled stores: the loop's entry then has the
                            // VMEM pattern of its back edge (window, then three
                            // stores), so the window's wait stays vmcnt(3)
                            lput3(S, 0, 0, 0, 0);
                            // the slot tables' cells, one sequence ahead
                            uint32_t ell_n = 0, eof_n = 0, eml_n = 0;
                            if (GM & 1)
                                ell_n = TLf(sll);
                            if (GM & 2)
                                eof_n = TOf(sof);
                            if (GM & 4)
                                eml_n = TMf(sml);
                            for (uint32_t i = 0; i < nseq; i++) {
                                const uint32_t ell = (GM & 1) ? ell_n : TLf(sll), eof = (GM & 2) ? eof_n : TOf(sof),
                                               eml = (GM & 4) ? eml_n : TMf(sml);
                                sr_use(b);
                                const uint32_t llc = ell & 63, ofc = eof & 63, mlc = eml & 63;
                                if (llc > 35 || ofc > 31 || mlc > 52) {
                                    err = ZE_CORRUPT;
                                    break;
                                }
                                // offset bits (<= 31; the window holds >= 33), a fill before
                                // the ML + LL extra bits (<= 32) and one before the three
                                // state updates (<= 26)
                                // offset value < 2^32 (ofc <= 31)
                                const uint32_t ofv = (1u << ofc) + sr_take(b, ofc);
                                const uint32_t mlcode = codes[36 + mlc], llcode = codes[llc];
                                sr_fill(b);
                                // the ML and LL extra bits (<= 32, ML above LL) in one extract
                                const uint32_t mlb = mlcode >> 24, llb = llcode >> 24;
                                const uint32_t X = (uint32_t)(b.C >> ((uint32_t)(b.nb - (int32_t)(mlb + llb)) & 63));
                                b.nb -= (int32_t)(mlb + llb);
                                const uint32_t ll = (llcode & 0xFFFFFF) + __builtin_amdgcn_ubfe(X, 0u, llb);
                                const uint32_t ml = (mlcode & 0xFFFFFF) + __builtin_amdgcn_ubfe(X, llb, mlb);
                                // repeat offsets as selects (RFC 8878 §3.1.2.5): a new
                                // offset (ofv > 3) or repeat idx 0..3; idx 0 keeps the
                                // history, idx 1 swaps the first two, 2 and 3 rotate
                                // (selects by the index bits: a nested ?: chain
                                // compiled to branches)
                                const bool fresh = ofv > 3;
                                const uint32_t idx = fresh ? 0u : ofv - 1 + (ll == 0);
                                const uint32_t r01 = (idx & 1) ? rep1 : rep0,
                                               r23 = (idx & 1) ? max(rep0 - 1, 1u) : rep2;   // rep0 - 1, 0 read as 1
                                const uint32_t off = fresh ? ofv - 3 : (idx & 2) ? r23 : r01;
                                const bool sh1 = fresh || idx != 0, sh2 = fresh || idx >= 2;
                                rep2 = sh2 ? rep1 : rep2;
                                rep1 = sh1 ? rep0 : rep1;
                                rep0 = sh1 ? off : rep0;
                                sr_fill(b);
                                // the three next states (fse_next's bits, <= 26: LL, ML,
                                // OF from the top) in one extract
                                const uint32_t nsl = ell >> 6, nsm = eml >> 6, nso = eof >> 6;
                                const uint32_t bl = tll + (uint32_t)__builtin_clz(nsl) - 31,
                                               bm = tml + (uint32_t)__builtin_clz(nsm) - 31,
                                               bo = tof + (uint32_t)__builtin_clz(nso) - 31;
                                const uint32_t Y = (uint32_t)(b.C >> ((uint32_t)(b.nb - (int32_t)(bl + bm + bo)) & 63));
                                b.nb -= (int32_t)(bl + bm + bo);
                                sll = ((nsl << bl) - (1u << tll)) + __builtin_amdgcn_ubfe(Y, bm + bo, bl);
                                sml = ((nsm << bm) - (1u << tml)) + __builtin_amdgcn_ubfe(Y, bo, bm);
                                sof = ((nso << bo) - (1u << tof)) + __builtin_amdgcn_ubfe(Y, 0u, bo);
                                if (GM & 1)
                                    ell_n = TLf(sll);
                                if (GM & 2)
                                    eof_n = TOf(sof);
                                if (GM & 4)
                                    eml_n = TMf(sml);
                                sr_done(b);
                                sr_issue<ONE>(b);
                                // o <= cap: no 32-bit overflow in these tests
                                if (ll + ml > cap - o)
                                    err = ZE_DST_SMALL;
                                else if (le - lp_ < ll)
                                    err = ZE_CORRUPT;
                                else if (off > o + ll)
                                    err = ZE_CORRUPT;
                                else if (!lemit(S, lp_, ll, (uint32_t)off, ml))
                                    err = ZE_GENERIC;
                                if (err)
                                    break;
                                lp_ += ll;
                                o += ll + ml;
                            }
                        };
                        const uint32_t tb = (uint32_t)(uintptr_t)lp<uint16_t>(mytab);
                        if (fit)
                            seqs([&](uint32_t x) -> uint32_t {
                                     return (GM & 1) ? (uint32_t)TL[x] : (uint32_t)*la<uint16_t>(tb + 2 * x);
                                 },
                                 [&](uint32_t x) -> uint32_t {
                                     return (GM & 2) ? (uint32_t)TO[x] : (uint32_t)*la<uint16_t>(tb + 2 * (nlll + x));
                                 },
                                 [&](uint32_t x) -> uint32_t {
                                     return (GM & 4) ? (uint32_t)TM[x]
                                                     : (uint32_t)*la<uint16_t>(tb + 2 * (nlll + nofl + x));
                                 });
                        else
                            seqs([&](uint32_t x) -> uint32_t { return TL[x]; }, [&](uint32_t x) -> uint32_t { return TO[x]; },
                                 [&](uint32_t x) -> uint32_t { return TM[x]; });
                      }
                        if (!err && b.cur - b.xs > 0)
                            err = ZE_CORRUPT;
                    }
                }
                if (!err) {
                    const uint32_t last = le - lp_;
                    if (o + last > cap)
                        err = ZE_DST_SMALL;
                    else if (last && !lemit<ONE>(S, lp_, last, 0, 0))
                        err = ZE_GENERIC;
                    else
                        o += last;
                }
            } else if (P.k == OP_RUN) {
                if (P.b > cap - o)
                    err = ZE_DST_SMALL;
                else if (P.b && !lemit<ONE>(S, P.a, P.b, 0, 0))
                    err = ZE_GENERIC;
                else
                    o += P.b;
            } else if (P.k == OP_FBEGIN) {
                rep0 = 1;
                rep1 = 4;
                rep2 = 8;
                o0 = o;
            } else if (P.k == OP_FEND) {
                if ((P.a & 1) && (uint64_t)(o - o0) != ((uint64_t)P.c << 32 | P.b))
                    err = ZE_CORRUPT;
                else if (P.a & 2)
                    c = (1ull << 63) | ((uint64_t)o0 << 32) | P.d;
            } else if (P.k == OP_ERR) {
                st = (int32_t)P.a;
                break;
            } else {   // OP_DONE (anything else: a list the frame kernel never wrote)
                st = P.k == OP_DONE ? (o == cap ? ST_OK : ST_SHORT_FRAME) : zerr(ZE_GENERIC);
                break;
            }
            if (err) {
                st = zerr(err);
                break;
            }
        }
    };
    auto irsrc = [&](uint64_t a, uint64_t b) {
        return __builtin_amdgcn_make_buffer_rsrc((void *)(items + a), 0, (int)(uint32_t)(8 * (b - a)), kRsrcDw3);
    };
    if (ONE || (hi > lo && hi - lo < kMaxSpan && 8 * (ihi - ilo) < kMaxSpan)) {
        // (ONE: one frame's span, < 4 GiB compressed and items)
        replay(span_rsrc(comp, lo, hi - lo), lo, irsrc(ilo, ihi), ilo);
    } else {
        for (uint64_t m = __ballot(true); m; m &= m - 1) {
            const int l = __builtin_ctzll(m);
            const uint64_t s0 = uni64(__shfl(d.c_off, l, 64)) & ~15ull;
            const uint64_t s1 = uni64(__shfl(d.c_off + d.c_size, l, 64));
            const uint64_t i0 = uni64(__shfl(rb, l, 64)), i1 = uni64(__shfl(rb + S.cap, l, 64));
            if ((int)lane == l)
                replay(span_rsrc(comp, s0, s1 - s0), s0, irsrc(i0, i1), i0);
        }
    }
    if (ONE && threadIdx.x != 0)
        return;
#ifdef ZSK_TUNING
    if (ONE) {
        atomicAdd(&g_sdiag[0], (unsigned long long)(__builtin_readcyclecounter() - tk0));
        atomicAdd(&g_sdiag[1], (unsigned long long)tloop);
        atomicAdd(&g_sdiag[5], (unsigned long long)tchain);
        atomicAdd(&g_sdiag[2], (unsigned long long)nseqs);
        atomicAdd(&g_sdiag[3], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - rt0));
        atomicAdd(&g_sdiag[4], 1ull);
    }
#endif
    status[f] = st;
    nitems[f] = S.k;
    ck[f] = c;
    stop[f] = kstop;
    if (fail_at)
        fail_at[f] = st == ST_OK ? 0 : fa;
}

template <uint32_t LANES, uint32_t CELLS, uint32_t GM = 0, bool ONE = false>
__global__ __launch_bounds__(64) void zstd_seq_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    uint8_t *__restrict__ ops, const uint64_t *__restrict__ blk_base,
    const uint8_t *__restrict__ slots, uint32_t *__restrict__ stop,
    const uint64_t *__restrict__ rec_base, uint64_t *__restrict__ items, uint32_t *__restrict__ nitems,
    int32_t *__restrict__ status, uint64_t *__restrict__ ck, uint32_t *__restrict__ fail_at, uint32_t f0)
{
    __shared__ SeqLds<LANES, CELLS, ONE> SH;
    seq_body<LANES, CELLS, GM, ONE>(SH, blockIdx.x, desc, n, comp, ops, blk_base, slots, stop, rec_base, items,
                                    nitems, status, ck, fail_at, f0);
}

__device__ __forceinline__ void lit_fix(uint32_t f, const uint8_t *__restrict__ ops,
                                        const uint64_t *__restrict__ blk_base, const uint8_t *__restrict__ hbad,
                                        const uint32_t *__restrict__ stop, int32_t *__restrict__ status,
                                        uint32_t *__restrict__ nitems, uint32_t *__restrict__ fail_at);

// The one-frame route's replay and Huffman streams in one launch: workgroups
// [0, m) replay frame f0 + b on their first wave (the others leave), the rest
// decode Huffman job b - m with all kHufOneT threads -- no second stream, so
// no event between the frame kernel and them or between them and the
// literal fix-up (~8-11 us each on the request's timeline).  LDS: the union.
// The workgroup finishing last (a counter in `done`, zero between launches:
// the last one resets it) runs the literal fix-up (zstd_lit_fix_kernel's
// work) -- every replay and Huffman job is done by then; nothing waits.
__global__ __launch_bounds__(kHufOneT) void zstd_one_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    uint8_t *__restrict__ ops, const uint64_t *__restrict__ blk_base,
    const uint8_t *__restrict__ slots, uint32_t *__restrict__ stop,
    const uint64_t *__restrict__ rec_base, uint64_t *__restrict__ items, uint32_t *__restrict__ nitems,
    int32_t *__restrict__ status, uint64_t *__restrict__ ck, uint32_t *__restrict__ fail_at, uint32_t f0,
    uint32_t m, const uint8_t *__restrict__ jobs, uint8_t *__restrict__ lit, uint8_t *__restrict__ hbad,
    uint32_t *__restrict__ done)
{
    __shared__ union {
        SeqLds<1, 0, true> s;
        HufOneLds h;
    } U;
    __shared__ uint32_t last;
    const uint32_t b = blockIdx.x, t = threadIdx.x;
    if (b < m) {
        // waves 0 and 1: the replay's chain and its vector phase.  Waves 2
        // and 3 leave before any barrier: a wave that has ended no longer
        // counts at s_barrier (CDNA), so seq_body's data-dependent barriers
        // and the two below are met by waves 0 and 1 alone, and no wave
        // reads `last` before thread 0 has written it.
        if (t >= 128)
            return;
        seq_body<1, 0, 0, true, true>(U.s, b, desc, n, comp, ops, blk_base, slots, stop, rec_base, items, nitems,
                                      status, ck, fail_at, f0);
    } else {
        huf_one_body(U.h, b - m, t, jobs, comp, slots, lit, hbad);
    }
    // (thread 0 wrote what the fix-up reads: status, items, stop, hbad)
    __syncthreads();
    if (t == 0) {
        __threadfence();
        last = atomicAdd(done, 1u) == gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (!last)
        return;
    __threadfence();
    if (t < 64)
        for (uint32_t f = f0 + t; f < n; f += 64)
            lit_fix(f, ops, blk_base, hbad, stop, status, nitems, fail_at);
    if (t == 0)
        *done = 0;
}

// After the Huffman and sequence kernels (which run side by side): a frame
// whose replay passed a literals op of a block with a corrupt Huffman stream
// fails there, as libzstd does — that block's literals are decoded before its
// sequences — with the items and output offset the replay had at that op.
__device__ __forceinline__ void lit_fix(uint32_t f, const uint8_t *__restrict__ ops,
                                        const uint64_t *__restrict__ blk_base, const uint8_t *__restrict__ hbad,
                                        const uint32_t *__restrict__ stop, int32_t *__restrict__ status,
                                        uint32_t *__restrict__ nitems, uint32_t *__restrict__ fail_at)
{
    const ZOp *op = reinterpret_cast<const ZOp *>(ops) + op_base(blk_base, f);
    const uint32_t ks = stop[f];
    for (uint32_t k = 0; k < ks; k++) {
        const ZOp P = op[k];
        if (P.k == OP_LIT && *reinterpret_cast<const uint32_t *>(hbad + 4ull * P.a)) {
            status[f] = zerr(ZE_CORRUPT);
            nitems[f] = P.b;
            if (fail_at)
                fail_at[f] = P.c;
            return;
        }
    }
}

__global__ __launch_bounds__(256) void zstd_lit_fix_kernel(uint32_t n, const uint8_t *__restrict__ ops,
                                                           const uint64_t *__restrict__ blk_base,
                                                           const uint8_t *__restrict__ hbad,
                                                           const uint32_t *__restrict__ stop,
                                                           int32_t *__restrict__ status,
                                                           uint32_t *__restrict__ nitems,
                                                           uint32_t *__restrict__ fail_at, uint32_t f0)
{
    const uint32_t f = f0 + blockIdx.x * 256 + threadIdx.x;   // frames [f0, n)
    if (f < n)
        lit_fix(f, ops, blk_base, hbad, stop, status, nitems, fail_at);
}

// XXH64 of [o0, cap) of a frame's output for frames flagged by the frame
// kernel: lanes 0..3 run the four accumulators over 1 KiB chunks staged in
// LDS by the whole wave; lane 0 merges and finishes.
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r)
{
    return (x << r) | (x >> (64 - r));
}

constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full,
                   P64_3 = 0x165667B19E3779F9ull, P64_4 = 0x85EBCA77C2B2AE63ull,
                   P64_5 = 0x27D4EB2F165667C5ull;

__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t v)
{
    acc += v * P64_2;
    acc = rotl64(acc, 31);
    return acc * P64_1;
}

__device__ __forceinline__ uint64_t xmerge(uint64_t acc, uint64_t v)
{
    acc ^= xround(0, v);
    return acc * P64_1 + P64_4;
}

__global__ __launch_bounds__(256) void zstd_check_kernel(const FrameDesc *__restrict__ desc, uint32_t n,
                                                         const uint8_t *__restrict__ out,
                                                         const uint64_t *__restrict__ ck,
                                                         int32_t *__restrict__ status,
                                                         uint32_t *__restrict__ fail_at, uint32_t stop_last)
{
    __shared__ uint64_t buf[4][128];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t f = uni(blockIdx.x * 4 + w);
    if (f >= n)
        return;
    const uint64_t c = ck[f];
    if (!(c >> 63) || uni((uint32_t)status[f]) != (uint32_t)ST_OK)
        return;
    const FrameDesc d = desc[f];
    // (a no-cache read's last frame executed only up to the request's end:
    // libzstd's streaming decoder never reaches the frame's end and its
    // checksum there either)
    if (f + 1 == n && stop_last < d.d_size)
        return;
    const uint32_t o0 = (uint32_t)(c >> 32) & 0x7FFFFFFFu, want = (uint32_t)c;
    const uint8_t *p = out + d.d_off + o0;
    const uint32_t len = d.d_size - o0;
    const Span sp = make_span(p, len);
    uint64_t acc = lane == 0 ? P64_1 + P64_2 : lane == 1 ? P64_2 : lane == 2 ? 0 : 0ull - P64_1;
    const uint32_t stripes = len / 32;
    for (uint32_t s0 = 0; s0 < stripes; s0 += 32) {
        // 32 stripes = 1 KiB: 16 bytes per lane
        const u32x4 v = load16u(sp.r, sp.s0 + 1024 * (s0 / 32) + 16 * lane);
        *reinterpret_cast<u32x4 *>(&buf[w][2 * lane]) = v;
        const uint32_t m = stripes - s0 < 32 ? stripes - s0 : 32;
        if (lane < 4)
            for (uint32_t i = 0; i < m; i++)
                acc = xround(acc, buf[w][4 * i + lane]);
    }
    uint64_t h;
    const uint64_t a1 = __shfl(acc, 1, 64), a2 = __shfl(acc, 2, 64), a3 = __shfl(acc, 3, 64);
    if (len >= 32) {
        h = rotl64(acc, 1) + rotl64(a1, 7) + rotl64(a2, 12) + rotl64(a3, 18);
        h = xmerge(h, acc);
        h = xmerge(h, a1);
        h = xmerge(h, a2);
        h = xmerge(h, a3);
    } else {
        h = P64_5;
    }
    h += len;
    if (lane == 0) {
        uint32_t i = stripes * 32;
        for (; i + 8 <= len; i += 8) {
            uint64_t k = 0;
            for (int b = 0; b < 8; b++)
                k |= (uint64_t)p[i + b] << (8 * b);
            h ^= xround(0, k);
            h = rotl64(h, 27) * P64_1 + P64_4;
        }
        for (; i + 4 <= len; i += 4) {
            const uint64_t k = (uint64_t)p[i] | (uint64_t)p[i + 1] << 8 | (uint64_t)p[i + 2] << 16 |
                               (uint64_t)p[i + 3] << 24;
            h ^= k * P64_1;
            h = rotl64(h, 23) * P64_2 + P64_3;
        }
        for (; i < len; i++) {
            h ^= p[i] * P64_5;
            h = rotl64(h, 11) * P64_1;
        }
        h ^= h >> 33;
        h *= P64_2;
        h ^= h >> 29;
        h *= P64_3;
        h ^= h >> 32;
        if ((uint32_t)h != want) {
            status[f] = zerr(ZE_CHECKSUM);
            if (fail_at)
                fail_at[f] = d.d_size;   // checked at the frame's end
        }
    }
}

// blk_base at the decode's chunk boundaries (zstd_chunks) -> out[0..k]
__global__ void zstd_bounds_kernel(const uint64_t *__restrict__ blk_base, uint32_t n, uint32_t k,
                                   uint64_t *__restrict__ out)
{
    const uint32_t c = threadIdx.x;
    if (c <= k)
        out[c] = blk_base[(uint64_t)n * c / k];
}

}   // namespace

// ---- host side -----------------------------------------------------------------------------------

namespace {
template <typename T>
int grow(T **p, uint64_t &cap, uint64_t want, uint64_t unit)
{
    if (want <= cap)
        return 0;
    if (*p)
        (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    if (hipMalloc((void **)p, want * unit) != hipSuccess)
        return -1;
    cap = want;
    return 0;
}

// The Huffman kernel's side stream and its two events belong to the scratch.
// Teardown (zstd_scratch_free) drains the side stream and destroys it before
// its events and before the caller's stream goes: the side stream's wait on
// an event recorded on the caller's stream is released while that stream is
// still alive.
void drop_streams(ZstdScratch *s)
{
    for (hipStream_t *q : {&s->side, &s->sq})
        if (*q) {
            (void)hipStreamSynchronize(*q);
            hip_stream_put(*q);
            *q = nullptr;
        }
}

// streams first, then the events recorded on them
void side_destroy(ZstdScratch *s)
{
    drop_streams(s);
    for (int c = 0; c < ZstdScratch::kChunks; c++)
        for (hipEvent_t *e : {&s->ev_f[c], &s->ev_s[c], &s->ev_h[c]})
            if (*e) {
                hip_event_put(*e);
                *e = nullptr;
            }
}

int side_create(ZstdScratch *s)
{
    // the Huffman stream at the lowest priority: the sequence kernel, the
    // longer of the two, gets the CUs' LDS first (10.9 -> 10.6 ms per launch
    // at config 5; launching the sequence kernel first made no difference)
    (void)hipGetDevice(&s->side_dev);
    bool ok = hip_stream_get(&s->side, true) == hipSuccess && hip_stream_get(&s->sq, false) == hipSuccess;
    for (int c = 0; ok && c < ZstdScratch::kChunks; c++)
        for (hipEvent_t *e : {&s->ev_f[c], &s->ev_s[c], &s->ev_h[c]})
            ok = ok && (*e || hip_event_get(e) == hipSuccess);
    if (!ok) {   // partly created, nothing recorded on it yet
        side_destroy(s);
        return -1;
    }
    return 0;
}

// Chunks a decode of n frames runs in (frames [n c / k, n (c + 1) / k)): the
// frame kernel of chunk c + 1 and the execute of chunk c - 1 run beside the
// sequence and Huffman kernels of chunk c, which leave most of each CU's
// issue slots idle.  Env ZSEEK_ZSTD_CHUNKS (A/B runs).  Config
// 5 (65,536 frames), same box, after the round-3 kernel changes: 2 chunks
// 9.50 / 9.57 ms, 3 8.71 / 8.73, 4 9.04 / 9.03, 6 10.07 / 10.17.
uint32_t zstd_chunks(uint32_t n)
{
    static const int forced = getenv("ZSEEK_ZSTD_CHUNKS") ? atoi(getenv("ZSEEK_ZSTD_CHUNKS")) : 0;
    uint32_t k = n >= 16384 ? 3 : n >= 4096 ? 2 : 1;
    if (forced > 0)
        k = (uint32_t)forced;
    if (k > (uint32_t)ZstdScratch::kChunks)
        k = ZstdScratch::kChunks;
    return k > n ? (n ? n : 1) : k;
}
}   // namespace

int zstd_scratch_reserve(ZstdScratch *s, uint32_t frames, uint64_t out_bytes, uint64_t items,
                         uint64_t blocks, hipStream_t stream)
{
    (void)stream;
    if (!s->side && side_create(s) != 0)
        return -1;
    if (frames + 1 > s->frames_cap) {
        const uint32_t cap = frames + 1 < 4096 ? 4096 : frames + 1;
        for (void *p : {(void *)s->bound, (void *)s->bblk, (void *)s->rec_base, (void *)s->blk_base,
                        (void *)s->nitems, (void *)s->ck, (void *)s->stop, (void *)s->d_total})
            if (p)
                (void)hipFree(p);
        if (s->total)
            (void)hipHostFree(s->total);
        s->bound = s->bblk = s->nitems = s->stop = nullptr;
        s->rec_base = s->blk_base = s->ck = s->d_total = s->total = nullptr;
        s->frames_cap = 0;
        if (hipMalloc((void **)&s->bound, sizeof(uint32_t) * cap) != hipSuccess ||
            hipMalloc((void **)&s->bblk, sizeof(uint32_t) * cap) != hipSuccess ||
            hipMalloc((void **)&s->rec_base, sizeof(uint64_t) * (cap + 1)) != hipSuccess ||
            hipMalloc((void **)&s->blk_base, sizeof(uint64_t) * (cap + 1)) != hipSuccess ||
            hipMalloc((void **)&s->nitems, sizeof(uint32_t) * cap) != hipSuccess ||
            hipMalloc((void **)&s->ck, sizeof(uint64_t) * cap) != hipSuccess ||
            hipMalloc((void **)&s->stop, sizeof(uint32_t) * cap) != hipSuccess ||
            hipMalloc((void **)&s->d_total, (6 + ZstdScratch::kChunks) * sizeof(uint64_t)) != hipSuccess ||
            hipMemset(s->d_total, 0, (6 + ZstdScratch::kChunks) * sizeof(uint64_t)) != hipSuccess ||
            hipHostMalloc((void **)&s->total, (5 + ZstdScratch::kChunks) * sizeof(uint64_t), hipHostMallocDefault) !=
                hipSuccess)
            return -1;
        s->total[0] = s->total[1] = s->total[2] = 0;
        s->frames_cap = cap;
    }
    if (grow(&s->lit, s->lit_cap, out_bytes + 64, 1) != 0 || grow(&s->items, s->items_cap, items, 8) != 0)
        return -1;
    if (blocks > s->blocks_cap) {
        uint64_t c0 = s->blocks_cap, c1 = s->blocks_cap, c2 = s->blocks_cap;
        if (grow(&s->hjobs, c0, blocks, 4 * sizeof(HufJob)) != 0 ||
            grow(&s->hbad, c1, blocks, 4) != 0 || grow(&s->slots, c2, blocks, kZSlot) != 0)
            return -1;
        s->blocks_cap = blocks;
    }
    // op lists: 4 per block + 4 per frame
    return grow(&s->ops, s->ops_cap, blocks + frames, 4 * sizeof(ZOp));
}

void zstd_scratch_drop_streams(ZstdScratch *s)
{
    drop_streams(s);
}

void zstd_scratch_release_memory(ZstdScratch *s)
{
    for (hipStream_t q : {s->side, s->sq})
        if (q)
            (void)hipStreamSynchronize(q);
    for (void *p : {(void *)s->bound, (void *)s->bblk, (void *)s->rec_base, (void *)s->blk_base,
                    (void *)s->nitems, (void *)s->ck, (void *)s->stop, (void *)s->lit, (void *)s->items,
                    (void *)s->ops, (void *)s->hjobs, (void *)s->slots, (void *)s->hbad, (void *)s->d_total})
        if (p)
            (void)hipFree(p);
    if (s->total)
        (void)hipHostFree(s->total);
    if (s->h_plan)
        (void)hipHostFree(s->h_plan);
    if (s->d_plan)
        (void)hipFree(s->d_plan);
    s->h_plan = s->d_plan = nullptr;
    s->h_plan_cap = 0;
    s->bound = s->bblk = s->nitems = s->stop = nullptr;
    s->rec_base = s->blk_base = s->ck = s->d_total = s->total = nullptr;
    s->lit = s->slots = s->hbad = nullptr;
    s->items = nullptr;
    s->ops = s->hjobs = nullptr;
    s->frames_cap = 0;
    s->lit_cap = s->items_cap = s->blocks_cap = s->ops_cap = 0;
}

// memory (its streams drained), then streams, then events
void zstd_scratch_free(ZstdScratch *s)
{
    zstd_scratch_release_memory(s);
    side_destroy(s);
    *s = ZstdScratch();
}

// Plan only: bounds + offsets, then the item total, output extent and block
// total copied into s->total (pinned host memory), valid once the stream
// reaches it.
int launch_zstd_plan(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                     ZstdScratch *s, hipStream_t stream)
{
    if (nframes == 0)
        return 0;
    if (hipMemsetAsync(s->d_total, 0, 4 * sizeof(uint64_t), stream) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(zstd_plan_kernel, dim3((nframes + 255) / 256), dim3(256), 0, stream, d_desc,
                       nframes, d_comp, s->bound, s->bblk, reinterpret_cast<unsigned long long *>(s->d_total + 1));
    hipLaunchKernelGGL(zstd_scan_kernel, dim3(1), dim3(1024), 0, stream, s->bound, s->bblk, nframes,
                       s->rec_base, s->blk_base, s->d_total);
    const uint32_t k = zstd_chunks(nframes);
    hipLaunchKernelGGL(zstd_bounds_kernel, dim3(1), dim3(64), 0, stream, s->blk_base, nframes, k, s->d_total + 4);
    if (hipGetLastError() != hipSuccess)
        return -1;
    return hipMemcpyAsync(s->total, s->d_total, (5 + k) * sizeof(uint64_t), hipMemcpyDeviceToHost, stream) ==
                   hipSuccess
               ? 0
               : -1;
}

// Frame kernel -> Huffman kernel beside the sequence kernel -> literal fix-up
// -> execute -> checksums, in zstd_chunks(n) chunks of frames pipelined over
// three streams: the caller's stream runs every chunk's frame kernel, then
// each chunk's fix-up, execute and checksums once its sequence (s->sq) and
// Huffman (s->side) kernels are done; those start on a chunk as soon as its
// frame kernel is.  s must hold the last plan of these frames.
int launch_zstd_decode(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                       uint8_t *d_out, int32_t *d_status, ZstdScratch *s, hipStream_t stream,
                       uint32_t *d_fail_at, uint32_t stop_last, bool cks)
{
    if (nframes == 0)
        return 0;
    const uint64_t blocks = s->total[2];
    if (blocks > s->blocks_cap)
        return -1;
    const uint32_t K = zstd_chunks(nframes);
    static const bool serial = getenv("ZSEEK_ZSTD_SERIAL") != nullptr;   // diagnostics: one stream
    // the one-frame route (a request's few frames): the execute a workgroup
    // per frame (env ZSEEK_ONE_ROUTE=0: the wave kernels, as round 4)
    static const bool one_off = [] {
        const char *v = getenv("ZSEEK_ONE_ROUTE");
        return v && !strcmp(v, "0");
    }();
    const bool one = !one_off && nframes <= kOneMaxFrames;
    // (the one-frame route's sequence replay on the caller's stream, right
    // behind the frame kernel: a cross-stream hand-off cost ~30 us each way;
    // with its Huffman jobs in the same launch, zstd_one_kernel -- env
    // ZSEEK_ONE_FUSE=0: the Huffman kernel on the side stream, as before)
    static const bool fuse_off = [] {
        const char *v = getenv("ZSEEK_ONE_FUSE");
        return v && !strcmp(v, "0");
    }();
    const bool fuse = one && !fuse_off;
    hipStream_t const hs = serial ? stream : s->side, qs = serial || one ? stream : s->sq;
#ifdef ZSK_TUNING
    static const int diag = getenv("ZSEEK_ZSTD_HUF_DIAG") ? atoi(getenv("ZSEEK_ZSTD_HUF_DIAG")) : 0;
#endif
    auto drain = [&] {   // an enqueue failed: nothing may still write the scratch
        (void)hipStreamSynchronize(stream);
        (void)hipStreamSynchronize(s->side);
        (void)hipStreamSynchronize(s->sq);
        return -1;
    };
    auto bnd = [&](uint32_t c) { return (uint32_t)((uint64_t)nframes * c / K); };
    for (uint32_t c = 0; c < K; c++) {
        const uint32_t f0 = bnd(c), f1 = bnd(c + 1), m = f1 - f0;
        if (m == 0)
            continue;
        const uint64_t b0 = s->total[4 + c], b1 = s->total[5 + c];
        hipEvent_t tf = kernel_span_begin(stream);   // (per-kernel spans: timing on only)
        // (the one-frame route: a workgroup per frame, its second wave the
        // Huffman descriptions' helper; env ZSEEK_FRAME_HELP=0: off)
        static const bool help_off = [] {
            const char *v = getenv("ZSEEK_FRAME_HELP");
            return v && !strcmp(v, "0");
        }();
        if (one && !help_off)
            hipLaunchKernelGGL(zstd_frame_kernel<true>, dim3(m), dim3(64 * kZW), 0, stream, d_desc, f1, d_comp,
                               s->lit, s->lit_cap, s->rec_base, s->items_cap, s->blk_base, s->ops, s->slots,
                               s->hjobs, f0);
        else
            hipLaunchKernelGGL(zstd_frame_kernel<false>, dim3((m + kZW - 1) / kZW), dim3(64 * kZW), 0, stream,
                               d_desc, f1, d_comp, s->lit, s->lit_cap, s->rec_base, s->items_cap, s->blk_base,
                               s->ops, s->slots, s->hjobs, f0);
#ifdef ZSK_TUNING
        {
            static const bool ztimers = getenv("ZSEEK_ZFRAME_TIMERS") != nullptr;
            static int zcalls = 0;
            if (ztimers && ++zcalls % 100 == 0) {
                unsigned long long z[12] = {0};
                (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_zftime), sizeof(z), 0, hipMemcpyDeviceToHost, stream);
                (void)hipStreamSynchronize(stream);
                const double fr = z[4] ? (double)z[4] : 1.0;
                fprintf(stderr,
                        "zstd frame kernel cycles per frame: total %.0f huffman descriptions %.0f sequence tables %.0f "
                        "window stagings %.0f | weights: ncount %.0f build %.0f walk %.0f | sequence tables: "
                        "ncount %.0f build %.0f cells out %.0f (%llu frames)\n",
                        z[0] / fr, z[1] / fr, z[2] / fr, z[3] / fr, z[5] / fr, z[6] / fr, z[7] / fr, z[8] / fr,
                        z[9] / fr, z[10] / fr, z[4]);
            }
        }
#endif
        kernel_span_end(SPAN_ZFRAME, tf, stream);
        const uint32_t nj = (uint32_t)(4 * (b1 - b0));
        if (fuse) {
            hipEvent_t tq = kernel_span_begin(stream);
            hipLaunchKernelGGL(zstd_one_kernel, dim3(m + nj), dim3(kHufOneT), 0, stream, d_desc, f1, d_comp, s->ops,
                               s->blk_base, s->slots, s->stop, s->rec_base, s->items, s->nitems, d_status, s->ck,
                               d_fail_at, f0, m, s->hjobs + 4 * b0 * sizeof(HufJob), s->lit, s->hbad + 4 * b0,
                               reinterpret_cast<uint32_t *>(s->d_total + 5 + ZstdScratch::kChunks));
            kernel_span_end(SPAN_ZSEQ, tq, stream);
#ifdef ZSK_TUNING
            static const bool timers = getenv("ZSEEK_SEQ_TIMERS") != nullptr;
            static int calls = 0;
            if (timers && ++calls % 100 == 0) {
                unsigned long long z[8] = {0};
                (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_sdiag), sizeof(z), 0, hipMemcpyDeviceToHost, stream);
                (void)hipStreamSynchronize(stream);
                const double fr = z[4] ? (double)z[4] : 1.0, sq = z[2] ? (double)z[2] : 1.0;
                fprintf(stderr,
                        "one-frame sequences: kernel %.0f cycles (%.1f us, %.0f MHz) per frame, loop %.0f cycles "
                        "(%.0f per sequence, chain alone %.0f, %.0f sequences per frame)\n",
                        z[0] / fr, z[3] / fr / 100.0, z[3] ? z[0] * 100.0 / z[3] : 0.0, z[1] / fr, z[1] / sq,
                        z[5] / sq, sq / fr);
            }
#endif
            continue;
        }
        if (hipEventRecord(s->ev_f[c], stream) != hipSuccess || hipStreamWaitEvent(qs, s->ev_f[c], 0) != hipSuccess)
            return drain();
        // the Huffman streams decode beside the sequence replay (neither reads
        // the other's output); zstd_lit_fix_kernel joins them
        if (nj) {
            if (hipStreamWaitEvent(hs, s->ev_f[c], 0) != hipSuccess)
                return drain();
            const uint8_t *jb = s->hjobs + 4 * b0 * sizeof(HufJob);
            uint8_t *hb = s->hbad + 4 * b0;
            const dim3 g((nj + 63) / 64), b(64);
            hipEvent_t th = kernel_span_begin(hs);
#ifdef ZSK_TUNING
            // diagnostics (tuning builds, ZSEEK_ZSTD_HUF_DIAG): 1 / 3 / 7 / 8
            // counters and elisions (printed)
            const bool counters = diag != 0;
            if (counters) {
                unsigned int z[32] = {};
                (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_hdiag), z, sizeof(z), 0, hipMemcpyHostToDevice, hs);
            }
            switch (one ? -1 : diag) {
            case -1:
                hipLaunchKernelGGL(zstd_huf_one_kernel, dim3(nj), dim3(kHufOneT), 0, hs, jb, d_comp, s->slots, s->lit, hb);
                break;
            case 0: hipLaunchKernelGGL(zstd_huf_kernel<0>, g, b, 0, hs, jb, nj, d_comp, s->slots, s->lit, hb); break;
            case 1: hipLaunchKernelGGL(zstd_huf_kernel<1>, g, b, 0, hs, jb, nj, d_comp, s->slots, s->lit, hb); break;
            case 3: hipLaunchKernelGGL(zstd_huf_kernel<3>, g, b, 0, hs, jb, nj, d_comp, s->slots, s->lit, hb); break;
            case 7: hipLaunchKernelGGL(zstd_huf_kernel<7>, g, b, 0, hs, jb, nj, d_comp, s->slots, s->lit, hb); break;
            default: hipLaunchKernelGGL(zstd_huf_kernel<8>, g, b, 0, hs, jb, nj, d_comp, s->slots, s->lit, hb); break;
            }
#else
            if (one)
                hipLaunchKernelGGL(zstd_huf_one_kernel, dim3(nj), dim3(kHufOneT), 0, hs, jb, d_comp, s->slots, s->lit, hb);
            else
                hipLaunchKernelGGL(zstd_huf_kernel<0>, g, b, 0, hs, jb, nj, d_comp, s->slots, s->lit, hb);
#endif
#ifdef ZSK_TUNING
            if (counters) {
                unsigned int z[32] = {};
                (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_hdiag), sizeof(z), 0, hipMemcpyDeviceToHost, hs);
                (void)hipStreamSynchronize(hs);
                fprintf(stderr, "huf diag %d (chunk %u): lgmax", diag, c);
                for (int i = 0; i < 16; i++)
                    if (z[i])
                        fprintf(stderr, " %d:%u", i, z[i]);
                fprintf(stderr, "  global %u lds %u\n", z[16], z[17]);
            }
#endif
            kernel_span_end(SPAN_ZHUF, th, hs);
            if (hipEventRecord(s->ev_h[c], hs) != hipSuccess)
                return drain();
        }
        hipEvent_t tq = kernel_span_begin(qs);
#ifdef ZSK_TUNING
        // A/B (tuning builds): ZSEEK_ZSTD_SEQ=1 tables from the slot (no LDS),
        // 64 frames per wave; 2: the same, 32 frames per wave; 3: all three
        // tables in LDS (800 cells per frame)
        static const int seqv = getenv("ZSEEK_ZSTD_SEQ") ? atoi(getenv("ZSEEK_ZSTD_SEQ")) : 0;
        if (seqv == 1)
            hipLaunchKernelGGL((zstd_seq_kernel<64, 0>), dim3((m + 63) / 64), dim3(64), 0, qs, d_desc, f1, d_comp,
                               s->ops, s->blk_base, s->slots, s->stop, s->rec_base, s->items, s->nitems, d_status,
                               s->ck, d_fail_at, f0);
        else if (seqv == 2)
            hipLaunchKernelGGL((zstd_seq_kernel<32, 0>), dim3((m + 31) / 32), dim3(64), 0, qs, d_desc, f1, d_comp,
                               s->ops, s->blk_base, s->slots, s->stop, s->rec_base, s->items, s->nitems, d_status,
                               s->ck, d_fail_at, f0);
        else if (seqv == 3)   // round 3's layout: all three tables in LDS (800 cells)
            hipLaunchKernelGGL((zstd_seq_kernel<32, 800>), dim3((m + 31) / 32), dim3(64), 0, qs, d_desc, f1, d_comp,
                               s->ops, s->blk_base, s->slots, s->stop, s->rec_base, s->items, s->nitems, d_status,
                               s->ck, d_fail_at, f0);
        else
#endif
        if (one) {
            hipLaunchKernelGGL((zstd_seq_kernel<1, 0, 0, true>), dim3(m), dim3(64), 0, qs, d_desc, f1, d_comp, s->ops,
                               s->blk_base, s->slots, s->stop, s->rec_base, s->items, s->nitems, d_status, s->ck,
                               d_fail_at, f0);
#ifdef ZSK_TUNING
            static const bool timers = getenv("ZSEEK_SEQ_TIMERS") != nullptr;
            static int calls = 0;
            if (timers && ++calls % 100 == 0) {
                unsigned long long z[8] = {0};
                (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_sdiag), sizeof(z), 0, hipMemcpyDeviceToHost, qs);
                (void)hipStreamSynchronize(qs);
                const double fr = z[4] ? (double)z[4] : 1.0, sq = z[2] ? (double)z[2] : 1.0;
                fprintf(stderr,
                        "one-frame sequences: kernel %.0f cycles (%.1f us, %.0f MHz) per frame, loop %.0f cycles "
                        "(%.0f per sequence, %.0f sequences per frame)\n",
                        z[0] / fr, z[3] / fr / 100.0, z[3] ? z[0] * 100.0 / z[3] : 0.0, z[1] / fr, z[1] / sq, sq / fr);
            }
        }
#else
        }
#endif
        else
        hipLaunchKernelGGL((zstd_seq_kernel<kSeqLanes, kSeqCells, kSeqGm>), dim3((m + kSeqLanes - 1) / kSeqLanes), dim3(64), 0,
                           qs, d_desc, f1, d_comp, s->ops, s->blk_base, s->slots, s->stop, s->rec_base, s->items,
                           s->nitems, d_status, s->ck, d_fail_at, f0);
        kernel_span_end(SPAN_ZSEQ, tq, qs);
        if (hipEventRecord(s->ev_s[c], qs) != hipSuccess)
            return drain();
    }
    stage_mark(2, stream);
    int rc = 0;
    for (uint32_t c = 0; c < K; c++) {
        const uint32_t f0 = bnd(c), f1 = bnd(c + 1), m = f1 - f0;
        if (m == 0)
            continue;
        const uint64_t b0 = s->total[4 + c], b1 = s->total[5 + c];
        if (!fuse && (hipStreamWaitEvent(stream, s->ev_s[c], 0) != hipSuccess ||
                      (b1 > b0 && hipStreamWaitEvent(stream, s->ev_h[c], 0) != hipSuccess)))
            return drain();
        if (b1 > b0 && !fuse)   // (fused: the last workgroup's)
            hipLaunchKernelGGL(zstd_lit_fix_kernel, dim3((m + 255) / 256), dim3(256), 0, stream, f1, s->ops,
                               s->blk_base, s->hbad, s->stop, d_status, s->nitems, d_fail_at, f0);
        hipEvent_t tx = kernel_span_begin(stream);
        const uint32_t stop = c + 1 == K ? stop_last : 0xFFFFFFFFu;   // (the batch's last frame)
        if (launch_seq_exec_lit(d_desc + f0, m, s->lit, d_out, s->rec_base + f0, s->items, s->nitems + f0,
                                d_status + f0, stream, one, (uint32_t)std::min<uint64_t>(s->total[3], 0xFFFFFFFFu),
                                stop) != 0)
            rc = -1;
        kernel_span_end(SPAN_ZEXEC, tx, stream);
        if (cks)   // (a host plan that met no content checksum: nothing to check)
            hipLaunchKernelGGL(zstd_check_kernel, dim3((m + 3) / 4), dim3(256), 0, stream, d_desc + f0, m, d_out,
                               s->ck + f0, d_status + f0, d_fail_at ? d_fail_at + f0 : nullptr, stop);
    }
    stage_mark(3, stream);
    stage_mark(4, stream);
    return rc == 0 && hipGetLastError() == hipSuccess ? 0 : -1;
}

// Plan, wait for the totals, size the scratch, decode.  The one
// synchronization point of the zstd path: the item slots and table slots of a
// frame are only known once its block headers and sequence counts are read.
int zstd_decode_frames(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                       uint8_t *d_out, int32_t *d_status, ZstdScratch *s, hipStream_t stream,
                       uint32_t *d_fail_at, uint32_t stop_last)
{
    if (nframes == 0)
        return 0;
    (void)hipGetLastError();   // a stale error of an earlier call is not this launch's
    if (zstd_scratch_reserve(s, nframes, 0, 0, 0, stream) != 0)
        return -1;
    stage_mark(0, stream);
    if (launch_zstd_plan(d_desc, nframes, d_comp, s, stream) != 0)
        return -1;
    stage_mark(1, stream);
    if (hipStreamSynchronize(stream) != hipSuccess)
        return -1;
    if (zstd_scratch_reserve(s, nframes, s->total[1], s->total[0], s->total[2], stream) != 0)
        return -1;
    return launch_zstd_decode(d_desc, nframes, d_comp, d_out, d_status, s, stream, d_fail_at, stop_last);
}

// zstd_plan_kernel's per-frame bound on the host: item slots (8 + 4 per
// block + 2 per sequence + the pairs' padding, rounded up to 4) and blocks,
// from the frame headers, block headers, literals section headers and
// sequence counts -- the same walk, the same arithmetic.
static void zstd_plan_frame_host(const uint8_t *c, uint32_t clen, uint32_t *bound, uint32_t *bblk, bool *cks)
{
    auto B = [&](uint32_t p) -> uint32_t { return p < clen ? (uint32_t)c[p] : 0u; };
    uint64_t items = 8;
    uint32_t ip = 0, blocks = 0;
    while (clen - ip >= 9 && items < (1u << 30)) {
        const uint32_t magic = B(ip) | B(ip + 1) << 8 | B(ip + 2) << 16 | B(ip + 3) << 24;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            ip += 8 + (B(ip + 4) | B(ip + 5) << 8 | B(ip + 6) << 16 | B(ip + 7) << 24);
            continue;
        }
        if (magic != kZMagic)
            break;
        const uint32_t fhd = B(ip + 4);
        const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, did = fhd & 3;
        ip += 5 + !single + (did == 3 ? 4 : did) + (fcs_flag == 0 ? single : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8);
        for (;;) {
            if (clen < ip + 3)
                break;
            const uint32_t bh = B(ip) | B(ip + 1) << 8 | B(ip + 2) << 16;
            const uint32_t type = (bh >> 1) & 3, bsize = bh >> 3;
            ip += 3;
            items += 4;
            blocks++;
            if (type == 2 && bsize >= 3) {
                const uint32_t b0 = B(ip), lt = b0 & 3, sf = (b0 >> 2) & 3;
                uint32_t sec;
                if (lt <= 1) {
                    const uint32_t lh = sf == 1 ? 2 : sf == 3 ? 3 : 1;
                    const uint32_t sz = sf == 1 ? (b0 | B(ip + 1) << 8) >> 4
                                      : sf == 3 ? (b0 | B(ip + 1) << 8 | B(ip + 2) << 16) >> 4
                                                : b0 >> 3;
                    sec = lt == 0 ? lh + sz : lh + 1;
                } else {
                    const uint32_t lhc = b0 | B(ip + 1) << 8 | B(ip + 2) << 16 | B(ip + 3) << 24;
                    sec = sf <= 1 ? 3 + ((lhc >> 14) & 0x3FF) : sf == 2 ? 4 + (lhc >> 18)
                                                                      : 5 + (lhc >> 22) + (B(ip + 4) << 10);
                }
                if (sec < bsize) {
                    const uint32_t q = ip + sec, s0 = B(q);
                    const uint32_t nseq = s0 < 128 ? s0 : s0 < 255 ? ((s0 - 128) << 8) + B(q + 1)
                                                                   : (B(q + 1) | B(q + 2) << 8) + 0x7F00;
                    items += 2ull * nseq + (2ull * nseq + 62) / 63;
                }
            }
            ip += type == 1 ? 1 : bsize;
            if ((bh & 1) || ip > clen)
                break;
        }
        if (ip > clen)
            break;
        if ((fhd >> 2) & 1) {
            ip += 4;
            *cks = true;   // a content checksum: the check kernel runs
        }
    }
    *bound = (uint32_t)((items + 3) & ~3ull);
    *bblk = blocks;
}

void zstd_host_plan(const FrameDesc *h_desc, const uint8_t *h_comp, uint32_t nframes, uint64_t *h_plan,
                    ZstdHostPlan *P)
{
    uint64_t items = 0, blocks = 0, extent = 0, dmax = 0;
    uint64_t *const rb = h_plan, *const bb = h_plan + nframes + 1;
    bool cks = false;
    for (uint32_t f = 0; f < nframes; f++) {
        const FrameDesc &d = h_desc[f];
        uint32_t bound = 0, bblk = 0;
        zstd_plan_frame_host(h_comp + d.c_off, d.c_size, &bound, &bblk, &cks);
        rb[f] = items;
        bb[f] = blocks;
        items += bound;
        blocks += bblk;
        extent = std::max<uint64_t>(extent, d.d_off + d.d_size);
        dmax = std::max<uint64_t>(dmax, d.d_size);
    }
    rb[nframes] = items;
    bb[nframes] = blocks;
    *P = ZstdHostPlan{items, blocks, extent, dmax, cks};
}

int zstd_decode_frames_planned(const ZstdHostPlan &P, const uint64_t *d_plan, const FrameDesc *d_desc,
                               uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out, int32_t *d_status,
                               ZstdScratch *s, hipStream_t stream, uint32_t *d_fail_at, uint32_t stop_last)
{
    if (nframes == 0)
        return 0;
    if (nframes > kOneMaxFrames || zstd_chunks(nframes) != 1)
        return zstd_decode_frames(d_desc, nframes, d_comp, d_out, d_status, s, stream, d_fail_at, stop_last);
    (void)hipGetLastError();   // a stale error of an earlier call is not this launch's
    stage_mark(0, stream);
    if (zstd_scratch_reserve(s, nframes, P.extent, P.items, P.blocks, stream) != 0)
        return -1;
    s->total[0] = P.items;
    s->total[1] = P.extent;
    s->total[2] = P.blocks;
    s->total[3] = P.dmax;
    s->total[4] = 0;   // one chunk: blocks [0, blocks)
    s->total[5] = P.blocks;
    stage_mark(1, stream);
    // this launch's kernels take both offset arrays from the plan's upload
    // (the scratch's own arrays are left alone)
    uint64_t *const keep_rb = s->rec_base, *const keep_bb = s->blk_base;
    s->rec_base = const_cast<uint64_t *>(d_plan);
    s->blk_base = const_cast<uint64_t *>(d_plan) + nframes + 1;
    const int rc =
        launch_zstd_decode(d_desc, nframes, d_comp, d_out, d_status, s, stream, d_fail_at, stop_last, P.cks);
    s->rec_base = keep_rb;
    s->blk_base = keep_bb;
    return rc;
}

int zstd_decode_frames_host(const FrameDesc *h_desc, const uint8_t *h_comp, const FrameDesc *d_desc,
                            uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out, int32_t *d_status,
                            ZstdScratch *s, hipStream_t stream, uint32_t *d_fail_at, uint32_t stop_last)
{
    if (nframes == 0)
        return 0;
    if (nframes > kOneMaxFrames || zstd_chunks(nframes) != 1)
        return zstd_decode_frames(d_desc, nframes, d_comp, d_out, d_status, s, stream, d_fail_at, stop_last);
    if (2ull * (nframes + 1) > s->h_plan_cap) {
        if (s->h_plan)
            (void)hipHostFree(s->h_plan);
        if (s->d_plan)
            (void)hipFree(s->d_plan);
        s->h_plan = s->d_plan = nullptr;
        s->h_plan_cap = 0;
        if (hipHostMalloc((void **)&s->h_plan, 2 * (kOneMaxFrames + 1) * sizeof(uint64_t), hipHostMallocDefault) !=
                hipSuccess ||
            hipMalloc((void **)&s->d_plan, 2 * (kOneMaxFrames + 1) * sizeof(uint64_t)) != hipSuccess)
            return -1;
        s->h_plan_cap = 2 * (kOneMaxFrames + 1);
    }
    // (a previous call's upload from h_plan must be done before it is rewritten)
    if (hipStreamSynchronize(stream) != hipSuccess)
        return -1;
    ZstdHostPlan P;
    zstd_host_plan(h_desc, h_comp, nframes, s->h_plan, &P);
    if (hipMemcpyAsync(s->d_plan, s->h_plan, 2 * (nframes + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, stream) !=
        hipSuccess)
        return -1;
    return zstd_decode_frames_planned(P, s->d_plan, d_desc, nframes, d_comp, d_out, d_status, s, stream, d_fail_at,
                                      stop_last);
}

}   // namespace zsk
