// zstd_decode.hip — zstd frame decoding on the GPU (gfx950), the reference's
// ZSTD_decompressDCtx / ZSTD_decompressStream call (decompress.c:434-538;
// libzstd 1.4.9, restated in oracle/zstd_oracle.c).
//
// Three launches per batch, then the LZ4 path's execute kernel:
//
//   zstd_plan_kernel   one LANE per frame: walks frame and block headers and
//                      each block's sequence count -> an exact bound on the
//                      frame's 8-byte sequence items; zstd_scan_kernel turns
//                      the bounds into slot offsets;
//   zstd_frame_kernel  one WAVE per frame: headers (wave-uniform, read from
//                      256-byte windows staged in LDS), Huffman tables and the
//                      three FSE tables (built in LDS, rank assignment
//                      wave-parallel by ballots), Huffman literals (one lane
//                      per stream) into a literal scratch laid out like the
//                      output, and the sequences (lane 0) -> items: literal
//                      source, lengths and the resolved offset (repeat offsets
//                      applied), with every libzstd validation; raw / RLE
//                      blocks become literal runs;
//   seq_exec_kernel    (seq_exec.hip) copies literal runs and matches;
//   zstd_check_kernel  XXH64 content checksums, for frames that carry one.
//
// Every backward bitstream is read by one lane through a 2 KiB LDS ring that
// the wave refills 512 bytes at a time with global_load_lds (no VGPRs held
// while the bytes are in flight; the ring is refilled long before the reader
// reaches the new bytes).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "lz4_dev.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4d;

constexpr uint32_t kZMagic = 0xFD2FB528u;
constexpr uint32_t kZBlockMax = 128u << 10;
constexpr uint32_t kZW = 2;          // waves (frames) per workgroup
constexpr uint32_t kRing = 2048;     // bitstream ring bytes per reader
constexpr uint32_t kSeg = 512;       // refill unit
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

// LDS per wave
struct ZLds {
    uint16_t huf[4096];       // Huffman X1 cells: symbol | nbits << 8
    uint32_t fse[3][512];     // LL / OF / ML cells: symbol | nbits << 8 | base << 16
    uint8_t ring[4][kRing];   // backward bitstream rings, one per reader lane
    uint8_t win[256];         // forward window: headers, table descriptions
    uint32_t wfse[64];        // FSE table of compressed Huffman weights
    int16_t norm[256];        // normalized counts
    uint8_t wts[256];         // Huffman weights
    uint32_t cnt[256];        // per-symbol next-state counters
    uint8_t lbuf[4][256];     // decoded literals of the 4 Huffman streams, staged
    uint32_t rank[16];        // Huffman: first cell of each weight
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
    const uint32_t a = (I.s0 + p) & ~3u;
    dma256(I, a, ldsaddr(L.win));
    dma_wait();
    return a;
}

__device__ __forceinline__ uint32_t wb(const ZLds &L, uint32_t wx, const In &I, uint32_t p)
{
    return *lp<uint8_t>(L.win + (I.s0 + p - wx));
}

// forward bits [bit, bit + n) (n <= 16) of the window, LSB first
__device__ __forceinline__ uint32_t win_bits(const ZLds &L, uint32_t bit, uint32_t n)
{
    const uint32_t b = bit >> 3;
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 4; i++)
        v |= (b + i < 256 ? (uint32_t)*lp<uint8_t>(L.win + b + i) : 0u) << (8 * i);
    return (v >> (bit & 7)) & ((1u << n) - 1);
}

// ---- backward bitstreams through LDS rings ----------------------------------
// A lane's stream bytes sit in its ring; the bits it reads next sit in a
// 64-bit register container C, refilled 32 bits at a time: C holds stream
// bits [pos, pos + nb), the next bit read being bit pos + nb - 1.
struct Rd {
    uint32_t ring;   // LDS address of this lane's ring
    uint32_t x0;     // coordinate of stream byte 0
    uint32_t rlo;    // the ring holds coordinates [rlo, rlo + kRing) (rlo multiple of kSeg)
    int32_t pos;     // lowest stream bit in C (< 0: zeros below the stream's start)
    int32_t nb;      // valid bits in C
    uint64_t C;
};

__device__ __forceinline__ uint32_t ring_dw(const Rd &r, uint32_t a)
{
    return *la<uint32_t>(r.ring + (a & (kRing - 1)));
}

// n (1..32) stream bits at bit lo >= 0
__device__ __forceinline__ uint32_t bits_at(const Rd &r, int32_t lo, uint32_t n)
{
    const uint32_t b = r.x0 + ((uint32_t)lo >> 3), a = b & ~3u;
    const uint64_t q = (uint64_t)ring_dw(r, a) | ((uint64_t)ring_dw(r, a + 4) << 32);
    const uint32_t sh = (b & 3) * 8 + ((uint32_t)lo & 7);
    return (uint32_t)((q >> sh) & ((1ull << n) - 1));
}

// make C hold >= 32 bits (bits below the stream's start read as 0)
__device__ __forceinline__ void rd_fill(Rd &r)
{
    if (r.nb < 32) {
        r.pos -= 32;
        const uint32_t v = r.pos >= 0 ? bits_at(r, r.pos, 32)
                         : r.pos > -32 ? bits_at(r, 0, (uint32_t)(32 + r.pos)) << (uint32_t)(-r.pos)
                                       : 0u;
        r.C = (r.C << 32) | v;
        r.nb += 32;
    }
}

// the next n (<= nb) bits, not consumed
__device__ __forceinline__ uint32_t rd_look(const Rd &r, uint32_t n)
{
    return (uint32_t)(r.C >> (uint32_t)(r.nb - (int32_t)n)) & (uint32_t)((1ull << n) - 1);
}

__device__ __forceinline__ uint32_t rd_read(Rd &r, uint32_t n)
{
    if (n == 0)
        return 0;
    if (r.nb < (int32_t)n)
        rd_fill(r);
    const uint32_t v = rd_look(r, n);
    r.nb -= (int32_t)n;
    return v;
}

// stream bits not consumed yet (< 0 once read past the start)
__device__ __forceinline__ int32_t rd_left(const Rd &r)
{
    return r.pos + r.nb;
}

// Start one stream per active lane: [xs, xs + len) (len >= 1).  Wave-wide.
// Returns false on a lane whose stream has no end mark.
__device__ __forceinline__ bool rd_init(const In &I, Rd &r, bool act, uint32_t ring, uint32_t xs,
                                        uint32_t len)
{
    r.ring = ring;
    r.x0 = xs;
    const uint32_t end = xs + len;
    r.rlo = ((end - 1) & ~(kSeg - 1)) - (kRing - kSeg);
    uint64_t m = __ballot(act);
    while (m) {
        const int j = __builtin_ctzll(m);
        m &= m - 1;
        const uint32_t rlo = lane_val(r.rlo, j), rg = lane_val(ring, j);
        for (uint32_t k = 0; k < kRing; k += 256)
            dma256(I, rlo + k, rg + ((rlo + k) & (kRing - 1)));
    }
    dma_wait();
    if (!act)
        return true;
    const uint32_t last = *la<uint8_t>(ring + ((end - 1) & (kRing - 1)));
    r.pos = last ? (int32_t)(8 * (len - 1)) + hibit(last) : 0;
    r.nb = 0;
    r.C = 0;
    return last != 0;
}

// Keep every active lane's ring ahead of its reader: when the reader is
// within 128 bytes (more than a reader consumes between two calls) of the
// ring's lowest segment, which may still be in flight, wait for the loads in
// flight and request the next 512 bytes below.  Wave-wide.
__device__ __forceinline__ void rd_refill(const In &I, Rd &r, bool act)
{
    const int32_t bmin = (int32_t)r.x0 + (r.pos >> 3) - 128;
    const bool need = act && (int32_t)r.rlo > (int32_t)r.x0 && bmin < (int32_t)(r.rlo + kSeg);
    uint64_t m = __ballot(need);
    if (!m)
        return;
    dma_wait();
    while (m) {
        const int j = __builtin_ctzll(m);
        m &= m - 1;
        const uint32_t a = lane_val(r.rlo, j) - kSeg, rg = lane_val(r.ring, j);
        dma256(I, a, rg + (a & (kRing - 1)));
        dma256(I, a + 256, rg + ((a + 256) & (kRing - 1)));
    }
    if (need)
        r.rlo -= kSeg;
}

// ---- FSE tables -----------------------------------------------------------------
// Normalized counts from the window at bit 0 of frame offset p (lane 0),
// RFC 8878 §4.1.1 / FSE_readNCount.  Returns bytes used, or 0 on error
// (*err set).  norm[] receives nsym entries.
__device__ __forceinline__ uint32_t read_ncount(ZLds &L, uint32_t wofs, uint32_t avail, uint32_t max_sym,
                                uint32_t max_log, uint32_t *tlog, uint32_t *nsym, uint32_t *err)
{
    uint32_t pos = 8 * wofs;
    const uint32_t tl = win_bits(L, pos, 4) + 5;
    pos += 4;
    if (tl > max_log) {
        *err = ZE_CORRUPT;
        return 0;
    }
    int32_t remaining = (1 << tl) + 1, threshold = 1 << tl;
    uint32_t nbits = tl + 1, sym = 0;
    bool prev0 = false;
    for (uint32_t i = 0; i <= max_sym; i++)
        L.norm[i] = 0;
    while (remaining > 1 && sym <= max_sym) {
        if (prev0) {
            uint32_t n0 = sym;
            while (win_bits(L, pos, 16) == 0xFFFF) {
                n0 += 24;
                pos += 16;
            }
            while (win_bits(L, pos, 2) == 3) {
                n0 += 3;
                pos += 2;
            }
            n0 += win_bits(L, pos, 2);
            pos += 2;
            if (n0 > max_sym) {
                *err = ZE_CORRUPT;
                return 0;
            }
            while (sym < n0)
                L.norm[sym++] = 0;
        }
        const int32_t mx = 2 * threshold - 1 - remaining;
        const int32_t v = (int32_t)win_bits(L, pos, nbits);
        int32_t count;
        if ((v & (threshold - 1)) < mx) {
            count = v & (threshold - 1);
            pos += nbits - 1;
        } else {
            count = v & (2 * threshold - 1);
            if (count >= threshold)
                count -= mx;
            pos += nbits;
        }
        count--;
        remaining -= count < 0 ? -count : count;
        L.norm[sym++] = (int16_t)count;
        prev0 = count == 0;
        while (remaining < threshold) {
            nbits--;
            threshold >>= 1;
        }
        if (pos > 8 * 256) {   // ran off the window: no valid description is that long
            *err = ZE_CORRUPT;
            return 0;
        }
    }
    const uint32_t used = (pos + 7) / 8 - wofs;
    if (remaining != 1 || used > avail) {
        *err = ZE_CORRUPT;
        return 0;
    }
    *tlog = tl;
    *nsym = sym;
    return used;
}

// Decoding table from norm[0..nsym) with accuracy log tl: symbol spread by
// lane 0, next states assigned wave-parallel (per 64-cell group, one ballot
// per distinct symbol, cells ranked in position order).  Wave-wide.
__device__ __forceinline__ void fse_build(ZLds &L, uint32_t *tab, uint32_t nsym, uint32_t tl)
{
    const uint32_t lane = lane_id();
    const uint32_t size = 1u << tl, mask = size - 1;
    wave_lds_sync();   // norm[] from lane 0
    if (lane == 0) {
        uint32_t high = size - 1;
        for (uint32_t s = 0; s < nsym; s++)
            if (L.norm[s] == -1)
                *lp<uint32_t>(tab + high--) = s;
        const uint32_t step = (size >> 1) + (size >> 3) + 3;
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
                const uint32_t ns = base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
                const uint32_t nb = tl - (uint32_t)hibit(ns);
                *lp<uint32_t>(tab + u) = sj | nb << 8 | ((ns << nb) - size) << 16;
            }
            if (lane == 0)
                L.cnt[sj] = base + (uint32_t)__builtin_popcountll(m);
            wave_lds_sync();
            rem &= ~m;
        }
    }
}

// ---- Huffman tables --------------------------------------------------------------
// Tree description at frame offset p (window staged at wx); returns its size
// or 0 on error.  Builds L.huf; *log receives the table log.  Wave-wide.
__device__ __forceinline__ uint32_t huf_read(ZLds &L, const In &I, uint32_t wx, uint32_t p, uint32_t avail,
                             uint32_t *log)
{
    const uint32_t lane = lane_id();
    const uint32_t hb = uni(wb(L, wx, I, p));
    const uint32_t wofs = I.s0 + p - wx + 1;   // window offset of the description body
    uint32_t nw = 0, used = 0, err = 0;
    if (hb < 128) {
        if (1 + hb > avail || wofs + hb > 256)
            return 0;
        uint32_t tl = 0, nsym = 0;
        uint32_t hs = 0;
        if (lane == 0)
            hs = read_ncount(L, wofs, hb, 255, 6, &tl, &nsym, &err);
        hs = uni(hs);
        if (uni(err))
            return 0;
        tl = uni(tl);
        nsym = uni(nsym);
        fse_build(L, L.wfse, nsym, tl);
        if (lane == 0) {
            // backward stream inside the window: two interleaved states
            const uint32_t b0 = wofs + hs, bn = hb - hs;
            const uint32_t lastb = bn ? *lp<uint8_t>(L.win + b0 + bn - 1) : 0;
            if (!lastb) {
                err = 1;
            } else {
                int32_t pos = (int32_t)(8 * (bn - 1)) + hibit(lastb);
                auto rb = [&](uint32_t n) -> uint32_t {
                    pos -= (int32_t)n;
                    uint32_t v = 0;
                    for (uint32_t i = 0; i < n; i++) {
                        const int32_t bit = pos + (int32_t)i;
                        if (bit >= 0 && ((*lp<uint8_t>(L.win + b0 + (bit >> 3)) >> (bit & 7)) & 1))
                            v |= 1u << i;
                    }
                    return v;
                };
                uint32_t s1 = rb(tl), s2 = rb(tl);
                for (;;) {
                    if (nw > 253) {
                        err = 1;
                        break;
                    }
                    uint32_t c = *lp<uint32_t>(L.wfse + s1);
                    L.wts[nw++] = (uint8_t)c;
                    s1 = (c >> 16) + rb((c >> 8) & 0xFF);
                    if (pos < 0) {
                        L.wts[nw++] = (uint8_t)*lp<uint32_t>(L.wfse + s2);
                        break;
                    }
                    if (nw > 253) {
                        err = 1;
                        break;
                    }
                    c = *lp<uint32_t>(L.wfse + s2);
                    L.wts[nw++] = (uint8_t)c;
                    s2 = (c >> 16) + rb((c >> 8) & 0xFF);
                    if (pos < 0) {
                        L.wts[nw++] = (uint8_t)*lp<uint32_t>(L.wfse + s1);
                        break;
                    }
                }
            }
        }
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
    // first cell of each weight class: classes in increasing weight order
    if (lane == 0) {
        uint32_t cntw[13];
        for (uint32_t k = 0; k <= 12; k++)
            cntw[k] = 0;
        for (uint32_t s = 0; s < nw; s++)
            cntw[L.wts[s]]++;
        uint32_t acc = 0;
        for (uint32_t k = 1; k <= lg; k++) {
            L.rank[k] = acc;
            acc += cntw[k] << (k - 1);
        }
    }
    wave_lds_sync();
    // cells: symbols in order, each takes 2^(w-1) cells of its class
    for (uint32_t s = 0; s < nw; s++) {
        const uint32_t w = uni(L.wts[s]);
        if (!w)
            continue;
        const uint32_t len = (1u << w) >> 1;
        const uint32_t c0 = uni(L.rank[w]);
        const uint16_t e = (uint16_t)(s | (lg + 1 - w) << 8);
        for (uint32_t c = lane; c < len; c += 64)
            L.huf[c0 + c] = e;
        if (lane == 0)
            L.rank[w] = c0 + len;
        wave_lds_sync();
    }
    *log = lg;
    return used;
}

// ---- items (format: lz4_split.hip Sink; full offset in extended items) ------------
struct Sink {
    uint64_t *base;
    uint32_t k, cap;
};

// lane 0 only
__device__ __forceinline__ bool emit(Sink &S, uint32_t src, uint32_t lit, uint32_t off, uint32_t ml)
{
    if (lit > 255 || ml > 258 || (ml != 0 && ml < 4) || off > 0xFFFF) {
        const uint32_t pad = (S.k & 63) == 63 ? 1 : 0;
        if (S.k + pad + 2 > S.cap)
            return false;
        if (pad)
            S.base[S.k++] = 0;
        S.base[S.k++] = ((uint64_t)off << 32) | src | kItemExt;
        S.base[S.k++] = ((uint64_t)ml << 32) | lit;
        return true;
    }
    if (S.k + 1 > S.cap)
        return false;
    S.base[S.k++] = ((uint64_t)(off | lit << 16 | (ml ? ml - 3 : 0) << 24) << 32) | src;
    return true;
}

// ---- literals ---------------------------------------------------------------------------
struct Frame {
    In I;
    uint32_t codes;    // LDS: literal-length codes [0, 36), match-length codes [36, 89)
    bool timed;
    uint64_t tm, t[4]; // section timers (timing builds): literals, tables, sequences, rest
    uint32_t clen;     // compressed entry bytes
    uint8_t *lit;      // literal scratch of this frame (laid out like its output)
    uint32_t cap;      // output capacity (seek-table dSize)
    uint32_t lo;       // literal bytes decoded into the scratch
    uint32_t o;        // output bytes accounted for
    uint32_t huf_log;  // 0: no Huffman table yet
    uint32_t tlog[3];  // LL / OF / ML table logs (valid flags below)
    uint32_t tvalid;   // bit t: table t valid
    uint32_t rep0, rep1, rep2;
};

__device__ __forceinline__ void zmark(Frame &F, int i)
{
    if (F.timed) {
        const uint64_t t = __builtin_readcyclecounter();
        F.t[i] += t - F.tm;
        F.tm = t;
    }
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

// Huffman streams: lane l < ns decodes stream l into [dst, dst + cnt)
__device__ __forceinline__ bool huf_streams(ZLds &L, Frame &F, uint32_t ns, uint32_t x_s, const uint32_t *len,
                            uint32_t dst0, uint32_t size)
{
    const uint32_t lane = lane_id();
    const uint32_t seg = ns == 1 ? size : (size + 3) / 4;
    const bool act = lane < ns;
    uint32_t xs = x_s, sl = 0, dst = dst0, cnt = 0;
    for (uint32_t k = 0; k < ns; k++) {
        if (lane == k) {
            sl = len[k];
            dst = dst0 + k * seg;
            cnt = k + 1 < ns ? seg : size - k * seg;
        }
        if (lane > k)
            xs += len[k];
    }
    Rd r;
    const bool ok = rd_init(F.I, r, act && sl > 0, ldsaddr(L.ring[lane & 3]), xs, sl ? sl : 1);
    bool bad = act && (sl == 0 || !ok);
    if (__ballot(bad))
        return false;
    const uint32_t lg = F.huf_log;
    const uint32_t maxc = uni(__builtin_amdgcn_readlane(cnt, 0));   // stream 0 is the longest
    // decoded bytes go to a 256-byte LDS buffer per stream, one ds_write_b8
    // per symbol; every 256 symbols the wave copies the buffers out (4 bytes
    // per lane, coalesced)
    const uint32_t lb = ldsaddr(L.lbuf[lane & 3]);
    auto flush = [&](uint32_t i0, uint32_t m) {   // symbols [i0, i0 + m) of every stream
        wave_lds_sync();   // lbuf[k] written by lane k, read by all
        for (uint32_t k = 0; k < ns; k++) {
            const uint32_t ck = lane_val(cnt, (int)k), dk = lane_val(dst, (int)k);
            const uint32_t mk = ck > i0 ? (ck - i0 < m ? ck - i0 : m) : 0;
            if (4 * lane < mk) {
                const uint32_t v = *la<uint32_t>(ldsaddr(L.lbuf[k]) + 4 * lane);
                lit_put(F, dk + i0 + 4 * lane, (u32x4){v, 0, 0, 0}, mk - 4 * lane < 4 ? mk - 4 * lane : 4);
            }
        }
        wave_lds_sync();   // before lane k writes lbuf[k] again
    };
    uint32_t i = 0;
    for (; i < maxc; i++) {
        if ((i & 63) == 0)
            rd_refill(F.I, r, act);
        if (act && i < cnt) {
            rd_fill(r);
            const uint32_t e = L.huf[rd_look(r, lg)];
            r.nb -= (int32_t)(e >> 8);
            *la<uint8_t>(lb + (i & 255)) = (uint8_t)e;
        }
        if ((i & 255) == 255)
            flush(i - 255, 256);
    }
    if (maxc & 255)
        flush(maxc & ~255u, maxc & 255);
    bad = act && rd_left(r) != 0;
    return !__ballot(bad);
}

// Literals section at frame offset p (block bytes [p, p + n)); *used, *litn.
// Returns 0 or a zstd error.  Wave-wide.
__device__ __forceinline__ uint32_t literals(ZLds &L, Frame &F, uint32_t p, uint32_t n, uint32_t *used,
                             uint32_t *litn)
{
    const uint32_t lane = lane_id();
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
        uint32_t lg = 0;
        const uint32_t hs = huf_read(L, F.I, wx, q, qn, &lg);
        if (!hs)
            return ZE_CORRUPT;
        F.huf_log = lg;
        q += hs;
        qn -= hs;
    } else if (!F.huf_log) {
        return ZE_DICT_CORRUPT;
    }
    uint32_t len[4];
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
    if (!huf_streams(L, F, ns, F.I.s0 + q, len, F.lo, size))
        return ZE_CORRUPT;
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
        if (lane == 0)
            used = read_ncount(L, F.I.s0 + p - wx, avail, max_sym, max_log, &tl, &nsym, &e);
        if (uni(e) || uni(used) == 0) {
            *err = ZE_CORRUPT;
            return ~0u;
        }
        fse_build(L, tab, uni(nsym), uni(tl));
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

// One compressed block [p, p + n) -> items.  Returns 0 or a zstd error.
__device__ __forceinline__ uint32_t block(ZLds &L, Frame &F, Sink &S, uint32_t p, uint32_t n)
{
    const uint32_t lane = lane_id();
    if (n >= kZBlockMax)
        return ZE_SRC_WRONG;
    uint32_t lused = 0, litn = 0;
    zmark(F, 3);
    uint32_t e = literals(L, F, p, n, &lused, &litn);
    zmark(F, 0);
    if (e)
        return e;
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
    uint32_t o = F.o, lp_ = F.lo;
    const uint32_t le = F.lo + litn;
    bool full = false;
    if (nseq) {
        if (q + 1 > qe)
            return ZE_SRC_WRONG;
        const uint32_t modes = uni(wb(L, wx, F.I, q));
        q++;
        const uint32_t mode[3] = {modes >> 6, (modes >> 4) & 3, (modes >> 2) & 3};
#pragma unroll
        for (uint32_t t = 0; t < 3; t++) {
            uint32_t err = 0;
            const uint32_t u = seq_table(L, F, t, mode[t], q, qe - q, &err);
            if (u == ~0u)
                return err;
            q += u;
        }
        zmark(F, 1);
        Rd r;
        const bool ok = rd_init(F.I, r, lane == 0, ldsaddr(L.ring[0]), F.I.s0 + q, qe > q ? qe - q : 1);
        if (!uni(ok && qe > q ? 1u : 0u))
            return ZE_CORRUPT;
        uint32_t sll = 0, sof = 0, sml = 0, err = 0;
        uint32_t rep0 = F.rep0, rep1 = F.rep1, rep2 = F.rep2;
        if (lane == 0) {
            sll = rd_read(r, F.tlog[0]);
            sof = rd_read(r, F.tlog[1]);
            sml = rd_read(r, F.tlog[2]);
        }
        for (uint32_t i = 0; i < nseq; i++) {
            if ((i & 7) == 0)   // <= 8 sequences x 12 bytes < the refill margin
                rd_refill(F.I, r, lane == 0);
            if (lane == 0 && !err) {
                const uint32_t cll = *lp<uint32_t>(L.fse[0] + sll), cof = *lp<uint32_t>(L.fse[1] + sof),
                               cml = *lp<uint32_t>(L.fse[2] + sml);
                const uint32_t llc = cll & 0xFF, ofc = cof & 0xFF, mlc = cml & 0xFF;
                if (llc > 35 || ofc > 31 || mlc > 52) {
                    err = ZE_CORRUPT;
                } else {
                    const uint64_t ofv = (1ull << ofc) + rd_read(r, ofc);
                    const uint32_t mlcode = *la<uint32_t>(F.codes + 4 * (36 + mlc)),
                                   llcode = *la<uint32_t>(F.codes + 4 * llc);
                    const uint32_t ml = (mlcode & 0xFFFFFF) + rd_read(r, mlcode >> 24);
                    const uint32_t ll = (llcode & 0xFFFFFF) + rd_read(r, llcode >> 24);
                    uint64_t off;
                    if (ofv > 3) {
                        off = ofv - 3;
                        rep2 = rep1;
                        rep1 = rep0;
                        rep0 = (uint32_t)off;
                    } else {
                        const uint32_t idx = (uint32_t)ofv - 1 + (ll == 0);
                        if (idx == 0) {
                            off = rep0;
                        } else {
                            off = idx == 1 ? rep1 : idx == 2 ? rep2 : rep0 - 1;
                            if (off == 0)
                                off = 1;
                            if (idx != 1)
                                rep2 = rep1;
                            rep1 = rep0;
                            rep0 = (uint32_t)off;
                        }
                    }
                    sll = (cll >> 16) + rd_read(r, (cll >> 8) & 0xFF);
                    sml = (cml >> 16) + rd_read(r, (cml >> 8) & 0xFF);
                    sof = (cof >> 16) + rd_read(r, (cof >> 8) & 0xFF);
                    if ((uint64_t)o + ll + ml > F.cap)
                        err = ZE_DST_SMALL;
                    else if (le - lp_ < ll)
                        err = ZE_CORRUPT;
                    else if (off > (uint64_t)o + ll)
                        err = ZE_CORRUPT;
                    else if (!emit(S, lp_, ll, (uint32_t)off, ml))
                        full = true, err = ZE_GENERIC;
                    lp_ += ll;
                    o += ll + ml;
                }
            }
            if (uni(err))
                break;
        }
        zmark(F, 2);
        err = uni(err);
        if (err)
            return err;
        if (uni(lane == 0 && rd_left(r) > 0 ? 1u : 0u))
            return ZE_CORRUPT;
        F.rep0 = uni(rep0);
        F.rep1 = uni(rep1);
        F.rep2 = uni(rep2);
        o = uni(o);
        lp_ = uni(lp_);
    }
    const uint32_t last = le - lp_;
    if (o + last > F.cap)
        return ZE_DST_SMALL;
    if (last) {
        uint32_t ok = 1;
        if (lane == 0)
            ok = emit(S, lp_, last, 0, 0);
        if (!uni(ok))
            return ZE_GENERIC;
    }
    (void)full;
    S.k = uni(S.k);
    F.o = o + last;
    F.lo = le;
    return 0;
}

// literal-only item for a raw / RLE block already in the scratch at F.lo
__device__ __forceinline__ bool run_item(Sink &S, uint32_t src, uint32_t n)
{
    uint32_t ok = 1;
    if (lane_id() == 0 && n)
        ok = emit(S, src, n, 0, 0);
    S.k = uni(S.k);
    return uni(ok) != 0;
}

// One seek-table entry: every zstd frame in it (ZSTD_decompressDCtx).
__device__ __forceinline__ int32_t decode_entry(ZLds &L, Frame &F, Sink &S, uint32_t clen, uint64_t *ck)
{
    const uint32_t lane = lane_id();
    uint32_t ip = 0, frames = 0;
    bool summed = false;   // a checksummed frame was decoded: it must be the entry's last
    while (clen - ip >= 5) {
        if (summed)
            return zerr(ZE_GENERIC);
        uint32_t wx = stage_win(L, F.I, ip);
        auto B = [&](uint32_t i) { return uni(wb(L, wx, F.I, ip + i)); };
        const uint32_t magic = B(0) | B(1) << 8 | B(2) << 16 | B(3) << 24;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            if (clen - ip < 8)
                return zerr(ZE_SRC_WRONG);
            const uint64_t sk = 8 + (uint64_t)(B(4) | B(5) << 8 | B(6) << 16 | B(7) << 24);
            if (sk > clen - ip)
                return zerr(ZE_SRC_WRONG);
            ip += (uint32_t)sk;
            continue;
        }
        if (magic != kZMagic)
            return zerr(frames ? ZE_SRC_WRONG : ZE_PREFIX);
        frames++;
        const uint32_t n = clen - ip;
        if (n < 9)
            return zerr(ZE_SRC_WRONG);
        const uint32_t fhd = B(4);
        const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, csum = (fhd >> 2) & 1,
                       did = fhd & 3;
        const uint32_t dsz = did == 3 ? 4 : did;
        const uint32_t hsize = 5 + !single + dsz + (fcs_flag == 0 ? single : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8);
        if (n < hsize + 3)
            return zerr(ZE_SRC_WRONG);
        if (fhd & 0x08)
            return zerr(ZE_FRAMEPARAM);
        uint32_t h = 5;
        if (!single) {
            if ((B(h) >> 3) + 10 > 31)
                return zerr(ZE_WINDOW);
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
            return zerr(ZE_DICT_WRONG);
        ip += hsize;
        // frame state
        F.huf_log = 0;
        F.tvalid = 0;
        F.rep0 = 1;
        F.rep1 = 4;
        F.rep2 = 8;
        const uint32_t o0 = F.o;
        for (;;) {
            if (clen - ip < 3)
                return zerr(ZE_SRC_WRONG);
            wx = stage_win(L, F.I, ip);
            const uint32_t bh = B(0) | B(1) << 8 | B(2) << 16;
            const uint32_t lastb = bh & 1, type = (bh >> 1) & 3, bsize = bh >> 3;
            const uint32_t csz = type == 1 ? 1 : bsize;
            if (type == 3)
                return zerr(ZE_CORRUPT);
            ip += 3;
            if (csz > clen - ip)
                return zerr(ZE_SRC_WRONG);
            if (type == 0 || type == 1) {
                if (bsize > F.cap - F.o)
                    return zerr(ZE_DST_SMALL);
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
                if (!run_item(S, F.lo, bsize))
                    return zerr(ZE_GENERIC);
                F.lo += bsize;
                F.o += bsize;
            } else {
                const uint32_t e = block(L, F, S, ip, bsize);
                if (e)
                    return zerr(e);
            }
            ip += csz;
            if (lastb)
                break;
        }
        if (fcs != ~0ull && F.o - o0 != fcs)
            return zerr(ZE_CORRUPT);
        if (csum) {
            if (clen - ip < 4)
                return zerr(ZE_CHECKSUM);
            wx = stage_win(L, F.I, ip);
            const uint32_t want = B(0) | B(1) << 8 | B(2) << 16 | B(3) << 24;
            *ck = (1ull << 63) | ((uint64_t)o0 << 32) | want;   // covers [o0, dSize)
            summed = true;
            ip += 4;
        }
    }
    if (clen != ip)
        return zerr(ZE_SRC_WRONG);
    return F.o == F.cap ? ST_OK : ST_SHORT_FRAME;
}

// ---- kernels -------------------------------------------------------------------------------

// item bound per frame (lane per frame): 2 items per sequence + padding + 4 per block
__global__ __launch_bounds__(256) void zstd_plan_kernel(const FrameDesc *__restrict__ desc, uint32_t n,
                                                        const uint8_t *__restrict__ comp,
                                                        uint32_t *__restrict__ bound)
{
    const uint32_t f = blockIdx.x * 256 + threadIdx.x;
    if (f >= n)
        return;
    const FrameDesc d = desc[f];
    const Span sp = make_span(comp + d.c_off, d.c_size);
    auto B = [&](uint32_t p) -> uint32_t {
        return p < d.c_size ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(sp.r, sp.s0 + p, 0, 0) : 0u;
    };
    const uint32_t clen = d.c_size;
    uint64_t items = 8;
    uint32_t ip = 0;
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
}

// exclusive scan of per-frame bounds -> rec_base[0..n], item total and the
// output extent max(d_off + d_size) into total[0..1] (device memory, copied
// to the host by the launcher; one workgroup)
__global__ __launch_bounds__(1024) void zstd_scan_kernel(const FrameDesc *__restrict__ desc,
                                                         const uint32_t *__restrict__ bound, uint32_t n,
                                                         uint64_t *__restrict__ rec_base,
                                                         uint64_t *__restrict__ total)
{
    __shared__ uint64_t part[1024];
    __shared__ uint64_t ext[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t chunk = (n + 1023) / 1024;
    const uint32_t i0 = t * chunk < n ? t * chunk : n;
    const uint32_t i1 = i0 + chunk < n ? i0 + chunk : n;
    uint64_t s = 0, e = 0;
    for (uint32_t i = i0; i < i1; i++) {
        s += bound[i];
        const uint64_t x = desc[i].d_off + desc[i].d_size;
        e = x > e ? x : e;
    }
    part[t] = s;
    ext[t] = e;
    __syncthreads();
    for (uint32_t d = 512; d >= 1; d >>= 1) {
        if (t < d && ext[t + d] > ext[t])
            ext[t] = ext[t + d];
        __syncthreads();
    }
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - s;
    for (uint32_t i = i0; i < i1; i++) {
        rec_base[i] = run;
        run += bound[i];
    }
    if (t == 1023) {
        rec_base[n] = part[t];
        total[0] = part[t];
        total[1] = ext[0];
    }
}

__device__ unsigned long long g_ztime[4];   // timing builds: cycles per section

template <bool TIMED>
__global__ __launch_bounds__(64 * kZW) void zstd_frame_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    uint8_t *__restrict__ lit, uint64_t lit_cap, const uint64_t *__restrict__ rec_base,
    uint64_t capacity, uint64_t *__restrict__ items, uint32_t *__restrict__ nitems,
    int32_t *__restrict__ status, uint64_t *__restrict__ ck)
{
    __shared__ ZLds lds[kZW];
    __shared__ uint32_t codes[89];
    for (uint32_t i = threadIdx.x; i < 89; i += 64 * kZW)
        codes[i] = i < 36 ? c_ll[i] : c_ml[i - 36];
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    const uint32_t f = uni(blockIdx.x * kZW + w);
    if (f >= n)
        return;
    ZLds &L = lds[w];
    const FrameDesc d = desc[f];
    Frame F;
    F.codes = ldsaddr(codes);
    F.timed = TIMED;
    F.t[0] = F.t[1] = F.t[2] = F.t[3] = 0;
    F.tm = TIMED ? __builtin_readcyclecounter() : 0;
    const uintptr_t fa = reinterpret_cast<uintptr_t>(comp + d.c_off);
    F.I.base4 = reinterpret_cast<const uint8_t *>(fa & ~(uintptr_t)3);
    F.I.s0 = (uint32_t)(fa & 3);
    F.I.amax = d.c_size ? (F.I.s0 + d.c_size - 1) & ~3u : 0;
    F.lit = lit + d.d_off;
    F.clen = d.c_size;
    F.cap = d.d_size;
    F.lo = F.o = 0;
    F.huf_log = 0;
    F.tvalid = 0;
    F.rep0 = 1;
    F.rep1 = 4;
    F.rep2 = 8;
    F.tlog[0] = F.tlog[1] = F.tlog[2] = 0;
    Sink S;
    const uint64_t rb = rec_base[f];
    S.base = items + rb;
    S.k = 0;
    S.cap = (uint32_t)(rec_base[f + 1] - rb);
    uint64_t c = 0;
    int32_t st;
    // scratch sized by the plan: a frame that would not fit is refused, never
    // written out of bounds
    if (rec_base[f + 1] > capacity || d.c_size >= 0x7FFFFF00u ||
        d.d_off + (uint64_t)d.d_size + 16 > lit_cap)
        st = zerr(ZE_GENERIC);
    else
        st = decode_entry(L, F, S, d.c_size, &c);
    if (lane == 0) {
        status[f] = st;
        nitems[f] = S.k;
        ck[f] = c;
    }
    if (TIMED) {
        zmark(F, 3);
        if (lane == 0)
            for (int i = 0; i < 4; i++)
                atomicAdd(&g_ztime[i], (unsigned long long)F.t[i]);
    }
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
                                                         int32_t *__restrict__ status)
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
        if ((uint32_t)h != want)
            status[f] = zerr(ZE_CHECKSUM);
    }
}

}   // namespace

// ---- host side -----------------------------------------------------------------------------------

int zstd_scratch_reserve(ZstdScratch *s, uint32_t frames, uint64_t out_bytes, uint64_t items,
                         hipStream_t stream)
{
    (void)stream;
    if (frames + 1 > s->frames_cap) {
        const uint32_t cap = frames + 1 < 4096 ? 4096 : frames + 1;
        zstd_scratch_free(s);
        if (hipMalloc((void **)&s->bound, sizeof(uint32_t) * cap) != hipSuccess ||
            hipMalloc((void **)&s->rec_base, sizeof(uint64_t) * (cap + 1)) != hipSuccess ||
            hipMalloc((void **)&s->nitems, sizeof(uint32_t) * cap) != hipSuccess ||
            hipMalloc((void **)&s->ck, sizeof(uint64_t) * cap) != hipSuccess ||
            hipMalloc((void **)&s->d_total, 2 * sizeof(uint64_t)) != hipSuccess ||
            hipHostMalloc((void **)&s->total, 2 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess)
            return -1;
        s->total[0] = s->total[1] = 0;
        s->frames_cap = cap;
    }
    if (out_bytes + 64 > s->lit_cap) {
        if (s->lit)
            (void)hipFree(s->lit);
        s->lit = nullptr;
        s->lit_cap = 0;
        if (hipMalloc((void **)&s->lit, out_bytes + 64) != hipSuccess)
            return -1;
        s->lit_cap = out_bytes + 64;
    }
    if (items > s->items_cap) {
        if (s->items)
            (void)hipFree(s->items);
        s->items = nullptr;
        s->items_cap = 0;
        if (hipMalloc((void **)&s->items, items * sizeof(uint64_t)) != hipSuccess)
            return -1;
        s->items_cap = items;
    }
    return 0;
}

void zstd_scratch_free(ZstdScratch *s)
{
    if (s->bound)
        (void)hipFree(s->bound);
    if (s->rec_base)
        (void)hipFree(s->rec_base);
    if (s->nitems)
        (void)hipFree(s->nitems);
    if (s->ck)
        (void)hipFree(s->ck);
    if (s->lit)
        (void)hipFree(s->lit);
    if (s->items)
        (void)hipFree(s->items);
    if (s->d_total)
        (void)hipFree(s->d_total);
    if (s->total)
        (void)hipHostFree(s->total);
    *s = ZstdScratch();
}

// Plan only: bounds + offsets, then the item total and output extent copied
// into s->total (pinned host memory), valid once the stream reaches it.
int launch_zstd_plan(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                     ZstdScratch *s, hipStream_t stream)
{
    if (nframes == 0)
        return 0;
    hipLaunchKernelGGL(zstd_plan_kernel, dim3((nframes + 255) / 256), dim3(256), 0, stream, d_desc,
                       nframes, d_comp, s->bound);
    hipLaunchKernelGGL(zstd_scan_kernel, dim3(1), dim3(1024), 0, stream, d_desc, s->bound, nframes,
                       s->rec_base, s->d_total);
    if (hipGetLastError() != hipSuccess)
        return -1;
    return hipMemcpyAsync(s->total, s->d_total, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, stream) ==
                   hipSuccess
               ? 0
               : -1;
}

int launch_zstd_decode(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                       uint8_t *d_out, int32_t *d_status, ZstdScratch *s, hipStream_t stream)
{
    if (nframes == 0)
        return 0;
    static const bool timed = getenv("ZSEEK_ZSTD_TIMING") != nullptr;
    if (timed) {
        unsigned long long z[4] = {0, 0, 0, 0};
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_ztime), z, sizeof(z), 0, hipMemcpyHostToDevice, stream);
        hipLaunchKernelGGL(zstd_frame_kernel<true>, dim3((nframes + kZW - 1) / kZW), dim3(64 * kZW), 0,
                           stream, d_desc, nframes, d_comp, s->lit, s->lit_cap, s->rec_base, s->items_cap, s->items,
                           s->nitems, d_status, s->ck);
        (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_ztime), sizeof(z), 0, hipMemcpyDeviceToHost, stream);
        (void)hipStreamSynchronize(stream);
        const double t = (double)(z[0] + z[1] + z[2] + z[3]);
        fprintf(stderr, "zstd frame kernel (wave cycles): literals %.1f%%  tables %.1f%%  sequences %.1f%%  rest %.1f%%  total %.3g\n",
                100 * z[0] / t, 100 * z[1] / t, 100 * z[2] / t, 100 * z[3] / t, t);
    } else {
        hipLaunchKernelGGL(zstd_frame_kernel<false>, dim3((nframes + kZW - 1) / kZW), dim3(64 * kZW), 0,
                           stream, d_desc, nframes, d_comp, s->lit, s->lit_cap, s->rec_base, s->items_cap, s->items,
                           s->nitems, d_status, s->ck);
    }
    stage_mark(2, stream);
    const int rc = launch_seq_exec_lit(d_desc, nframes, s->lit, d_out, s->rec_base, s->items,
                                       s->nitems, d_status, stream);
    stage_mark(3, stream);
    hipLaunchKernelGGL(zstd_check_kernel, dim3((nframes + 3) / 4), dim3(256), 0, stream, d_desc, nframes,
                       d_out, s->ck, d_status);
    stage_mark(4, stream);
    return rc == 0 && hipGetLastError() == hipSuccess ? 0 : -1;
}

// Plan, wait for the item total and output extent, size the
// scratch, decode.  The one synchronization point of the zstd path: the item
// slots of a frame are only known once its sequence counts are read.
int zstd_decode_frames(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                       uint8_t *d_out, int32_t *d_status, ZstdScratch *s, hipStream_t stream)
{
    if (nframes == 0)
        return 0;
    if (zstd_scratch_reserve(s, nframes, 0, 0, stream) != 0)
        return -1;
    stage_mark(0, stream);
    if (launch_zstd_plan(d_desc, nframes, d_comp, s, stream) != 0)
        return -1;
    stage_mark(1, stream);
    if (hipStreamSynchronize(stream) != hipSuccess)
        return -1;
    if (zstd_scratch_reserve(s, nframes, s->total[1], s->total[0], stream) != 0)
        return -1;
    return launch_zstd_decode(d_desc, nframes, d_comp, d_out, d_status, s, stream);
}

}   // namespace zsk
