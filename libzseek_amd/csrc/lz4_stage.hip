// lz4_stage.hip — execute phase of the two-phase LZ4 decoder with each
// frame's output staged in LDS (gfx950).
//
// Input: the per-sequence items written by lz4_parse_kernel (lz4_split.hip).
// One wave executes one frame, a batch of up to 64 sequences at a time
// (one per lane).  The batch's output is assembled in a per-wave LDS ring
// and leaves it in aligned 16-byte chunks: consecutive lanes store
// consecutive chunks, so every HBM write is a full, coalesced line.
//
//   round 0   literal runs (from the compressed image) and matches whose
//             source is already final: in HBM if it was flushed, else in the
//             ring.  Runs are cut into 16-byte pieces dealt over the wave
//             (all loads in flight together), written into the ring exactly
//             (runs of >= 16 bytes as overlapping full pieces, shorter runs
//             byte by byte);
//   rounds    matches whose source lies in a still-pending match of the same
//             batch: multi-round resolution inside the ring (LDS latency,
//             not HBM);
//   flush     every complete aligned chunk of the batch -> HBM.
//
// A sequence producing more than kBatchOut bytes (stored blocks, very long
// runs) is copied straight in HBM by the whole wave after the ring is
// flushed.  The ring always holds frame bytes [flushed - 16, produced), so a
// 16-byte source piece either ends at or below `flushed` (read from HBM,
// whose stores were issued earlier by this wave: in order) or lies in it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4_dev.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4d;

constexpr uint32_t kItemExt = 0x80000000u;
constexpr uint32_t kItemPos = 0x3FFFFFFFu;
constexpr uint32_t kSW = 8;                  // waves (frames) per workgroup
constexpr uint32_t kStage = 16384;           // ring bytes per wave
constexpr uint32_t kStageRegion = kStage + 32;   // + 16-byte pads both sides
constexpr uint32_t kBatchOut = 12288;        // output bytes staged per batch at most

typedef u32x4 u32x4_lds __attribute__((aligned(1)));

// ---- LDS ring -------------------------------------------------------------------
// Frame output byte x lives at ring index (x + a0) & (kStage - 1); a0 aligns
// ring chunks with 16-byte output addresses.  The 16 bytes after the ring
// mirror its first 16 (and the pad before it its last), so a 16-byte access
// at any index is contiguous.
struct Ring {
    uint32_t base;   // LDS address of ring index 0
    uint32_t a0;     // output address & 15
};

__device__ __forceinline__ __attribute__((address_space(3))) uint8_t *lds_p(uint32_t a)
{
    return (__attribute__((address_space(3))) uint8_t *)(uintptr_t)a;
}

__device__ __forceinline__ u32x4 ring_read16(const Ring &R, uint32_t x)
{
    const uint32_t i = (x + R.a0) & (kStage - 1);
    return *reinterpret_cast<__attribute__((address_space(3))) u32x4_lds *>(lds_p(R.base + i));
}

__device__ __forceinline__ void ring_write16(const Ring &R, uint32_t x, u32x4 v)
{
    const uint32_t i = (x + R.a0) & (kStage - 1);
    *reinterpret_cast<__attribute__((address_space(3))) u32x4_lds *>(lds_p(R.base + i)) = v;
    if (i > kStage - 16)
        *reinterpret_cast<__attribute__((address_space(3))) u32x4_lds *>(lds_p(R.base + i - kStage)) = v;
    if (i < 16)
        *reinterpret_cast<__attribute__((address_space(3))) u32x4_lds *>(lds_p(R.base + i + kStage)) = v;
}

// N-byte LDS store at ring index of frame output x (N = 1, 2, 4, 8), mirrored
// into the pads at the ring's ends
template <int N, typename T>
__device__ __forceinline__ void ring_put(const Ring &R, uint32_t x, T v)
{
    typedef T T_u __attribute__((aligned(1)));
    const uint32_t i = (x + R.a0) & (kStage - 1);
    *reinterpret_cast<__attribute__((address_space(3))) T_u *>(lds_p(R.base + i)) = v;
    if (i > kStage - N)
        *reinterpret_cast<__attribute__((address_space(3))) T_u *>(lds_p(R.base + i - kStage)) = v;
    if (i < 16)
        *reinterpret_cast<__attribute__((address_space(3))) T_u *>(lds_p(R.base + i + kStage)) = v;
}

// first n (< 16) bytes of v at frame output x: 8/4/2/1-byte stores
__device__ __forceinline__ void ring_write_small(const Ring &R, uint32_t x, u32x4 v, uint32_t n)
{
    if (n & 8) {
        ring_put<8>(R, x, ((uint64_t)v.y << 32) | v.x);
        x += 8;
        v.x = v.z;
        v.y = v.w;
    }
    if (n & 4) {
        ring_put<4>(R, x, v.x);
        x += 4;
        v.x = v.y;
    }
    if (n & 2) {
        ring_put<2>(R, x, (uint16_t)v.x);
        x += 2;
        v.x >>= 16;
    }
    if (n & 1)
        ring_put<1>(R, x, (uint8_t)v.x);
}

// ---- HBM output --------------------------------------------------------------------
struct Out {
    uint8_t *o;        // frame output byte 0
    uint32_t dlen;
    Span sp;           // range-checked reads of the frame output
};

// store ring chunk c (output addresses [16c, 16c+16) relative to o - a0)
__device__ __forceinline__ void flush_chunk(const Ring &R, const Out &O, uint32_t c)
{
    const uint32_t i = (16 * c) & (kStage - 1);
    const u32x4 v = *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(lds_p(R.base + i));
    const int64_t x0 = (int64_t)16 * c - R.a0;   // frame offset of the chunk's first byte
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

// flush ring chunks [c0, c1) with the whole wave
__device__ __forceinline__ void flush_range(const Ring &R, const Out &O, uint32_t c0, uint32_t c1,
                                            uint32_t lane)
{
    for (uint32_t c = c0 + lane; c < c1; c += 64)
        flush_chunk(R, O, c);
}

// ---- pieces -------------------------------------------------------------------------
// A run of n bytes is cut into ceil(n/16) pieces: piece i covers
// [min(16 i, n - 16), +16) when n >= 16 (exact cover, overlaps rewrite equal
// bytes), else one short piece of n bytes.
__device__ __forceinline__ uint32_t npieces(uint32_t n)
{
    return (n + 15) >> 4;
}

__device__ __forceinline__ uint32_t piece_off(uint32_t n, uint32_t i)
{
    return n < 16 ? 0 : (16 * i < n - 16 ? 16 * i : n - 16);
}

__device__ __forceinline__ int run_of(uint32_t ex, uint32_t t)
{
    int k = 0;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1)
        if ((uint32_t)__shfl(ex, k + s, 64) <= t)
            k += s;
    return k;
}

__device__ __forceinline__ uint32_t excl_scan(uint32_t v, uint32_t lane, uint32_t *total)
{
    uint32_t inc = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        uint32_t u = __shfl_up(inc, d, 64);
        if (lane >= d)
            inc += u;
    }
    *total = (uint32_t)__shfl(inc, 63, 64);
    return inc - v;
}

// 16 source bytes of a match piece at frame output offset s: from HBM when
// the piece ends at or below `flushed`, else from the ring
__device__ __forceinline__ u32x4 match_src(const Ring &R, const Out &O, uint32_t flushed, uint32_t s)
{
    if (s + 16 <= flushed)
        return load16u(O.sp.r, O.sp.s0 + s);
    return ring_read16(R, s);
}

__device__ __forceinline__ void put_piece(const Ring &R, uint32_t d, u32x4 v, uint32_t n)
{
    if (n >= 16)
        ring_write16(R, d, v);
    else
        ring_write_small(R, d, v, n);
}

// Copy two runs per lane into the ring, pieces dealt over the wave: a literal
// run (ln bytes from compressed offset ls to output ld) and a match run (mn
// bytes from output ms to output md, non-overlapping, source final).
__device__ __forceinline__ void stage_runs(const Ring &R, const Out &O, const Span &isp,
                                           uint32_t flushed, uint32_t ls, uint32_t ld,
                                           uint32_t ln, uint32_t ms, uint32_t md, uint32_t mn,
                                           uint32_t lane)
{
    const uint32_t lp = npieces(ln), mp = npieces(mn);
    uint32_t lt, mt;
    const uint32_t lx = excl_scan(lp, lane, &lt);
    const uint32_t mx = excl_scan(mp, lane, &mt);
    const uint32_t tt = lt > mt ? lt : mt;
    for (uint32_t t = lane; t - lane < tt; t += 64) {
        const int kl = run_of(lx, t), km = run_of(mx, t);
        const bool pl = t < lt, pm = t < mt;
        const uint32_t nl = (uint32_t)__shfl(ln, kl, 64), nm = (uint32_t)__shfl(mn, km, 64);
        const uint32_t ol = piece_off(nl, t - (uint32_t)__shfl(lx, kl, 64));
        const uint32_t om = piece_off(nm, t - (uint32_t)__shfl(mx, km, 64));
        const uint32_t sl = (uint32_t)__shfl(ls, kl, 64) + ol, dl = (uint32_t)__shfl(ld, kl, 64) + ol;
        const uint32_t sm = (uint32_t)__shfl(ms, km, 64) + om, dm = (uint32_t)__shfl(md, km, 64) + om;
        u32x4 vl, vm;
        if (pl)
            vl = load16u(isp.r, isp.s0 + sl);
        if (pm)
            vm = match_src(R, O, flushed, sm);
        if (pl)
            put_piece(R, dl, vl, nl < 16 ? nl : 16);
        if (pm)
            put_piece(R, dm, vm, nm < 16 ? nm : 16);
    }
}

// Overlapping match (off < n) inside the ring, one lane: byte recurrence
// out[x] = out[x - off], 16 bytes at a time at distance eoff >= 16.
__device__ __forceinline__ void stage_overlap(const Ring &R, const Out &O, uint32_t flushed,
                                              uint32_t dst, uint32_t off, uint32_t n)
{
    uint32_t k = 0, eoff = off;
    if (off < 16) {
        const u32x4 pat = match_src(R, O, flushed, dst - off);
        uint32_t w[4] = {0, 0, 0, 0};
        uint32_t m = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) {
            w[i >> 2] |= vbyte(pat, m) << (8 * (i & 3));
            m = m + 1 == off ? 0 : m + 1;
        }
        const u32x4 v = (u32x4){w[0], w[1], w[2], w[3]};
        put_piece(R, dst, v, n < 16 ? n : 16);
        k = 16;
        eoff = off * ((16 + off - 1) / off);
    }
    for (; k < n; k += 16) {
        const u32x4 v = match_src(R, O, flushed, dst + k - eoff);
        const uint32_t r = n - k;
        put_piece(R, dst + k, v, r < 16 ? r : 16);
    }
}

__device__ __forceinline__ uint32_t uni_lane(uint32_t v, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// Whole-wave copy straight in HBM (no overlap between source and destination
// within a step of 1 KiB): used for sequences too long to stage.
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
        const uint32_t e = off * ((done + off) / off);   // a multiple of off <= done + off
        uint32_t step = e < 1024 ? e : 1024;
        if (step > n - done)
            step = n - done;
        if (e < 16) {
            // the first bytes of a short-period run: one lane, byte by byte
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

__global__ __launch_bounds__(64 * kSW) void lz4_stage_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ rec_base,
    const uint64_t *__restrict__ items, const uint32_t *__restrict__ nitems,
    const int32_t *__restrict__ status)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[kSW * kStageRegion];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t f = uni(blockIdx.x * kSW + w);
    if (f >= n)
        return;
    if (uni((uint32_t)status[f]) != (uint32_t)ST_OK)
        return;
    const FrameDesc d = desc[f];
    const uint32_t nit = uni(nitems[f]);
    const uint64_t *it = items + rec_base[f];
    Out O;
    O.o = out + d.d_off;
    O.dlen = d.d_size;
    O.sp = make_span(O.o, d.d_size);
    const Span isp = make_span(comp + d.c_off, d.c_size);
    Ring R;
    R.base = (uint32_t)(uintptr_t)(lds + w * kStageRegion + 16);
    R.a0 = (uint32_t)(reinterpret_cast<uintptr_t>(O.o) & 15);
    uint32_t produced = 0;   // frame output bytes decoded
    uint32_t fc = 0;         // ring chunks [0, fc) flushed
    uint64_t cur = lane < nit ? it[lane] : 0;
    uint32_t b = 0;
    while (b < nit) {
        const uint64_t nxt = b + 64 + lane < nit ? it[b + 64 + lane] : 0;
        const uint32_t w0 = (uint32_t)cur, w1 = (uint32_t)(cur >> 32);
        const uint32_t w0n = __shfl_down(w0, 1, 64), w1n = __shfl_down(w1, 1, 64);
        const uint32_t w0p = __shfl_up(w0, 1, 64);
        const bool act0 = b + lane < nit;
        const bool is_ext = lane > 0 && (w0p & kItemExt);
        const uint32_t src = w0 & kItemPos;
        const uint32_t off = w1 & 0xFFFF;
        uint32_t lit = 0, ml = 0;
        if (act0 && !is_ext) {
            if (w0 & kItemExt) {
                lit = w0n;
                ml = w1n;
            } else {
                lit = (w1 >> 16) & 0xFF;
                const uint32_t mc = w1 >> 24;
                ml = mc ? mc + 3 : 0;
            }
        }
        // batch = the lanes before the first one whose output would overflow
        // the ring budget; an extended item keeps its second half
        const uint32_t len = lit + ml;
        uint32_t tot;
        const uint32_t ex = excl_scan(len, lane, &tot);
        const uint64_t over = __ballot(act0 && ex + len > kBatchOut);
        uint32_t nb = over ? (uint32_t)__builtin_ctzll(over) : 64;
        if (nb == 64 && (uni_lane(w0, 63) & kItemExt))
            nb = 63;   // its second half is in the next batch: keep the pair together
        else if (nb > 0 && nb < 64 && (uni_lane(w0, (int)nb - 1) & kItemExt))
            nb++;
        if (b + nb > nit)
            nb = nit - b;
        const uint32_t flushed = 16 * fc > R.a0 ? 16 * fc - R.a0 : 0;   // frame bytes < this are in HBM
        if (nb == 0) {
            // lane 0 alone is too long to stage: flush the ring, copy in HBM
            const uint32_t l0 = uni_lane(lit, 0), m0 = uni_lane(ml, 0);
            const uint32_t s0 = uni_lane(src, 0), o0 = uni_lane(off, 0);
            const uint32_t end_c = (produced + R.a0 + 15) >> 4;
            flush_range(R, O, fc, end_c, lane);
            __builtin_amdgcn_s_waitcnt(0);
            if (l0)
                hbm_run(isp, s0, O.o + produced, l0, lane);
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
            // the ring restarts holding [flushed - 16, produced) from HBM
            fc = (produced + R.a0) >> 4;
            if (lane < 2) {
                const uint32_t c = fc - 1 + lane;   // chunks fc-1, fc
                const int64_t x0 = (int64_t)16 * c - R.a0;
                if ((fc > 0 || lane == 1) && x0 >= 0) {
                    const u32x4 v = load16u(O.sp.r, (uint32_t)((int64_t)O.sp.s0 + x0));
                    const uint32_t i = (16 * c) & (kStage - 1);
                    *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(lds_p(R.base + i)) = v;
                    if (i == 0)
                        *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(lds_p(R.base + kStage)) = v;
                    if (i == kStage - 16)
                        *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(lds_p(R.base - 16)) = v;
                }
            }
            const uint32_t used = uni_lane(w0, 0) & kItemExt ? 2 : 1;
            b += used;
            // next items: lanes shift down by `used`
            const uint64_t a = __shfl_down(cur, used, 64);
            const uint64_t c2 = __shfl(nxt, (int)((lane + used) & 63), 64);
            cur = lane + used < 64 ? a : c2;
            continue;
        }
        const bool act = lane < nb;
        if (!act) {
            lit = 0;
            ml = 0;
        }
        const uint32_t bstart = produced;
        const uint32_t op = produced + ex;
        const uint32_t mb = op + lit;
        const uint32_t me = mb + ml;
        const uint32_t msrc = mb - off;
        const bool overlap = ml != 0 && off < ml;
        const uint32_t need = overlap ? mb : msrc + ml;   // end of the bytes the copy reads
        const bool early = ml != 0 && !overlap && need <= bstart;
        produced += (uint32_t)__shfl(ex + len, (int)nb - 1, 64);
        // round 0: literal runs + matches with final sources
        stage_runs(R, O, isp, flushed, src, op, lit, msrc, mb, early ? ml : 0, lane);
        // rounds: the rest, inside the ring
        uint64_t pending = __ballot(ml != 0 && !early);
        while (pending) {
            const uint64_t below = pending & ((1ull << lane) - 1);
            const int hb = below ? 63 - __builtin_clzll(below) : (int)lane;
            const uint32_t me_hb = (uint32_t)__shfl(me, hb, 64);
            const uint32_t frontier = uni_lane(mb, __builtin_ctzll(pending));
            const bool mine = (pending >> lane) & 1;
            const bool ready = mine && (below == 0 || need <= frontier || msrc >= me_hb);
            if (ready && overlap)
                stage_overlap(R, O, flushed, mb, off, ml);
            stage_runs(R, O, isp, flushed, 0, 0, 0, msrc, mb, ready && !overlap ? ml : 0, lane);
            pending &= ~__ballot(ready);
        }
        // flush complete chunks (the frame's last chunk is flushed exactly)
        const bool last = b + nb >= nit;
        const uint32_t end_c = last ? (produced + R.a0 + 15) >> 4 : (produced + R.a0) >> 4;
        flush_range(R, O, fc, end_c, lane);
        fc = end_c;
        b += nb;
        // next items: lanes shift down by nb
        const uint64_t a = __shfl_down(cur, nb & 63, 64);
        const uint64_t c2 = __shfl(nxt, (int)((lane + nb) & 63), 64);
        cur = nb == 64 ? nxt : (lane + nb < 64 ? a : c2);
    }
}

// ---- pipelined variant: the next batch's loads fly while this one is staged

constexpr uint32_t kOff = 0xFFFFFFFFu;   // no piece
constexpr uint32_t kPF = 6;          // prefetched 16-byte pieces per lane per batch
constexpr uint32_t kBatch2 = 6144;   // output bytes per batch at most (2 batches + carry fit the ring)

struct PBatch {
    uint32_t b, nb, used;            // first item, items staged (0 = one long sequence), items consumed
    uint32_t bs, be;                 // frame output range
    uint32_t hv;                     // frame bytes below this were in HBM when prepared
    uint32_t lit, ml, off, src, op;  // this lane's sequence
    uint32_t early;                  // 1: match source final at prepare and in HBM (prefetched),
                                     // 2: final but (partly) in the ring
    uint32_t tp;                     // prefetched pieces (literal + HBM match) in the batch
    u32x4 pd[kPF];                   // prefetched piece data, pieces lane + 64 j
    uint32_t pdst[kPF], pn[kPF];     // piece output offset (kOff = none), bytes
};

// Decode the items at B.b (lane's item: itc), cut the batch, lay out its
// output from `produced`, and issue the loads of its literal pieces and of
// the pieces of matches whose source is already in HBM (below hv).
__device__ __forceinline__ void prepare(PBatch &B, uint64_t itc, uint32_t nit, uint32_t produced,
                                        uint32_t hv, const Span &isp, const Out &O, uint32_t lane)
{
    const uint32_t w0 = (uint32_t)itc, w1 = (uint32_t)(itc >> 32);
    const uint32_t w0n = __shfl_down(w0, 1, 64), w1n = __shfl_down(w1, 1, 64);
    const uint32_t w0p = __shfl_up(w0, 1, 64);
    const bool act0 = B.b + lane < nit;
    const bool is_ext = lane > 0 && (w0p & kItemExt);
    uint32_t lit = 0, ml = 0;
    if (act0 && !is_ext) {
        if (w0 & kItemExt) {
            lit = w0n;
            ml = w1n;
        } else {
            lit = (w1 >> 16) & 0xFF;
            const uint32_t mc = w1 >> 24;
            ml = mc ? mc + 3 : 0;
        }
    }
    const uint32_t len = lit + ml;
    uint32_t tot;
    const uint32_t ex = excl_scan(len, lane, &tot);
    const uint64_t over = __ballot(act0 && ex + len > kBatch2);
    uint32_t nb = over ? (uint32_t)__builtin_ctzll(over) : 64;
    if (nb == 64 && (uni_lane(w0, 63) & kItemExt))
        nb = 63;
    else if (nb > 0 && nb < 64 && (uni_lane(w0, (int)nb - 1) & kItemExt))
        nb++;
    if (B.b + nb > nit)
        nb = nit - B.b;
    B.nb = nb;
    B.bs = produced;
    B.hv = hv;
    B.src = w0 & kItemPos;
    B.off = w1 & 0xFFFF;
    B.tp = 0;
#pragma unroll
    for (int j = 0; j < (int)kPF; j++)
        B.pdst[j] = kOff;
    if (nb == 0) {
        // one sequence too long to stage: copied in HBM when processed
        B.used = (uni_lane(w0, 0) & kItemExt) ? 2 : 1;
        B.lit = lit;
        B.ml = ml;
        B.op = produced;
        B.early = 0;
        B.be = produced + uni_lane(len, 0);
        return;
    }
    B.used = nb;
    const bool act = lane < nb;
    if (!act) {
        lit = 0;
        ml = 0;
    }
    B.lit = lit;
    B.ml = ml;
    B.op = produced + ex;
    B.be = produced + (uint32_t)__shfl(ex + len, (int)nb - 1, 64);
    const uint32_t mb = B.op + lit;
    const uint32_t msrc = mb - B.off;
    const bool overlap = ml != 0 && B.off < ml;
    const bool early = ml != 0 && !overlap && msrc + ml <= produced;
    const bool in_hbm = early && msrc + ml <= hv;
    B.early = early ? (in_hbm ? 1 : 2) : 0;
    const uint32_t lp = npieces(lit), mp = in_hbm ? npieces(ml) : 0;
    uint32_t lt, mt;
    const uint32_t lx = excl_scan(lp, lane, &lt);
    const uint32_t mx = excl_scan(mp, lane, &mt);
    B.tp = lt + mt;
#pragma unroll
    for (int j = 0; j < (int)kPF; j++) {
        const uint32_t t = lane + 64 * j;
        if ((uint32_t)(64 * j) >= lt + mt)
            break;
        const int kl = run_of(lx, t);
        const uint32_t tm = t - lt;
        const int km = run_of(mx, tm);
        const uint32_t nl = (uint32_t)__shfl(lit, kl, 64), nm = (uint32_t)__shfl(ml, km, 64);
        const uint32_t ol = piece_off(nl, t - (uint32_t)__shfl(lx, kl, 64));
        const uint32_t om = piece_off(nm, tm - (uint32_t)__shfl(mx, km, 64));
        const uint32_t sl = (uint32_t)__shfl(B.src, kl, 64) + ol, dl = (uint32_t)__shfl(B.op, kl, 64) + ol;
        const uint32_t sm = (uint32_t)__shfl(msrc, km, 64) + om, dm = (uint32_t)__shfl(mb, km, 64) + om;
        if (t < lt) {
            B.pd[j] = load16u(isp.r, isp.s0 + sl);
            B.pdst[j] = dl;
            B.pn[j] = nl < 16 ? nl : 16;
        } else if (t < lt + mt) {
            B.pd[j] = load16u(O.sp.r, O.sp.s0 + sm);
            B.pdst[j] = dm;
            B.pn[j] = nm < 16 ? nm : 16;
        }
    }
}

__global__ __launch_bounds__(64 * kSW) void lz4_stage2_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ rec_base,
    const uint64_t *__restrict__ items, const uint32_t *__restrict__ nitems,
    const int32_t *__restrict__ status)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[kSW * kStageRegion];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t f = uni(blockIdx.x * kSW + w);
    if (f >= n)
        return;
    if (uni((uint32_t)status[f]) != (uint32_t)ST_OK)
        return;
    const FrameDesc d = desc[f];
    const uint32_t nit = uni(nitems[f]);
    const uint64_t *it = items + rec_base[f];
    Out O;
    O.o = out + d.d_off;
    O.dlen = d.d_size;
    O.sp = make_span(O.o, d.d_size);
    const Span isp = make_span(comp + d.c_off, d.c_size);
    Ring R;
    R.base = (uint32_t)(uintptr_t)(lds + w * kStageRegion + 16);
    R.a0 = (uint32_t)(reinterpret_cast<uintptr_t>(O.o) & 15);
    uint32_t fc = 0;   // ring chunks [0, fc) are in HBM
    PBatch A, B;
    A.b = 0;
    uint64_t itc = lane < nit ? it[lane] : 0;
    if (nit)
        prepare(A, itc, nit, 0, 0, isp, O, lane);
    uint32_t nextb = A.used;
    itc = nextb + lane < nit ? it[nextb + lane] : 0;
    bool have_next = false;
    while (A.b < nit) {
        const uint32_t hv = 16 * fc > R.a0 ? 16 * fc - R.a0 : 0;   // frame bytes < hv are in HBM
        // the next batch's loads fly while this one is staged (not after a
        // long sequence: the ring restarts there)
        have_next = false;
        if (A.nb != 0 && nextb < nit) {
            B.b = nextb;
            prepare(B, itc, nit, A.be, hv, isp, O, lane);
            nextb = B.b + B.used;
            itc = nextb + lane < nit ? it[nextb + lane] : 0;
            have_next = true;
        }
        if (A.nb == 0) {
            // one sequence too long to stage: flush the ring, copy in HBM
            const uint32_t l0 = uni_lane(A.lit, 0), m0 = uni_lane(A.ml, 0);
            const uint32_t s0 = uni_lane(A.src, 0), o0 = uni_lane(A.off, 0);
            const uint32_t produced = A.bs;
            flush_range(R, O, fc, (produced + R.a0 + 15) >> 4, lane);
            __builtin_amdgcn_s_waitcnt(0);
            if (l0)
                hbm_run(isp, s0, O.o + produced, l0, lane);
            __builtin_amdgcn_s_waitcnt(0);
            if (m0) {
                const uint32_t mb = produced + l0;
                if (o0 >= m0)
                    hbm_run(O.sp, mb - o0, O.o + mb, m0, lane);
                else
                    hbm_match(O, mb, o0, m0, lane);
            }
            __builtin_amdgcn_s_waitcnt(0);
            const uint32_t end = produced + l0 + m0;
            fc = (end + R.a0) >> 4;
            if (lane < 2) {
                const uint32_t c = fc - 1 + lane;   // ring chunks fc-1, fc from HBM
                const int64_t x0 = (int64_t)16 * c - R.a0;
                if ((fc > 0 || lane == 1) && x0 >= 0) {
                    const u32x4 v = load16u(O.sp.r, (uint32_t)((int64_t)O.sp.s0 + x0));
                    const uint32_t i = (16 * c) & (kStage - 1);
                    *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(lds_p(R.base + i)) = v;
                    if (i == 0)
                        *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(lds_p(R.base + kStage)) = v;
                    if (i == kStage - 16)
                        *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(lds_p(R.base - 16)) = v;
                }
            }
            __builtin_amdgcn_s_waitcnt(0);
            if (nextb < nit) {
                const uint32_t hv2 = 16 * fc > R.a0 ? 16 * fc - R.a0 : 0;
                B.b = nextb;
                prepare(B, itc, nit, end, hv2, isp, O, lane);
                nextb = B.b + B.used;
                itc = nextb + lane < nit ? it[nextb + lane] : 0;
                have_next = true;
            }
        } else {
            // prefetched pieces: literal runs, matches sourced in HBM
#pragma unroll
            for (int j = 0; j < (int)kPF; j++)
                if (A.pdst[j] != kOff)
                    put_piece(R, A.pdst[j], A.pd[j], A.pn[j]);
            const uint32_t mb = A.op + A.lit;
            const uint32_t me = mb + A.ml;
            const uint32_t msrc = mb - A.off;
            const bool overlap = A.ml != 0 && A.off < A.ml;
            const uint32_t need = overlap ? mb : msrc + A.ml;
            if (A.tp > 64 * kPF) {
                // pieces beyond the prefetch budget: copied now
                const bool in_hbm = A.early == 1;
                const uint32_t lp = npieces(A.lit), mp = in_hbm ? npieces(A.ml) : 0;
                uint32_t lt, mt;
                const uint32_t lx = excl_scan(lp, lane, &lt);
                const uint32_t mx = excl_scan(mp, lane, &mt);
                for (uint32_t t = 64 * kPF + lane; t - lane < lt + mt; t += 64) {
                    const int kl = run_of(lx, t);
                    const uint32_t tm = t - lt;
                    const int km = run_of(mx, tm);
                    const uint32_t nl = (uint32_t)__shfl(A.lit, kl, 64), nm = (uint32_t)__shfl(A.ml, km, 64);
                    const uint32_t ol = piece_off(nl, t - (uint32_t)__shfl(lx, kl, 64));
                    const uint32_t om = piece_off(nm, tm - (uint32_t)__shfl(mx, km, 64));
                    const uint32_t sl = (uint32_t)__shfl(A.src, kl, 64) + ol, dl = (uint32_t)__shfl(A.op, kl, 64) + ol;
                    const uint32_t sm = (uint32_t)__shfl(msrc, km, 64) + om, dm = (uint32_t)__shfl(mb, km, 64) + om;
                    if (t < lt) {
                        const u32x4 v = load16u(isp.r, isp.s0 + sl);
                        put_piece(R, dl, v, nl < 16 ? nl : 16);
                    } else if (t < lt + mt) {
                        const u32x4 v = load16u(O.sp.r, O.sp.s0 + sm);
                        put_piece(R, dm, v, nm < 16 ? nm : 16);
                    }
                }
            }
            const uint32_t flushed = 16 * fc > R.a0 ? 16 * fc - R.a0 : 0;
            // matches with final sources still (partly) in the ring
            stage_runs(R, O, isp, flushed, 0, 0, 0, msrc, mb, A.early == 2 ? A.ml : 0, lane);
            // the rest: multi-round resolution inside the ring
            uint64_t pending = __ballot(A.ml != 0 && A.early == 0);
            while (pending) {
                const uint64_t below = pending & ((1ull << lane) - 1);
                const int hb = below ? 63 - __builtin_clzll(below) : (int)lane;
                const uint32_t me_hb = (uint32_t)__shfl(me, hb, 64);
                const uint32_t frontier = uni_lane(mb, __builtin_ctzll(pending));
                const bool mine = (pending >> lane) & 1;
                const bool ready = mine && (below == 0 || need <= frontier || msrc >= me_hb);
                if (ready && overlap)
                    stage_overlap(R, O, flushed, mb, A.off, A.ml);
                stage_runs(R, O, isp, flushed, 0, 0, 0, msrc, mb, ready && !overlap ? A.ml : 0, lane);
                pending &= ~__ballot(ready);
            }
            const bool last = A.b + A.used >= nit;
            const uint32_t end_c = last ? (A.be + R.a0 + 15) >> 4 : (A.be + R.a0) >> 4;
            flush_range(R, O, fc, end_c, lane);
            fc = end_c;
        }
        if (!have_next)
            break;
        A = B;
    }
}

}   // namespace

int launch_lz4_exec_stage(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                          uint8_t *d_out, const uint64_t *rec_base, const uint64_t *items,
                          const uint32_t *nitems, const int32_t *d_status, hipStream_t stream,
                          int version)
{
    if (nframes == 0)
        return 0;
    if (version == 2)
        hipLaunchKernelGGL(lz4_stage2_kernel, dim3((nframes + kSW - 1) / kSW), dim3(64 * kSW), 0,
                           stream, d_desc, nframes, d_comp, d_out, rec_base, items, nitems, d_status);
    else
        hipLaunchKernelGGL(lz4_stage_kernel, dim3((nframes + kSW - 1) / kSW), dim3(64 * kSW), 0,
                           stream, d_desc, nframes, d_comp, d_out, rec_base, items, nitems, d_status);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk
