// lz4_split.hip — two-phase LZ4-frame decoder for CDNA4 (gfx950).
//
// Replaces the per-frame liblz4 call of the reference hot path
// (/root/reference/src/decompress.c:752-773, LZ4F_decompress in a loop) with
// three launches over every frame a zseek_pread range covers:
//
//   plan   one workgroup: per-frame item slots (exclusive scan of
//          align4(cSize/3 + 2)) — an LZ4 sequence takes >= 3 compressed bytes,
//          so a frame never needs more slots than that;
//   parse  ONE LANE PER FRAME: the serial part of LZ4 (token -> lengths ->
//          next token) runs 64 frames per wave instruction.  Each lane walks
//          its frame's header and blocks with the full liblz4 1.9.3
//          validation (same rules and status codes as lz4_wave.hip / the
//          oracle) and emits one 4-byte item per sequence: the token's frame
//          offset (bit 30: literals-only last sequence of a block) or, for a
//          stored block, its data offset (bit 31);
//   exec   ONE WAVE PER FRAME: items in batches of 64 (one per lane).  Each
//          lane re-reads its own token (lengths, offset), a wave prefix-sum
//          gives every sequence its output position, literal runs are copied
//          straight from the compressed image to the output in HBM, then
//          back-references are resolved in rounds: a lane copies its match
//          once no lower lane still owes bytes its source range needs
//          (multi-round resolution), so independent matches of a batch copy
//          in parallel;
//   defer  frames with block / content checksums (rare; not written by the
//          reference's writer) or that do not fit the parse scratch are
//          handed to the wave-per-frame kernel (lz4_wave.hip), which checks
//          XXH32 as it decodes.
//
// Output bytes are written once, with 16/8/4/2/1-byte stores that never cross
// the end of a sequence, so neighbouring frames' outputs are never touched.
// All compressed-image reads go through buffer resources with range checks.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <array>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "lz4_dev.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4d;

constexpr uint32_t kItemExt = 0x80000000u;   // item w0: next item holds the full lengths
constexpr uint32_t kItemPos = 0x3FFFFFFFu;
constexpr uint32_t kExecWaves = 4;
constexpr uint32_t kLongCopy = 256;   // longer literal runs / matches: copied by the whole wave

// Per-lane reader over one frame of the compressed image with a 16-byte
// register window on dword-aligned coordinates.
struct LaneIn {
    __amdgpu_buffer_rsrc_t r;
    uint32_t s0;     // frame offset p = coordinate p + s0
    uint32_t wp;     // window covers frame offsets [wp, wp+16) (wp may wrap below 0)
    u32x4 w;

    __device__ __forceinline__ u32x4 load16(uint32_t p) const { return load16u(r, p + s0); }
    __device__ __forceinline__ void at(uint32_t p)
    {
        const uint32_t x = (p + s0) & ~3u;
        w = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, x, 0, 0));
        wp = x - s0;
    }
    __device__ __forceinline__ uint32_t byte(uint32_t p)
    {
        if (p - wp >= 16)
            at(p);
        return vbyte(w, p - wp);
    }
    __device__ __forceinline__ uint32_t word(uint32_t p)
    {
        if (p - wp > 12)
            at(p);
        return vword(w, p - wp);
    }
};

// XXH32 (seed 0) of n < 16 bytes at frame offset p: the LZ4 frame header
// checksum.
__device__ uint32_t xxh32_short(LaneIn &in, uint32_t p, uint32_t n)
{
    uint32_t acc = 0x165667B1u + n;
    uint32_t i = 0;
    for (; i + 4 <= n; i += 4) {
        acc += in.word(p + i) * 0xC2B2AE3Du;
        acc = ((acc << 17) | (acc >> 15)) * 0x27D4EB2Fu;
    }
    for (; i < n; i++) {
        acc += in.byte(p + i) * 0x165667B1u;
        acc = ((acc << 11) | (acc >> 21)) * 0x9E3779B1u;
    }
    acc ^= acc >> 15;
    acc *= 0x85EBCA77u;
    acc ^= acc >> 13;
    acc *= 0xC2B2AE3Du;
    acc ^= acc >> 16;
    return acc;
}

// Items of one frame, two per 16-byte store.  Item = (w0, w1):
//   w0 = frame offset of the sequence's first literal byte (bits 0-29),
//        bit 31 = extended: the NEXT item is (literal length, match length);
//   w1 = match offset (bits 0-15) | literal length (16-23) |
//        match code (24-31: 0 = no match, else match length - 3).
// Extended items (literal > 255 or match > 258: long runs, stored blocks)
// never start at slot 63 of a 64-item batch (a zero padding item goes
// first), so the exec kernel finds both halves in one wave.
struct Sink {
    uint64_t *base;
    uint32_t k, cap;
    u32x4 acc;

    __device__ __forceinline__ bool put1(uint32_t w0, uint32_t w1)
    {
        if (k >= cap)
            return false;
        if (k & 1) {
            acc.z = w0;
            acc.w = w1;
            *reinterpret_cast<u32x4 *>(base + k - 1) = acc;
        } else {
            acc.x = w0;
            acc.y = w1;
        }
        k++;
        return true;
    }
    __device__ __forceinline__ bool seq(uint32_t lsrc, uint32_t lit, uint32_t off, uint32_t ml)
    {
        if (lit > 255 || ml > 258) {
            if ((k & 63) == 63 && !put1(0, 0))
                return false;
            return put1(lsrc | kItemExt, off) && put1(lit, ml);
        }
        return put1(lsrc, off | (lit << 16) | ((ml ? ml - 3 : 0) << 24));
    }
    __device__ __forceinline__ void finish()
    {
        if (k & 1)
            *reinterpret_cast<u32x4 *>(base + k - 1) = acc;
    }
};

// One compressed LZ4 block [ip, ip+bsize) producing output from op (liblz4
// 1.9.3 LZ4_decompress_safe rules; mirrors WaveDec::block in lz4_wave.hip
// and decode_block in oracle/lz4_oracle.c).
__device__ int32_t parse_block(LaneIn &in, Sink &sink, uint32_t ip, uint32_t bsize, uint32_t op,
                               uint32_t cap, uint32_t floor_, uint32_t dlen, uint32_t *op_out)
{
    const uint32_t iend = ip + bsize;
    const uint32_t oend = op + cap;
    if (bsize == 0)
        return ST_BLOCK_ERR;
    for (;;) {
        if (ip >= iend)
            return ST_BLOCK_ERR;
        if (ip - in.wp > 12)
            in.at(ip);
        uint32_t tok = in.byte(ip);
        uint32_t lit = tok >> 4;
        uint32_t p = ip + 1;
        if (lit == 15) {
            if (iend - p <= 15)
                return ST_BLOCK_ERR;
            uint32_t s;
            do {
                if (p >= iend)
                    return ST_BLOCK_ERR;
                s = in.byte(p++);
                lit += s;
            } while (s == 255);
        }
        if (op + lit > oend - kMfLimit || iend - p < lit + 2 + 1 + kLastLiterals) {
            if (iend - p != lit || op + lit > oend)
                return ST_BLOCK_ERR;
            if (op + lit > dlen)
                return ST_DST_OVERFLOW;
            if (!sink.seq(p, lit, 0, 0))
                return ST_NOT_RUN;
            *op_out = op + lit;
            return ST_OK;
        }
        if (op + lit > dlen)
            return ST_DST_OVERFLOW;
        const uint32_t lsrc = p;
        const uint32_t nlit = lit;
        p += lit;
        op += lit;
        uint32_t off = in.word(p) & 0xFFFF;
        p += 2;
        uint32_t ml = tok & 15;
        if (ml == 15) {
            uint32_t s;
            do {
                if (p >= iend)
                    return ST_BLOCK_ERR;
                s = in.byte(p++);
                ml += s;
                if (p >= iend - (kLastLiterals - 1))
                    return ST_BLOCK_ERR;
            } while (s == 255);
        }
        ml += kMinMatch;
        if (off == 0)
            return ST_NOT_RUN;   // zeros (liblz4): the wave kernel decodes the frame
        if (off > op - floor_)
            return ST_BLOCK_ERR;
        if (op + ml > oend - kLastLiterals)
            return ST_BLOCK_ERR;
        if (op + ml > dlen)
            return ST_DST_OVERFLOW;
        if (!sink.seq(lsrc, nlit, off, ml))
            return ST_NOT_RUN;
        op += ml;
        ip = p;
    }
}

// Whole-frame parse (mirrors WaveDec::frame in lz4_wave.hip).  ST_NOT_RUN
// means "hand to the wave kernel".
__device__ int32_t parse_frame(LaneIn &in, Sink &sink, uint32_t clen, uint32_t dlen,
                               uint32_t *fail_op)
{
    if (clen < 7)
        return ST_HDR_INCOMPLETE;
    in.at(0);
    uint32_t magic = in.word(0);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u)
        return ST_SHORT_FRAME;
    if (magic != kLz4Magic)
        return ST_FRAME_TYPE;
    uint32_t desc = in.word(4);
    uint32_t flg = desc & 0xFF, bd = (desc >> 8) & 0xFF;
    if (flg & 0x14)   // block or content checksums: the wave kernel verifies them
        return ST_NOT_RUN;
    uint32_t indep = (flg >> 5) & 1;
    uint32_t csize_flag = (flg >> 3) & 1;
    uint32_t dictid = flg & 1;
    if ((flg >> 1) & 1)
        return ST_RESERVED;
    if (((flg >> 6) & 3) != 1)
        return ST_VERSION;
    uint32_t hdr = 7 + (csize_flag ? 8 : 0) + (dictid ? 4 : 0);
    if (clen < hdr)
        return ST_HDR_INCOMPLETE;
    uint32_t bsid = (bd >> 4) & 7;
    if ((bd >> 7) & 1)
        return ST_RESERVED;
    if (bsid < 4)
        return ST_MAXBLOCK;
    if (bd & 15)
        return ST_RESERVED;
    if (((xxh32_short(in, 4, hdr - 5) >> 8) & 0xFF) != in.byte(hdr - 1))
        return ST_HDR_CHECKSUM;
    uint64_t content_size = 0;
    if (csize_flag)
        content_size = (uint64_t)in.word(6) | ((uint64_t)in.word(10) << 32);
    const uint32_t max_block = 1u << (8 + 2 * bsid);
    uint32_t ip = hdr;
    uint32_t op = 0;
    for (;;) {
        *fail_op = op;
        if (clen - ip < 4)
            return ST_TRUNCATED;
        uint32_t bh = in.word(ip);
        ip += 4;
        if (bh == 0)
            break;
        uint32_t bsize = bh & 0x7FFFFFFFu;
        if (bsize > max_block)
            return ST_MAXBLOCK;
        if (clen - ip < bsize)
            return ST_TRUNCATED;
        if (bh & 0x80000000u) {
            if (op + bsize > dlen)
                return ST_DST_OVERFLOW;
            if (!sink.seq(ip, bsize, 0, 0))
                return ST_NOT_RUN;
            op += bsize;
        } else {
            uint32_t floor_ = indep ? op : 0;   // offsets <= 65535 anyway
            uint32_t nop = op;
            int32_t st = parse_block(in, sink, ip, bsize, op, max_block, floor_, dlen, &nop);
            if (st != ST_OK) {
                if (st == ST_BLOCK_ERR) {
                    bool direct = (dlen - op) >= max_block;
                    int32_t bits = (int32_t)((bsid - 4) << ST_BSID_SHIFT);
                    return (direct ? (ST_GENERIC | ST_DIRECT_FLAG) : ST_DECOMPRESS_FAILED) |
                           ST_BLOCK_FAIL_FLAG | bits;
                }
                return st;
            }
            op = nop;
        }
        ip += bsize;
    }
    *fail_op = op;
    if (csize_flag && content_size != op)
        return ST_FRAME_SIZE;
    if (op != dlen)
        return ST_SHORT_FRAME;
    return ST_OK;
}

// ---- plan: per-frame item slot offsets ------------------------------------
// Slot offsets without a scan (the usual case): when the frames lie in order
// in the input (c_off[f+1] >= c_off[f] + c_size[f], as in every batch the
// reader builds), frame f's slots start at ceil4((c_off[f] - c_off[0]) / 8 +
// 40 f), and the gap to frame f+1 is >= c_size/8 + 37 > slots_of(c_size).  A
// frame out of order sets *redo, and lz4_plan_kernel scans instead.
__global__ __launch_bounds__(256) void lz4_plan_direct_kernel(const FrameDesc *__restrict__ desc,
                                                               uint32_t n, uint64_t *__restrict__ rec_base,
                                                               uint64_t *__restrict__ total,
                                                               uint32_t *__restrict__ redo)
{
    const uint32_t f = blockIdx.x * 256 + threadIdx.x;
    if (f >= n)
        return;
    const FrameDesc d = desc[f];
    const uint64_t c0 = desc[0].c_off;
    const uint64_t r = (((d.c_off - c0) >> 3) + 40ull * f + 3) & ~3ull;
    rec_base[f] = r;
    if (d.c_off < c0 || (f + 1 < n && desc[f + 1].c_off < d.c_off + d.c_size))
        *redo = 1;
    if (f + 1 == n)
        *total = r + slots_of(d.c_size);
}

// Slot offsets by an exclusive scan of slots_of(c_size), one workgroup; runs
// only when lz4_plan_direct_kernel flagged the batch (*redo != 0).
__global__ __launch_bounds__(1024) void lz4_plan_kernel(const FrameDesc *__restrict__ desc,
                                                        uint32_t n, uint64_t *__restrict__ rec_base,
                                                        uint64_t *__restrict__ total,
                                                        const uint32_t *__restrict__ redo)
{
    __shared__ uint64_t part[1024];
    if (*redo == 0)
        return;
    const uint32_t t = threadIdx.x;
    const uint32_t chunk = (n + 1023) / 1024;
    const uint32_t i0 = t * chunk < n ? t * chunk : n;
    const uint32_t i1 = i0 + chunk < n ? i0 + chunk : n;
    uint64_t s = 0;
    for (uint32_t i = i0; i < i1; i++)
        s += slots_of(desc[i].c_size);
    part[t] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - s;
    for (uint32_t i = i0; i < i1; i++) {
        rec_base[i] = run;
        run += slots_of(desc[i].c_size);
    }
    if (t == 1023)
        *total = part[t];
}

// ---- parse: one lane per frame --------------------------------------------
__global__ __launch_bounds__(256) void lz4_parse_kernel(const FrameDesc *__restrict__ desc,
                                                        uint32_t n, const uint8_t *__restrict__ comp,
                                                        const uint64_t *__restrict__ rec_base,
                                                        uint64_t capacity, uint64_t *__restrict__ items,
                                                        uint32_t *__restrict__ nitems,
                                                        int32_t *__restrict__ status,
                                                        uint32_t *__restrict__ fail_at)
{
    const uint32_t f = blockIdx.x * 256 + threadIdx.x;
    const bool act = f < n;
    FrameDesc d = {0, 0, 0, 0};
    if (act)
        d = desc[f];
    // one buffer resource per wave spanning its frames' compressed bytes
    const uint64_t lo = wave_min64(act ? d.c_off : ~0ull);
    const uint64_t hi = wave_max64(act ? d.c_off + d.c_size : 0ull);
    if (!act)
        return;
    uint32_t fail_op = 0;
    int32_t st;
    Sink sink;
    sink.k = 0;
    sink.acc = (u32x4){0, 0, 0, 0};
    const uint64_t rb = rec_base[f];
    const uint32_t cap = slots_of(d.c_size);
    sink.base = items + rb;
    sink.cap = cap;
    if (hi - lo >= 0xFFFFFF00ull || d.c_size > kItemPos || rb + cap > capacity) {
        st = ST_NOT_RUN;
    } else {
        const Span sp = make_span(comp + lo, hi - lo);
        LaneIn in;
        in.r = sp.r;
        in.s0 = sp.s0 + (uint32_t)(d.c_off - lo);
        in.wp = 0x80000000u;
        st = parse_frame(in, sink, d.c_size, d.d_size, &fail_op);
        sink.finish();
    }
    status[f] = st;
    nitems[f] = sink.k;
    if (fail_at)
        fail_at[f] = fail_op;
}

// ---- exec: one wave per frame ----------------------------------------------

// 16 bytes of the frame's output at offset p (bytes past the frame read as 0)
__device__ __forceinline__ u32x4 load16_out(const Span &o, uint32_t p)
{
    return load16u(o.r, p + o.s0);
}

// Copy an n-byte match at distance off to out[dst..]: 16-byte pieces; a
// distance under 16 first writes one period-off pattern piece, then continues
// at the distance rounded up to a multiple of off that is >= 16.  A lane's
// own earlier stores are visible to its later loads (in-order per wave).
__device__ __forceinline__ void copy_match(uint8_t *out, const Span &orr, uint32_t dst,
                                           uint32_t off, uint32_t n)
{
    uint32_t k = 0;
    uint32_t eoff = off;
    if (off < 16) {
        u32x4 pat = load16_out(orr, dst - off);
        u32x4 v = (u32x4){0, 0, 0, 0};
        uint32_t m = 0;
        for (uint32_t i = 0; i < 16; i++) {
            uint32_t b = vbyte(pat, m);
            uint32_t sh = (i & 3) * 8;
            if ((i >> 2) == 0) v.x |= b << sh;
            else if ((i >> 2) == 1) v.y |= b << sh;
            else if ((i >> 2) == 2) v.z |= b << sh;
            else v.w |= b << sh;
            m = m + 1 == off ? 0 : m + 1;
        }
        store_exact(out + dst, v, n < 16 ? n : 16);
        k = 16;
        eoff = off * ((16 + off - 1) / off);
    }
    for (; k < n; k += 16) {
        u32x4 v = load16_out(orr, dst + k - eoff);
        uint32_t r = n - k;
        store_exact(out + dst + k, v, r < 16 ? r : 16);
    }
}

__device__ __forceinline__ uint32_t uni_lane(uint32_t v, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// A long match copied by the whole wave: 16 bytes per lane per step.  Having
// produced `done` bytes, the source may be any multiple E of off with
// E <= done + off (those bytes are already final); a step writes at most E
// bytes so no lane reads what another lane of the same step writes.
__device__ __forceinline__ void copy_match_wave(uint8_t *out, const Span &orr, uint32_t dst,
                                             uint32_t off, uint32_t n, uint32_t lane)
{
    uint32_t done = 0;
    if (off < 16) {
        if (lane == 0)
            copy_match(out, orr, dst, off, 16);
        done = 16;
    }
    while (done < n) {
        __builtin_amdgcn_s_waitcnt(0);
        const uint32_t e = off * ((done + off) / off);
        uint32_t step = e < 1024 ? (e & ~15u) : 1024;
        if (step > n - done)
            step = n - done;
        const uint32_t k = done + 16 * lane;
        if (16 * lane < step) {
            u32x4 v = load16_out(orr, dst + k - e);
            uint32_t r = n - k;
            store_exact(out + dst + k, v, r < 16 ? r : 16);
        }
        done += step;
    }
}

// Largest lane k with ex[k] <= t (ex non-decreasing over lanes, ex[0] = 0).
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

// Byte-parallel copy of two sets of runs, one of each per lane: a literal run
// (ln bytes from compressed offset ls to output offset ld) and a match run
// (mn bytes from output offset ms to output offset md; source and destination
// must not overlap).  Every lane copies the first 16-byte piece of its own
// runs; the remaining pieces of all runs are dealt round-robin over the wave
// (run found by binary search over the piece prefix sums), so a batch with one
// long run costs as many wave steps as its pieces / 64, not its length / 16.
__device__ __forceinline__ void copy_runs(const Span &isp, const Span &osp, uint8_t *o,
                                          uint32_t ls, uint32_t ld, uint32_t ln,
                                          uint32_t ms, uint32_t md, uint32_t mn, uint32_t lane)
{
    u32x4 a, b;
    if (ln)
        a = load16u(isp.r, isp.s0 + ls);
    if (mn)
        b = load16_out(osp, ms);
    const uint32_t lr = ln > 16 ? (ln - 1) >> 4 : 0;   // pieces after the first
    const uint32_t mr = mn > 16 ? (mn - 1) >> 4 : 0;
    uint32_t lt, mt;
    const uint32_t lx = excl_scan(lr, lane, &lt);
    const uint32_t mx = excl_scan(mr, lane, &mt);
    if (ln)
        store_exact(o + ld, a, ln < 16 ? ln : 16);
    if (mn)
        store_exact(o + md, b, mn < 16 ? mn : 16);
    const uint32_t tt = lt > mt ? lt : mt;
    for (uint32_t t = lane; t - lane < tt; t += 128) {
        const uint32_t t1 = t + 64;
        // literal pieces t, t1 and match pieces t, t1
        const int kl0 = run_of(lx, t), kl1 = run_of(lx, t1);
        const int km0 = run_of(mx, t), km1 = run_of(mx, t1);
        const uint32_t il0 = 16 * (t - (uint32_t)__shfl(lx, kl0, 64) + 1);
        const uint32_t il1 = 16 * (t1 - (uint32_t)__shfl(lx, kl1, 64) + 1);
        const uint32_t im0 = 16 * (t - (uint32_t)__shfl(mx, km0, 64) + 1);
        const uint32_t im1 = 16 * (t1 - (uint32_t)__shfl(mx, km1, 64) + 1);
        const uint32_t sl0 = (uint32_t)__shfl(ls, kl0, 64) + il0, dl0 = (uint32_t)__shfl(ld, kl0, 64) + il0;
        const uint32_t sl1 = (uint32_t)__shfl(ls, kl1, 64) + il1, dl1 = (uint32_t)__shfl(ld, kl1, 64) + il1;
        const uint32_t sm0 = (uint32_t)__shfl(ms, km0, 64) + im0, dm0 = (uint32_t)__shfl(md, km0, 64) + im0;
        const uint32_t sm1 = (uint32_t)__shfl(ms, km1, 64) + im1, dm1 = (uint32_t)__shfl(md, km1, 64) + im1;
        const uint32_t nl0 = (uint32_t)__shfl(ln, kl0, 64) - il0, nl1 = (uint32_t)__shfl(ln, kl1, 64) - il1;
        const uint32_t nm0 = (uint32_t)__shfl(mn, km0, 64) - im0, nm1 = (uint32_t)__shfl(mn, km1, 64) - im1;
        const bool pl0 = t < lt, pl1 = t1 < lt, pm0 = t < mt, pm1 = t1 < mt;
        u32x4 v0, v1, v2, v3;
        if (pl0)
            v0 = load16u(isp.r, isp.s0 + sl0);
        if (pl1)
            v1 = load16u(isp.r, isp.s0 + sl1);
        if (pm0)
            v2 = load16_out(osp, sm0);
        if (pm1)
            v3 = load16_out(osp, sm1);
        if (pl0)
            store_exact(o + dl0, v0, nl0 < 16 ? nl0 : 16);
        if (pl1)
            store_exact(o + dl1, v1, nl1 < 16 ? nl1 : 16);
        if (pm0)
            store_exact(o + dm0, v2, nm0 < 16 ? nm0 : 16);
        if (pm1)
            store_exact(o + dm1, v3, nm1 < 16 ? nm1 : 16);
    }
}

// Diagnostic counters of the exec kernel (tuning builds only, DIAG & 8):
// [0] batches, [1] resolution rounds, [2] long literal runs, [3] long matches,
// [4] sequences, [5] matches copied in round 0
__device__ unsigned long long g_exec_stats[8];

// DIAG (tuning builds): 1 = no wait between resolution rounds, 2 = skip
// back-references, 8 = count (g_exec_stats), 16 = round 0 only.  OCC: minimum
// waves per SIMD the register allocation must allow.
template <int DIAG, int OCC = 1>
__global__ __launch_bounds__(64 * kExecWaves) __attribute__((amdgpu_waves_per_eu(OCC))) void lz4_exec_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ rec_base,
    const uint64_t *__restrict__ items, const uint32_t *__restrict__ nitems,
    const int32_t *__restrict__ status)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t f = uni(blockIdx.x * kExecWaves + (threadIdx.x >> 6));
    if (f >= n)
        return;
    if (uni((uint32_t)status[f]) != (uint32_t)ST_OK)
        return;
    const FrameDesc d = desc[f];
    const uint32_t nit = uni(nitems[f]);
    const uint64_t *it = items + rec_base[f];
    uint8_t *o = out + d.d_off;
    const Span osp = make_span(o, d.d_size);
    const Span isp = make_span(comp + d.c_off, d.c_size);
    uint32_t obase = 0;
    uint64_t cur = lane < nit ? it[lane] : 0;
    for (uint32_t b = 0; b < nit; b += 64) {
        const uint64_t nxt = b + 64 + lane < nit ? it[b + 64 + lane] : 0;   // next batch, early
        const uint32_t w0 = (uint32_t)cur, w1 = (uint32_t)(cur >> 32);
        const uint32_t w0n = __shfl_down(w0, 1, 64), w1n = __shfl_down(w1, 1, 64);
        const uint32_t w0p = __shfl_up(w0, 1, 64);
        const bool is_ext = lane > 0 && (w0p & kItemExt);
        const uint32_t src = w0 & kItemPos;
        const uint32_t off = w1 & 0xFFFF;
        uint32_t lit, ml;
        if (is_ext) {
            lit = 0;
            ml = 0;
        } else if (w0 & kItemExt) {
            lit = w0n;
            ml = w1n;
        } else {
            lit = (w1 >> 16) & 0xFF;
            const uint32_t mc = w1 >> 24;
            ml = mc ? mc + 3 : 0;
        }
        // output positions: exclusive wave prefix sum of lit + ml
        const uint32_t len = lit + ml;
        uint32_t inc = len;
        for (uint32_t dlt = 1; dlt < 64; dlt <<= 1) {
            uint32_t v = __shfl_up(inc, dlt, 64);
            if (lane >= dlt)
                inc += v;
        }
        const uint32_t bstart = obase;
        const uint32_t op = obase + inc - len;
        obase += (uint32_t)__shfl(inc, 63, 64);
        const uint32_t mb = op + lit;
        const uint32_t me = mb + ml;
        const uint32_t msrc = mb - off;
        const uint32_t need = off >= ml ? msrc + ml : mb;   // end of the bytes the copy reads
        if (DIAG & 2)
            ml = 0;
        // round 0: literal runs and matches whose source lies before this
        // batch (already final), loads of both in flight together
        const bool early = ml != 0 && off >= ml && need <= bstart;
        copy_runs(isp, osp, o, src, op, lit, msrc, mb, early ? ml : 0, lane);
        if (DIAG & 8) {
            const uint64_t bl = __ballot(lit > kLongCopy), bm = __ballot(ml > kLongCopy), be = __ballot(early);
            if (lane == 0) {
                atomicAdd(&g_exec_stats[0], 1ull);
                atomicAdd(&g_exec_stats[4], (unsigned long long)(nit - b < 64 ? nit - b : 64));
                atomicAdd(&g_exec_stats[2], (unsigned long long)__popcll(bl));
                atomicAdd(&g_exec_stats[3], (unsigned long long)__popcll(bm));
                atomicAdd(&g_exec_stats[5], (unsigned long long)__popcll(be));
            }
        }
        // the rest: multi-round resolution.  Lane k may copy once its source
        // range [msrc, need) misses every pending match below it: it ends
        // before the lowest pending match starts, or starts after the nearest
        // pending one below ends (pending ranges are ordered by lane).
        uint64_t pending = (DIAG & 16) ? 0 : __ballot(ml != 0 && !early);
        while (pending) {
            if (!(DIAG & 1))
                __builtin_amdgcn_s_waitcnt(0);   // earlier rounds' stores complete
            const uint64_t below = pending & ((1ull << lane) - 1);
            const int hb = below ? 63 - __builtin_clzll(below) : (int)lane;
            const uint32_t me_hb = (uint32_t)__shfl(me, hb, 64);
            const uint32_t frontier = uni_lane(mb, __builtin_ctzll(pending));
            const bool mine = (pending >> lane) & 1;
            const bool ready = mine && (below == 0 || need <= frontier || msrc >= me_hb);
            const bool over = off < ml;   // overlapping copy: serial pieces
            if (ready && over && ml <= kLongCopy)
                copy_match(o, osp, mb, off, ml);
            copy_runs(isp, osp, o, 0, 0, 0, msrc, mb, ready && !over ? ml : 0, lane);
            const uint64_t rmask = __ballot(ready);
            for (uint64_t lm = __ballot(ready && over && ml > kLongCopy); lm; lm &= lm - 1) {
                const int l = __builtin_ctzll(lm);
                copy_match_wave(o, osp, uni_lane(mb, l), uni_lane(off, l), uni_lane(ml, l), lane);
            }
            pending &= ~rmask;
            if ((DIAG & 8) && lane == 0)
                atomicAdd(&g_exec_stats[1], 1ull);
        }
        cur = nxt;
    }
}

}   // namespace

// ---- host side ---------------------------------------------------------------

uint64_t split_items_needed(const FrameDesc *h_desc, uint32_t n)
{
    uint64_t s = 0;
    for (uint32_t i = 0; i < n; i++)
        s += slots_of(h_desc[i].c_size);
    // where lz4_plan_direct_kernel's layout ends (frames in order)
    if (n && h_desc[n - 1].c_off >= h_desc[0].c_off) {
        const uint64_t last = (((h_desc[n - 1].c_off - h_desc[0].c_off) >> 3) + 40ull * (n - 1) + 3) & ~3ull;
        const uint64_t d = last + slots_of(h_desc[n - 1].c_size);
        if (d > s)
            s = d;
    }
    return s;
}

void split_scratch_free(SplitScratch *s)
{
    if (s->rec_base)
        (void)hipFree(s->rec_base);
    if (s->nitems)
        (void)hipFree(s->nitems);
    if (s->items)
        (void)hipFree(s->items);
    if (s->total)
        (void)hipHostFree(s->total);
    if (s->redo)
        (void)hipFree(s->redo);
    *s = SplitScratch();
}

int split_scratch_reserve(SplitScratch *s, uint32_t frames, uint64_t items, hipStream_t stream)
{
    if (!s->total) {
        if (hipHostMalloc((void **)&s->total, sizeof(uint64_t), hipHostMallocMapped) != hipSuccess)
            return -1;
        *s->total = 0;
    }
    if (!s->redo && hipMalloc((void **)&s->redo, sizeof(uint32_t)) != hipSuccess)
        return -1;
    if (frames > s->frames_cap) {
        uint32_t cap = frames < 4096 ? 4096 : frames;
        (void)hipStreamSynchronize(stream);
        if (s->rec_base)
            (void)hipFree(s->rec_base);
        if (s->nitems)
            (void)hipFree(s->nitems);
        s->rec_base = nullptr;
        s->nitems = nullptr;
        s->frames_cap = 0;
        if (hipMalloc((void **)&s->rec_base, (size_t)cap * 8) != hipSuccess ||
            hipMalloc((void **)&s->nitems, (size_t)cap * 4) != hipSuccess)
            return -1;
        s->frames_cap = cap;
    }
    if (items > s->items_cap) {
        uint64_t cap = items + items / 8;
        (void)hipStreamSynchronize(stream);
        if (s->items)
            (void)hipFree(s->items);
        s->items = nullptr;
        s->items_cap = 0;
        if (hipMalloc((void **)&s->items, cap * 8 + 64) != hipSuccess)
            return -1;
        s->items_cap = cap;
    }
    return 0;
}

// ---- per-stage launch timing (zsk_kernel_timing / zsk_kernel_times) ----------
// Events around the stages of each launch on its stream: [plan, parse,
// execute, hand-off]; read back (and averaged) on request.
namespace {
struct StageTimer {
    std::mutex mu;
    bool on = false;
    std::vector<hipEvent_t> pool;
    std::vector<std::array<hipEvent_t, kTimedStages + 1>> pend;
    double sum[kTimedStages] = {};
    uint64_t n = 0;
};
StageTimer g_timer;
thread_local std::array<hipEvent_t, kTimedStages + 1> t_ev;
thread_local bool t_active = false;

hipEvent_t timer_event()
{
    if (!g_timer.pool.empty()) {
        hipEvent_t e = g_timer.pool.back();
        g_timer.pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}
}   // namespace

void stage_mark(int boundary, hipStream_t stream)
{
    if (boundary == 0) {
        std::lock_guard<std::mutex> g(g_timer.mu);
        t_active = g_timer.on;
        if (!t_active)
            return;
        for (auto &e : t_ev)
            e = timer_event();
    }
    if (!t_active)
        return;
    (void)hipEventRecord(t_ev[boundary], stream);
    if (boundary == kTimedStages) {
        std::lock_guard<std::mutex> g(g_timer.mu);
        g_timer.pend.push_back(t_ev);
        t_active = false;
    }
}

int kernel_timing(int on)
{
    std::lock_guard<std::mutex> g(g_timer.mu);
    for (auto &a : g_timer.pend) {
        (void)hipEventSynchronize(a[kTimedStages]);
        for (auto e : a)
            g_timer.pool.push_back(e);
    }
    g_timer.pend.clear();
    g_timer.on = on != 0;
    for (double &x : g_timer.sum)
        x = 0;
    g_timer.n = 0;
    return 0;
}

int kernel_times(double *ms, int cap)
{
    std::lock_guard<std::mutex> g(g_timer.mu);
    for (auto &a : g_timer.pend) {
        (void)hipEventSynchronize(a[kTimedStages]);
        for (int i = 0; i < kTimedStages; i++) {
            float t = 0;
            if (hipEventElapsedTime(&t, a[i], a[i + 1]) == hipSuccess)
                g_timer.sum[i] += t;
        }
        g_timer.n++;
        for (auto e : a)
            g_timer.pool.push_back(e);
    }
    g_timer.pend.clear();
    for (int i = 0; i < cap && i < kTimedStages; i++)
        ms[i] = g_timer.n ? g_timer.sum[i] / g_timer.n : 0.0;
    return (int)g_timer.n;
}

int launch_lz4_split(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                     uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at,
                     hipStream_t stream, SplitScratch *s, int stages, int diag)
{
    if (nframes == 0)
        return 0;
    if (s->frames_cap < nframes || !s->rec_base || !s->redo)
        return -1;
    uint64_t *total_dev = nullptr;
    (void)hipHostGetDevicePointer((void **)&total_dev, s->total, 0);
    stage_mark(0, stream);
    if (stages & 1) {
        // env ZSEEK_PLAN_SCAN=1 forces the scan layout (A/B runs)
        static const int force_scan = getenv("ZSEEK_PLAN_SCAN") ? 1 : 0;
        (void)hipMemsetAsync(s->redo, force_scan, sizeof(uint32_t), stream);
        hipLaunchKernelGGL(lz4_plan_direct_kernel, dim3((nframes + 255) / 256), dim3(256), 0, stream,
                           d_desc, nframes, s->rec_base, total_dev, s->redo);
        hipLaunchKernelGGL(lz4_plan_kernel, dim3(1), dim3(1024), 0, stream, d_desc, nframes,
                           s->rec_base, total_dev, s->redo);
    }
    stage_mark(1, stream);
    // diag (tuning builds): 0x800 = the first-generation parse kernel,
    // 0x1000 = the first-generation execute kernel (low bits: its variants),
    // 0x400 = the older scan's if/return fast path,
    // 0x200/0x201 = LDS-ring staged execute v1/v2, 0x203..0x20A = seq_exec
    // versions; 0 = the production pair lz4_lean_kernel + seq_exec v17;
    // 0x2000 = every frame to the lane-per-frame parse, 0x4000 = every frame
    // to lz4_chunk_kernel (default: frames of >= chunk_parse_min compressed
    // bytes to the chunk parse, the rest lane per frame); 0x8000 = the older
    // lz4_scan_kernel as the lane-per-frame parse (bits 16-17: lean DIAG).
    // The first-generation execute steps 64 items at a time and needs the
    // older scan's padding items.
    const bool old_parse = (diag & 0x800) != 0, old_exec = (diag & 0x1000) != 0;
    const bool old_scan = (diag & 0x8000) != 0 || old_exec;
    const int xd = diag & 0x3FF;
    const uint32_t cmin = ((diag & 0x2000) || old_exec) ? 0xFFFFFFFFu
                          : (diag & 0x4000)              ? 0u
                                                         : chunk_parse_min(nframes);
    if ((stages & 2) && !old_parse) {
        // lane per frame: lz4_lean_kernel for frames of [kLeanMinCsize, cmin)
        // compressed bytes, lz4_scan_kernel below (or for all with 0x8000)
        const uint32_t smax = old_scan ? cmin : (cmin < kLeanMinCsize ? cmin : kLeanMinCsize);
        if (cmin > smax)
            launch_lz4_lean(d_desc, nframes, d_comp, s->rec_base, (uint64_t)s->items_cap, s->items,
                            s->nitems, d_status, d_fail_at, stream, cmin, (diag >> 16) & 31, smax);
        if (smax != 0)
            launch_lz4_scan(d_desc, nframes, d_comp, s->rec_base, (uint64_t)s->items_cap, s->items,
                            s->nitems, d_status, d_fail_at, stream, (diag & 0x400) ? 1 : 0, smax);
        if (cmin != 0xFFFFFFFFu)
            launch_lz4_chunk(d_desc, nframes, d_comp, s->rec_base, (uint64_t)s->items_cap, s->items,
                             s->nitems, d_status, d_fail_at, stream, cmin);
    } else if (stages & 2)
        hipLaunchKernelGGL(lz4_parse_kernel, dim3((nframes + 255) / 256), dim3(256), 0, stream,
                           d_desc, nframes, d_comp, s->rec_base, (uint64_t)s->items_cap, s->items,
                           s->nitems, d_status, d_fail_at);
    stage_mark(2, stream);
    if ((stages & 4) && !old_exec && xd >= 0x203 && xd <= 0x21F) {
        launch_seq_exec(d_desc, nframes, d_comp, d_out, s->rec_base, s->items, s->nitems, d_status,
                        stream, xd - 0x200);
    } else if ((stages & 4) && !old_exec && (xd == 0x200 || xd == 0x201)) {
        launch_lz4_exec_stage(d_desc, nframes, d_comp, d_out, s->rec_base, s->items, s->nitems,
                              d_status, stream, xd == 0x201 ? 2 : 1);
    } else if ((stages & 4) && !old_exec) {
        launch_seq_exec(d_desc, nframes, d_comp, d_out, s->rec_base, s->items, s->nitems, d_status,
                        stream, 17);
    } else if (stages & 4) {
        const dim3 grid((nframes + kExecWaves - 1) / kExecWaves), block(64 * kExecWaves);
#define ZSK_EXEC(D, O)                                                                          \
    hipLaunchKernelGGL((lz4_exec_kernel<D, O>), grid, block, 0, stream, d_desc, nframes, d_comp, \
                       d_out, s->rec_base, s->items, s->nitems, d_status)
        switch (xd) {
        case 1: ZSK_EXEC(1, 1); break;
        case 2: ZSK_EXEC(2, 1); break;
        case 8: ZSK_EXEC(8, 1); break;
        case 16: ZSK_EXEC(16, 1); break;
        case 0x106: ZSK_EXEC(0, 6); break;
        case 0x108: ZSK_EXEC(0, 8); break;
        default: ZSK_EXEC(0, 1); break;
        }
#undef ZSK_EXEC
    }
    stage_mark(3, stream);
    if (hipGetLastError() != hipSuccess) {
        stage_mark(4, stream);
        return -1;
    }
    int rc = 0;
    if (stages & 8)
        rc = launch_lz4_wave_deferred(d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream);
    stage_mark(4, stream);
    return rc;
}

// Public device API (zsk_lz4_decode_frames): the host does not see the
// descriptors, so scratch is kept per (device, stream) and sized from the
// frame count and the item total the previous plan on that stream reported;
// frames that do not fit go to the wave kernel and the next call grows.
int launch_lz4_frames(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                      uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream)
{
    if (nframes == 0)
        return 0;
    switch (lz4_pick_engine(nframes)) {
    case ENGINE_LANE: return launch_lz4_lane(d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream);
    case ENGINE_WAVE: return launch_lz4_wave(0, d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream);
    default: break;
    }
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, SplitScratch> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    SplitScratch &s = cache[{dev, stream}];
    // first call: room for 64 KiB frames (capped at 2 GiB of items); later
    // calls: what the previous plan on this stream needed
    uint64_t want = (uint64_t)nframes * slots_of(65536 + 64);
    if (want > (512ull << 20))
        want = 512ull << 20;
    if (s.total && *s.total > want)
        want = *s.total;
    if (split_scratch_reserve(&s, nframes, want, stream) != 0)
        return launch_lz4_wave(0, d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream);
    return launch_lz4_split(d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream, &s);
}

// Automatic choice: the two-phase decoder (its parse per frame
// size and batch size, chunk_parse_min) from 64 frames on; a handful of frames
// go to the wave-per-frame kernel in one launch.
int lz4_pick_engine(uint32_t nframes)
{
    const int e = lz4_engine();
    if (e != ENGINE_AUTO)
        return e;
    return nframes >= 64 ? ENGINE_SPLIT : ENGINE_WAVE;
}

uint32_t chunk_parse_min(uint32_t nframes)
{
    static const int forced = [] {
        const char *v = getenv("ZSEEK_PARSE");
        if (v && !strcmp(v, "scan"))
            return 1;
        if (v && !strcmp(v, "chunk"))
            return 2;
        return 0;
    }();
    if (forced == 1)
        return 0xFFFFFFFFu;
    if (forced == 2)
        return 0;
    return nframes >= 32768 ? 49152u : 8192u;
}

int lz4_engine()
{
    static const int e = [] {
        const char *v = getenv("ZSEEK_HIP_KERNEL");
        if (!v)
            return (int)ENGINE_AUTO;
        if (!strcmp(v, "lane"))
            return (int)ENGINE_LANE;
        if (!strcmp(v, "split"))
            return (int)ENGINE_SPLIT;
        if (!strcmp(v, "wave"))
            return (int)ENGINE_WAVE;
        return (int)ENGINE_AUTO;
    }();
    return e;
}

// Tuning hook: the split decoder with a subset of its stages (bitmask:
// 1 plan, 2 parse, 4 exec, 8 hand-offs to the wave kernel).
int launch_lz4_split_stages(int stages, int diag, const FrameDesc *d_desc, uint32_t nframes,
                            const uint8_t *d_comp, uint8_t *d_out, int32_t *d_status,
                            hipStream_t stream)
{
    static std::mutex mu;
    static SplitScratch s;
    std::lock_guard<std::mutex> g(mu);
    uint64_t want = (uint64_t)nframes * slots_of(65536 + 64);
    if (want > (256ull << 20))
        want = 256ull << 20;
    if (s.total && *s.total > want)
        want = *s.total;
    if (split_scratch_reserve(&s, nframes, want, stream) != 0)
        return -1;
    if ((diag & 0x1000) && (diag & 8)) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_exec_stats), z, sizeof(z), 0,
                                     hipMemcpyHostToDevice, stream);
    }
    int rc = launch_lz4_split(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream, &s,
                              stages, diag);
    if ((diag & 0x1000) && (diag & 8)) {
        unsigned long long z[8];
        (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_exec_stats), sizeof(z), 0,
                                       hipMemcpyDeviceToHost, stream);
        (void)hipStreamSynchronize(stream);
        fprintf(stderr,
                "exec stats: batches %llu rounds %llu (%.2f/batch) sequences %llu long-lit %llu "
                "long-match %llu round1-resolved %llu\n",
                z[0], z[1], z[0] ? (double)z[1] / z[0] : 0.0, z[4], z[2], z[3], z[5]);
    }
    return rc;
}

const char *lz4_kernel_name(uint32_t nframes)
{
    switch (lz4_pick_engine(nframes)) {
    case ENGINE_LANE: return "lz4_lane_kernel";
    case ENGINE_SPLIT: return nframes >= 32768 ? "seq_exec_kernel" : "lz4_chunk_kernel";
    default: return "lz4_wave_kernel<4096, 4>";
    }
}

}   // namespace zsk
