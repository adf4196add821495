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

#include <map>
#include <mutex>
#include <utility>

#include "zsk_internal.h"

namespace zsk {

namespace {

constexpr uint32_t kRsrcDw3 = 0x00020000u;   // gfx9-family raw buffer, 32-bit data
constexpr uint32_t kLz4Magic = 0x184D2204u;
constexpr uint32_t kMinMatch = 4;
constexpr uint32_t kMfLimit = 12;
constexpr uint32_t kLastLiterals = 5;
constexpr uint32_t kItemStored = 0x80000000u;
constexpr uint32_t kItemLast = 0x40000000u;
constexpr uint32_t kItemPos = 0x3FFFFFFFu;
constexpr uint32_t kExecWaves = 4;
constexpr uint32_t kLongRun = 128;   // longer literal runs / matches: copied by the whole wave

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));
typedef uint64_t u64_u __attribute__((aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));

__device__ __forceinline__ uint32_t uni(uint32_t v)
{
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ uint32_t slots_of(uint32_t c_size)
{
    return (c_size / 3 + 2 + 3) & ~3u;
}

// byte i (0..15) of a 16-byte register vector
__device__ __forceinline__ uint32_t vbyte(const u32x4 &w, uint32_t i)
{
    uint32_t d = (i & 8) ? ((i & 4) ? w.w : w.z) : ((i & 4) ? w.y : w.x);
    return (d >> ((i & 3) * 8)) & 0xFF;
}

// 32 bits starting at byte i (0..12) of a 16-byte register vector
__device__ __forceinline__ uint32_t vword(const u32x4 &w, uint32_t i)
{
    uint32_t k = i >> 2;
    uint32_t lo = (k & 2) ? ((k & 1) ? w.w : w.z) : ((k & 1) ? w.y : w.x);
    uint32_t hi = (k & 2) ? w.w : ((k & 1) ? w.z : w.y);
    return __builtin_amdgcn_alignbyte(hi, lo, i & 3);
}

// 16 bytes at byte coordinate x of a buffer resource whose base is 4-byte
// aligned.  Loads are dword-aligned: the hardware range-checks every dword
// of a buffer load on its own (a dword straddling num_records reads as 0), so
// unaligned 16-byte loads would lose the last bytes of a range; aligned
// dwords with num_records rounded up to 4 never do.
__device__ __forceinline__ u32x4 load16u(__amdgpu_buffer_rsrc_t r, uint32_t x)
{
    const uint32_t a = x & ~3u, sh = x & 3;
    const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, a, 0, 0));
    const uint32_t e = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, a + 16, 0, 0);
    u32x4 o;
    o.x = __builtin_amdgcn_alignbyte(v.y, v.x, sh);
    o.y = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
    o.z = __builtin_amdgcn_alignbyte(v.w, v.z, sh);
    o.w = __builtin_amdgcn_alignbyte(e, v.w, sh);
    return o;
}

// A byte range [p0, p0+len) of device memory as (aligned resource, bias):
// frame offset p lives at resource coordinate p + s0.
struct Span {
    __amdgpu_buffer_rsrc_t r;
    uint32_t s0;
};

__device__ __forceinline__ Span make_span(const uint8_t *p0, uint64_t len)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p0);
    Span s;
    s.s0 = (uint32_t)(a & 3);
    s.r = __builtin_amdgcn_make_buffer_rsrc((void *)(a & ~(uintptr_t)3), 0,
                                            (int)(uint32_t)((s.s0 + len + 3) & ~3ull), kRsrcDw3);
    return s;
}

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

// Items of one frame, written 4 at a time (16-B aligned).
struct Sink {
    uint32_t *base;
    uint32_t k, cap;
    u32x4 acc;

    __device__ __forceinline__ bool put(uint32_t x)
    {
        if (k >= cap)
            return false;
        uint32_t s = k & 3;
        acc.x = s == 0 ? x : acc.x;
        acc.y = s == 1 ? x : acc.y;
        acc.z = s == 2 ? x : acc.z;
        acc.w = s == 3 ? x : acc.w;
        k++;
        if ((k & 3) == 0)
            *reinterpret_cast<u32x4 *>(base + k - 4) = acc;
        return true;
    }
    __device__ __forceinline__ void finish()
    {
        if (k & 3)
            *reinterpret_cast<u32x4 *>(base + (k & ~3u)) = acc;
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
            if (!sink.put(ip | kItemLast))
                return ST_NOT_RUN;
            *op_out = op + lit;
            return ST_OK;
        }
        if (op + lit > dlen)
            return ST_DST_OVERFLOW;
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
        if (off == 0 || off > op - floor_)
            return ST_BLOCK_ERR;
        if (op + ml > oend - kLastLiterals)
            return ST_BLOCK_ERR;
        if (op + ml > dlen)
            return ST_DST_OVERFLOW;
        if (!sink.put(ip))
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
            if (!sink.put(ip | kItemStored))
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

__device__ __forceinline__ uint64_t wave_min64(uint64_t v)
{
    for (int m = 32; m >= 1; m >>= 1) {
        uint64_t o = __shfl_xor(v, m, 64);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_max64(uint64_t v)
{
    for (int m = 32; m >= 1; m >>= 1) {
        uint64_t o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
    }
    return v;
}

// ---- plan: per-frame item slot offsets ------------------------------------
__global__ __launch_bounds__(1024) void lz4_plan_kernel(const FrameDesc *__restrict__ desc,
                                                        uint32_t n, uint64_t *__restrict__ rec_base,
                                                        uint64_t *__restrict__ total)
{
    __shared__ uint64_t part[1024];
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
                                                        uint64_t capacity, uint32_t *__restrict__ items,
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

// store the first n (1..16) bytes of v at p, never touching p[n..]
__device__ __forceinline__ void store_exact(uint8_t *p, u32x4 v, uint32_t n)
{
    if (n >= 16) {
        *reinterpret_cast<u32x4_u *>(p) = v;
        return;
    }
    if (n & 8) {
        *reinterpret_cast<u64_u *>(p) = ((uint64_t)v.y << 32) | v.x;
        p += 8;
        v.x = v.z;
        v.y = v.w;
    }
    if (n & 4) {
        *reinterpret_cast<u32_u *>(p) = v.x;
        p += 4;
        v.x = v.y;
    }
    if (n & 2) {
        p[0] = (uint8_t)v.x;
        p[1] = (uint8_t)(v.x >> 8);
        p += 2;
        v.x >>= 16;
    }
    if (n & 1)
        p[0] = (uint8_t)v.x;
}

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
__device__ __noinline__ void copy_match_wave(uint8_t *out, const Span &orr, uint32_t dst,
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

// Diagnostic counters of the exec kernel (tuning builds only, DIAG & 8):
// [0] batches, [1] resolution rounds, [2] long literal runs, [3] long matches,
// [4] sequences, [5] matches resolved in round 1
__device__ unsigned long long g_exec_stats[8];

// DIAG (tuning builds): 1 = no wait between resolution rounds, 2 = skip
// back-references, 4 = skip all copies, 8 = count (g_exec_stats)
template <int DIAG>
__global__ __launch_bounds__(64 * kExecWaves) void lz4_exec_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ rec_base,
    const uint32_t *__restrict__ items, const uint32_t *__restrict__ nitems,
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
    const uint32_t *it = items + rec_base[f];
    uint8_t *o = out + d.d_off;
    const Span osp = make_span(o, d.d_size);
    const Span sp = make_span(comp + d.c_off, d.c_size);
    LaneIn in;
    in.r = sp.r;
    in.s0 = sp.s0;
    in.wp = 0x80000000u;
    uint32_t obase = 0;
    for (uint32_t b = 0; b < nit; b += 64) {
        const uint32_t j = b + lane;
        const bool act = j < nit;
        uint32_t lit = 0, ml = 0, off = 0, src = 0;
        if (act) {
            const uint32_t item = it[j];
            const uint32_t pos = item & kItemPos;
            if (item & kItemStored) {
                lit = in.word(pos - 4) & 0x7FFFFFFFu;
                src = pos;
            } else {
                in.at(pos);
                uint32_t tok = in.byte(pos);
                lit = tok >> 4;
                uint32_t p = pos + 1;
                if (lit == 15) {
                    uint32_t s;
                    do {
                        s = in.byte(p++);
                        lit += s;
                    } while (s == 255);
                }
                src = p;
                if (!(item & kItemLast)) {
                    p += lit;
                    off = in.word(p) & 0xFFFF;
                    p += 2;
                    ml = tok & 15;
                    if (ml == 15) {
                        uint32_t s;
                        do {
                            s = in.byte(p++);
                            ml += s;
                        } while (s == 255);
                    }
                    ml += kMinMatch;
                }
            }
        }
        // output positions: exclusive wave prefix sum of lit + ml
        const uint32_t len = lit + ml;
        uint32_t inc = len;
        for (uint32_t dlt = 1; dlt < 64; dlt <<= 1) {
            uint32_t v = __shfl_up(inc, dlt, 64);
            if (lane >= dlt)
                inc += v;
        }
        const uint32_t op = obase + inc - len;
        obase += (uint32_t)__shfl(inc, 63, 64);
        if (DIAG & 8) {
            if (lane == 0) {
                atomicAdd(&g_exec_stats[0], 1ull);
                atomicAdd(&g_exec_stats[4], (unsigned long long)(nit - b < 64 ? nit - b : 64));
            }
        }
        if (DIAG & 4)
            continue;
        // literal runs: compressed image -> output; a lane copies its own
        // short run, long runs (and stored blocks) are copied by the wave
        if ((DIAG & 8) && lane == 0) {
            atomicAdd(&g_exec_stats[2], (unsigned long long)__popcll(__ballot(lit > kLongRun)));
            atomicAdd(&g_exec_stats[3], (unsigned long long)__popcll(__ballot(ml > kLongRun)));
        }
        if (lit <= kLongRun) {
            for (uint32_t k = 0; k < lit; k += 16) {
                u32x4 v = in.load16(src + k);
                uint32_t r = lit - k;
                store_exact(o + op + k, v, r < 16 ? r : 16);
            }
        }
        for (uint64_t lm = __ballot(lit > kLongRun); lm; lm &= lm - 1) {
            const int l = __builtin_ctzll(lm);
            const uint32_t ls = uni_lane(src, l), lo = uni_lane(op, l), ln = uni_lane(lit, l);
            for (uint32_t k = 16 * lane; k < ln; k += 1024) {
                u32x4 v = in.load16(ls + k);
                uint32_t r = ln - k;
                store_exact(o + lo + k, v, r < 16 ? r : 16);
            }
        }
        // back-references, multi-round resolution
        const uint32_t mb = op + lit;
        const uint32_t me = mb + ml;
        const uint32_t msrc = mb - off;
        const uint32_t need = off >= ml ? msrc + ml : mb;   // end of the bytes the copy reads
        uint64_t pending = (DIAG & 2) ? 0 : __ballot(ml != 0);
        bool first_round = true;
        while (pending) {
            if (!(DIAG & 1))
                __builtin_amdgcn_s_waitcnt(0);   // earlier rounds' stores complete
            // lane k may copy once its source range [msrc, need) misses every
            // pending match below it: it ends before the lowest pending
            // match starts, or starts after the nearest pending one below
            // ends (pending ranges are ordered by lane)
            const uint64_t below = pending & ((1ull << lane) - 1);
            const int hb = below ? 63 - __builtin_clzll(below) : (int)lane;
            const uint32_t me_hb = (uint32_t)__shfl(me, hb, 64);
            const uint32_t frontier = uni_lane(mb, __builtin_ctzll(pending));
            const bool mine = (pending >> lane) & 1;
            const bool ready = mine && (below == 0 || need <= frontier || msrc >= me_hb);
            if (ready && ml <= kLongRun)
                copy_match(o, osp, mb, off, ml);
            const uint64_t rmask = __ballot(ready);
            for (uint64_t lm = __ballot(ready && ml > kLongRun); lm; lm &= lm - 1) {
                const int l = __builtin_ctzll(lm);
                copy_match_wave(o, osp, uni_lane(mb, l), uni_lane(off, l), uni_lane(ml, l), lane);
            }
            pending &= ~rmask;
            if (DIAG & 8) {
                if (lane == 0) {
                    atomicAdd(&g_exec_stats[1], 1ull);
                    if (first_round)
                        atomicAdd(&g_exec_stats[5], (unsigned long long)__popcll(rmask));
                }
            }
            first_round = false;
        }
    }
}

}   // namespace

// ---- host side ---------------------------------------------------------------

uint64_t split_items_needed(const FrameDesc *h_desc, uint32_t n)
{
    uint64_t s = 0;
    for (uint32_t i = 0; i < n; i++)
        s += (h_desc[i].c_size / 3 + 2 + 3) & ~3u;
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
    *s = SplitScratch();
}

int split_scratch_reserve(SplitScratch *s, uint32_t frames, uint64_t items, hipStream_t stream)
{
    if (!s->total) {
        if (hipHostMalloc((void **)&s->total, sizeof(uint64_t), hipHostMallocMapped) != hipSuccess)
            return -1;
        *s->total = 0;
    }
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
        if (hipMalloc((void **)&s->items, cap * 4 + 64) != hipSuccess)
            return -1;
        s->items_cap = cap;
    }
    return 0;
}

int launch_lz4_split(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                     uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at,
                     hipStream_t stream, SplitScratch *s, int stages, int diag)
{
    if (nframes == 0)
        return 0;
    if (s->frames_cap < nframes || !s->rec_base)
        return -1;
    uint64_t *total_dev = nullptr;
    (void)hipHostGetDevicePointer((void **)&total_dev, s->total, 0);
    if (stages & 1)
        hipLaunchKernelGGL(lz4_plan_kernel, dim3(1), dim3(1024), 0, stream, d_desc, nframes,
                           s->rec_base, total_dev);
    if (stages & 2)
        hipLaunchKernelGGL(lz4_parse_kernel, dim3((nframes + 255) / 256), dim3(256), 0, stream,
                           d_desc, nframes, d_comp, s->rec_base, (uint64_t)s->items_cap, s->items,
                           s->nitems, d_status, d_fail_at);
    if (stages & 4) {
        const dim3 grid((nframes + kExecWaves - 1) / kExecWaves), block(64 * kExecWaves);
#define ZSK_EXEC(D)                                                                            \
    hipLaunchKernelGGL(lz4_exec_kernel<D>, grid, block, 0, stream, d_desc, nframes, d_comp, d_out, \
                       s->rec_base, s->items, s->nitems, d_status)
        switch (diag) {
        case 1: ZSK_EXEC(1); break;
        case 2: ZSK_EXEC(2); break;
        case 4: ZSK_EXEC(4); break;
        case 8: ZSK_EXEC(8); break;
        default: ZSK_EXEC(0); break;
        }
#undef ZSK_EXEC
    }
    if (hipGetLastError() != hipSuccess)
        return -1;
    if (stages & 8)
        return launch_lz4_wave_deferred(d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream);
    return 0;
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
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, SplitScratch> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    SplitScratch &s = cache[{dev, stream}];
    uint64_t want = (uint64_t)nframes * 21856;   // 64 KiB frames at any ratio
    if (s.total && *s.total > want)
        want = *s.total;
    if (split_scratch_reserve(&s, nframes, want, stream) != 0)
        return launch_lz4_wave(0, d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream);
    return launch_lz4_split(d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream, &s);
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
    if (split_scratch_reserve(&s, nframes, (uint64_t)nframes * 21856, stream) != 0)
        return -1;
    if (diag & 8) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_exec_stats), z, sizeof(z), 0,
                                     hipMemcpyHostToDevice, stream);
    }
    int rc = launch_lz4_split(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream, &s,
                              stages, diag);
    if (diag & 8) {
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

const char *lz4_kernel_name()
{
    return "lz4_exec_kernel";
}

}   // namespace zsk
