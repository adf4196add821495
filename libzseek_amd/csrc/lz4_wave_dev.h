// lz4_wave_dev.h -- the wave-per-frame LZ4-frame decoder (WaveDec,
// wave_frame) as device code shared by lz4_wave.hip (the wave kernel and the
// two-phase decoder's hand-off pass) and seq_exec.hip (the one-frame
// execute decodes its batch's hand-offs itself, so a one-frame batch needs
// no hand-off launch).  See lz4_wave.hip for the design.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4_dev.h"
#include "zsk_internal.h"

namespace zsk {
namespace lz4w {

using namespace lz4d;

constexpr uint32_t kFlush = 256;   // bytes per flush chunk (64 lanes x 4 B)

template <int RING>
struct WaveDec {
    static_assert((RING & (RING - 1)) == 0 && RING >= 1024, "RING: power of 2 >= 1 KiB");
    static constexpr uint32_t kMask = RING - 1;

    __amdgpu_buffer_rsrc_t in;    // [frame start aligned down to 4, +roundup(s0+clen,4))
    __amdgpu_buffer_rsrc_t outr;  // [frame output, +dlen)
    uint32_t s0;                  // frame start misalignment (coords = offset + s0)
    uint32_t clen, dlen;
    bool out_aligned;             // frame output base 4-byte aligned
    uint32_t wq;                  // window base coord (multiple of 4)
    uint32_t w0, w1, w2, w3;      // window dwords: [wq, wq+1024)
    uint8_t *ring;                // this wave's LDS ring
    uint32_t flushed;             // output bytes flushed to HBM
    uint32_t fail_op;             // output offset of the block that failed
    uint32_t lane;

    __device__ __forceinline__ uint32_t load_dw(uint32_t coord) const
    {
        return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(in, coord + 4 * lane, 0, 0);
    }

    __device__ __forceinline__ void window_at(uint32_t x)
    {
        wq = x & ~3u;
        w0 = load_dw(wq);
        w1 = load_dw(wq + 256);
        w2 = load_dw(wq + 512);
        w3 = load_dw(wq + 768);
    }

    // Make the window start within 256 B below coord x (so [x, x+256) is held
    // by w0/w1).  Usually one shift; long literal runs may jump further.
    __device__ __forceinline__ void ensure(uint32_t x)
    {
        if (x - wq < 256)
            return;
        if (x - wq >= 768) {
            window_at(x);
            return;
        }
        do {
            w0 = w1;
            w1 = w2;
            w2 = w3;
            wq += 256;
            w3 = load_dw(wq + 768);
        } while (x - wq >= 256);
    }

    // dword k (0..127) of the w0|w1 pair, uniform
    __device__ __forceinline__ uint32_t wdword(uint32_t k) const
    {
        uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)w0, (int)(k & 63));
        uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)w1, (int)(k & 63));
        return k < 64 ? a : b;
    }

    // 4 bytes at frame offset p (requires p+s0-wq < 504)
    __device__ __forceinline__ uint32_t peek32(uint32_t p) const
    {
        uint32_t x = p + s0 - wq;
        uint32_t k = x >> 2;
        uint64_t v = ((uint64_t)wdword(k + 1) << 32) | wdword(k);
        return (uint32_t)(v >> ((x & 3) * 8));
    }

    __device__ __forceinline__ uint32_t byte_at(uint32_t p)
    {
        ensure(p + s0);
        return peek32(p) & 0xFF;
    }

    // ---- output side -----------------------------------------------------
    __device__ __forceinline__ void flush_chunk()
    {
        uint32_t base = flushed;
        uint32_t v = *reinterpret_cast<const uint32_t *>(ring + ((base + 4 * lane) & kMask));
        if (out_aligned) {
            __builtin_amdgcn_raw_buffer_store_b32(v, outr, base + 4 * lane, 0, 0);
        } else {
#pragma unroll
            for (int b = 0; b < 4; b++)
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(v >> (8 * b)), outr,
                                                     base + 4 * lane + b, 0, 0);
        }
        flushed = base + kFlush;
    }

    __device__ __forceinline__ void flush_upto(uint32_t op)
    {
        while (op - flushed >= kFlush)
            flush_chunk();
    }

    __device__ __forceinline__ void flush_tail(uint32_t op)
    {
        flush_upto(op);
        for (uint32_t p = flushed + lane; p < op; p += 64)
            __builtin_amdgcn_raw_buffer_store_b8(ring[p & kMask], outr, p, 0, 0);
        flushed = op;
    }

    // Copy n literal bytes from frame offset ip to output offset op.
    __device__ __forceinline__ void copy_literals(uint32_t ip, uint32_t op, uint32_t n)
    {
        for (uint32_t c = 0; c < n; c += 64) {
            uint32_t x = ip + c + s0;
            ensure(x);
            uint32_t rel = x - wq + lane;           // < 320
            uint32_t k = rel >> 2;
            int addr = (int)((k & 63) << 2);
            uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)w0);
            uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)w1);
            uint32_t dw = k < 64 ? a : b;
            uint8_t byte = (uint8_t)(dw >> ((rel & 3) * 8));
            if (c + lane < n)
                ring[(op + c + lane) & kMask] = byte;
            flush_upto(op + (n - c < 64 ? n : c + 64));
        }
    }

    // Copy an n-byte match at distance off to output offset op.
    __device__ __forceinline__ void copy_match(uint32_t op, uint32_t off, uint32_t n)
    {
        if (off == 0) {   // liblz4 1.9.3 writes zeros for a zero offset
            for (uint32_t c = 0; c < n; c += 64) {
                if (c + lane < n)
                    ring[(op + c + lane) & kMask] = 0;
                flush_upto(op + (n - c < 64 ? n : c + 64));
            }
            return;
        }
        uint32_t c = 0;
        uint32_t eff = off;
        if (off < 64) {
            // first chunk: period-off pattern; then widen the distance to a
            // multiple of off >= 64 so later chunks never overlap themselves
            float r = __builtin_amdgcn_rcpf((float)off);
            uint32_t q = (uint32_t)(((float)lane + 0.5f) * r);
            uint32_t m = lane - q * off;
            uint8_t byte = ring[(op - off + m) & kMask];
            if (lane < n)
                ring[(op + lane) & kMask] = byte;
            flush_upto(op + (n < 64 ? n : 64));
            c = 64;
            eff = off * ((64 + off - 1) / off);
        }
        const bool in_ring = eff <= (uint32_t)RING - 64;
        for (; c < n; c += 64) {
            uint32_t src = op + c - eff + lane;
            uint8_t byte;
            if (in_ring)
                byte = ring[src & kMask];
            else
                byte = __builtin_amdgcn_raw_buffer_load_b8(outr, src, 0, 0);
            if (c + lane < n)
                ring[(op + c + lane) & kMask] = byte;
            flush_upto(op + (n - c < 64 ? n : c + 64));
        }
    }

    // Decode one LZ4 block [ip, ip+bsize) into output starting at op.
    // Returns status; *op_out = output end.
    __device__ __forceinline__ int32_t block(uint32_t ip, uint32_t bsize, uint32_t op, uint32_t cap,
                             uint32_t floor_, uint32_t *op_out)
    {
        const uint32_t iend = ip + bsize;
        const uint32_t oend = op + cap;
        if (bsize == 0)
            return ST_BLOCK_ERR;
        for (;;) {
            if (ip >= iend)
                return ST_BLOCK_ERR;
            ensure(ip + s0);
            uint32_t t4 = peek32(ip);
            uint32_t tok = t4 & 0xFF;
            uint32_t lit = tok >> 4;
            uint32_t p = ip + 1;
            if (lit == 15) {
                if (iend - p <= 15)
                    return ST_BLOCK_ERR;
                uint32_t s;
                do {
                    if (p >= iend)
                        return ST_BLOCK_ERR;
                    s = byte_at(p++);
                    lit += s;
                } while (s == 255);
            }
            if (op + lit > oend - kMfLimit || iend - p < lit + 2 + 1 + kLastLiterals) {
                // must be the last sequence: literals only, exactly to iend
                if (iend - p != lit || op + lit > oend)
                    return ST_BLOCK_ERR;
                if (op + lit > dlen)
                    return ST_DST_OVERFLOW;
                copy_literals(p, op, lit);
                *op_out = op + lit;
                return ST_OK;
            }
            if (op + lit > dlen)
                return ST_DST_OVERFLOW;
            if (lit)
                copy_literals(p, op, lit);
            p += lit;
            op += lit;
            ensure(p + s0);
            uint32_t o4 = peek32(p);
            uint32_t off = o4 & 0xFFFF;
            p += 2;
            uint32_t ml = tok & 15;
            if (ml == 15) {
                uint32_t s;
                do {
                    if (p >= iend)
                        return ST_BLOCK_ERR;
                    s = byte_at(p++);
                    ml += s;
                    if (p >= iend - (kLastLiterals - 1))
                        return ST_BLOCK_ERR;
                } while (s == 255);
            }
            ml += kMinMatch;
            // offset 0 is accepted as liblz4 1.9.3 does (zeros; oracle
            // decode_block)
            if (off > op - floor_)
                return ST_BLOCK_ERR;
            if (op + ml > oend - kLastLiterals)
                return ST_BLOCK_ERR;
            if (op + ml > dlen)
                return ST_DST_OVERFLOW;
            copy_match(op, off, ml);
            op += ml;
            ip = p;
        }
    }

    // Decode the whole LZ4 frame; returns status (code | direct flag).
    __device__ __forceinline__ int32_t frame()
    {
        if (clen < 7)
            return ST_HDR_INCOMPLETE;
        window_at(s0);
        uint32_t magic = peek32(0);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u)
            return ST_SHORT_FRAME;
        if (magic != kLz4Magic)
            return ST_FRAME_TYPE;
        uint32_t desc = peek32(4);
        uint32_t flg = desc & 0xFF, bd = (desc >> 8) & 0xFF;
        uint32_t block_ck = (flg >> 4) & 1, indep = (flg >> 5) & 1;
        uint32_t csize_flag = (flg >> 3) & 1, content_ck = (flg >> 2) & 1;
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
        // header checksum: (XXH32(descriptor, 0) >> 8) & 0xFF
        {
            uint32_t hc = xxh32_small(4, hdr - 5);
            if (((hc >> 8) & 0xFF) != byte_at(hdr - 1))
                return ST_HDR_CHECKSUM;
        }
        uint64_t content_size = 0;
        if (csize_flag)
            content_size = (uint64_t)peek32(6) | ((uint64_t)peek32(10) << 32);
        const uint32_t max_block = 1u << (8 + 2 * bsid);
        uint32_t ip = hdr;
        uint32_t op = 0;
        flushed = 0;
        for (;;) {
            fail_op = op;
            if (clen - ip < 4)
                return ST_TRUNCATED;
            ensure(ip + s0);
            uint32_t bh = peek32(ip);
            ip += 4;
            if (bh == 0)
                break;
            uint32_t bsize = bh & 0x7FFFFFFFu;
            if (bsize > max_block)
                return ST_MAXBLOCK;
            uint32_t need = bsize + (block_ck ? 4 : 0);
            if (clen - ip < need)
                return ST_TRUNCATED;
            if (block_ck) {
                uint32_t h = xxh32_in(ip, bsize);
                ensure(ip + bsize + s0);
                if (h != peek32(ip + bsize))
                    return ST_BLOCK_CHECKSUM;
            }
            if (bh & 0x80000000u) {
                if (op + bsize > dlen)
                    return ST_DST_OVERFLOW;
                copy_literals(ip, op, bsize);
                op += bsize;
            } else {
                uint32_t floor_ = indep ? op : 0;   // offsets <= 65535 anyway
                uint32_t nop = op;
                int32_t st = block(ip, bsize, op, max_block, floor_, &nop);
                if (st != ST_OK) {
                    if (st == ST_BLOCK_ERR) {
                        // liblz4 reports GENERIC when it decodes straight
                        // into dst (room >= max block), else
                        // decompressionFailed (via its tmp buffer).  Room
                        // here = the rest of the frame (the reference's
                        // cached path); the host re-derives it for no-cache
                        // reads from fail_op and the block size id.
                        bool direct = (dlen - op) >= max_block;
                        int32_t bits = (int32_t)((bsid - 4) << ST_BSID_SHIFT);
                        return (direct ? (ST_GENERIC | ST_DIRECT_FLAG) : ST_DECOMPRESS_FAILED) |
                               ST_BLOCK_FAIL_FLAG | bits;
                    }
                    return st;
                }
                op = nop;
            }
            ip += need;
        }
        flush_tail(op);
        fail_op = op;
        if (csize_flag && content_size != op)
            return ST_FRAME_SIZE;
        if (content_ck) {
            if (clen - ip < 4)
                return ST_TRUNCATED;
            uint32_t h = xxh32_out(op);
            ensure(ip + s0);
            if (h != peek32(ip))
                return ST_CONTENT_CHECKSUM;
        }
        if (op != dlen)
            return ST_SHORT_FRAME;
        return ST_OK;
    }

    // ---- XXH32 helpers (rare paths: header / block / content checksums) ----
    static __device__ __forceinline__ uint32_t rotl(uint32_t x, int r)
    {
        return (x << r) | (x >> (32 - r));
    }

    __device__ __forceinline__ uint32_t xxh32_finish(uint32_t acc, uint32_t len, uint32_t tail_p, bool from_out,
                                     uint32_t tail_len)
    {
        acc += len;
        uint32_t i = 0;
        for (; i + 4 <= tail_len; i += 4) {
            uint32_t w = 0;
            for (int b = 0; b < 4; b++)
                w |= get(tail_p + i + b, from_out) << (8 * b);
            acc += w * 0xC2B2AE3Du;
            acc = rotl(acc, 17) * 0x27D4EB2Fu;
        }
        for (; i < tail_len; i++) {
            acc += get(tail_p + i, from_out) * 0x165667B1u;
            acc = rotl(acc, 11) * 0x9E3779B1u;
        }
        acc ^= acc >> 15;
        acc *= 0x85EBCA77u;
        acc ^= acc >> 13;
        acc *= 0xC2B2AE3Du;
        acc ^= acc >> 16;
        return acc;
    }

    __device__ __forceinline__ uint32_t get(uint32_t p, bool from_out)
    {
        if (from_out)
            return uni(__builtin_amdgcn_raw_buffer_load_b8(outr, p, 0, 0));
        return byte_at(p);
    }

    // XXH32 (seed 0) over n bytes at frame offset / output offset p: simple
    // scalar stripes, used only for checksummed frames.
    __device__ __forceinline__ uint32_t xxh32_any(uint32_t p, uint32_t n, bool from_out)
    {
        uint32_t acc;
        uint32_t i = 0;
        if (n >= 16) {
            uint32_t a[4] = {0x9E3779B1u + 0x85EBCA77u, 0x85EBCA77u, 0u, 0u - 0x9E3779B1u};
            for (; i + 16 <= n; i += 16) {
                for (int l = 0; l < 4; l++) {
                    uint32_t w = 0;
                    for (int b = 0; b < 4; b++)
                        w |= get(p + i + 4 * l + b, from_out) << (8 * b);
                    a[l] += w * 0x85EBCA77u;
                    a[l] = rotl(a[l], 13) * 0x9E3779B1u;
                }
            }
            acc = rotl(a[0], 1) + rotl(a[1], 7) + rotl(a[2], 12) + rotl(a[3], 18);
        } else {
            acc = 0x165667B1u;
        }
        return xxh32_finish(acc, n, p + i, from_out, n - i);
    }

    __device__ __forceinline__ uint32_t xxh32_small(uint32_t p, uint32_t n) { return xxh32_any(p, n, false); }
    __device__ __forceinline__ uint32_t xxh32_in(uint32_t p, uint32_t n) { return xxh32_any(p, n, false); }
    __device__ __forceinline__ uint32_t xxh32_out(uint32_t n)
    {
        // the output was flushed by flush_tail; make the stores visible to
        // this wave's own loads before re-reading them
        __builtin_amdgcn_s_waitcnt(0);
        return xxh32_any(0, n, true);
    }
};

// One frame f (wave-uniform) on this wave, its ring at `ring`.
template <int RING>
__device__ __forceinline__ void wave_frame(const FrameDesc *__restrict__ desc, uint32_t f,
                                           const uint8_t *__restrict__ comp, uint8_t *__restrict__ out,
                                           int32_t *__restrict__ status, uint32_t *__restrict__ fail_at,
                                           uint8_t *ring)
{
    const FrameDesc d = desc[f];
    WaveDec<RING> w;
    w.lane = threadIdx.x & 63;
    const uint8_t *cbase = comp + d.c_off;
    uintptr_t ca = reinterpret_cast<uintptr_t>(cbase);
    w.s0 = uni((uint32_t)(ca & 3));
    w.clen = uni(d.c_size);
    w.dlen = uni(d.d_size);
    w.in = __builtin_amdgcn_make_buffer_rsrc((void *)(ca & ~(uintptr_t)3), 0,
                                             (int)((w.s0 + w.clen + 3) & ~3u), kRsrcDw3);
    uint8_t *obase = out + d.d_off;
    w.outr = __builtin_amdgcn_make_buffer_rsrc(obase, 0, (int)w.dlen, kRsrcDw3);
    w.out_aligned = (reinterpret_cast<uintptr_t>(obase) & 3) == 0;
    w.ring = ring;
    w.flushed = 0;
    w.fail_op = 0;
    int32_t st = w.frame();
    // a failed frame keeps the bytes of its blocks before the failing one
    // (fail_op): no-cache reads ending there succeed, as in the reference
    if (st != ST_OK && w.fail_op > w.flushed)
        w.flush_tail(w.fail_op);
    if (w.lane == 0) {
        status[f] = st;
        if (fail_at)
            fail_at[f] = w.fail_op;
    }
}

}   // namespace lz4w
}   // namespace zsk
