// lz4_decode.hip — batched LZ4-frame decoder for CDNA4 (gfx950).
//
// Replaces the per-frame liblz4 call of the reference hot path
// (/root/reference/src/decompress.c:752-773, LZ4F_decompress in a loop) with
// ONE grid over every frame a zseek_pread range covers.
//
// Mapping:
//   * a wave64 decodes G = 64/L frames at once: lane group g (L lanes) owns
//     one seek-table frame.  All parse state (ip, op, block bounds, ...) is
//     group-uniform but lives in VGPRs, so the token parse of G frames costs
//     ONE stream of vector instructions spread over the CU's four SIMDs —
//     a one-frame-per-wave scalar parse saturates the CU's single scalar
//     unit instead (measured: 125 SALU per sequence, 0.94 SALU/cycle/CU);
//   * the compressed frame streams through a per-frame LDS input window
//     (2 x CHUNK bytes, CHUNK = 16 B x L): each lane prefetches its 16 B of
//     the next chunk into registers (one coalesced global_load_dwordx4 per
//     lane) a whole chunk ahead of use; tokens / offsets are read from the
//     window with ds_read2_b32 + v_alignbyte;
//   * decoded bytes land in a per-frame LDS ring (RING bytes); matches whose
//     source is still in the ring are copied LDS -> LDS, older sources are
//     re-read from the frame's already-flushed output in HBM;
//   * completed CHUNK-byte ring slices are flushed with one 16-B store per
//     lane (global_store_dwordx4).
//
// Validation follows liblz4 1.9.3 (the library the reference links) so that
// success/failure matches the reference; oracle/lz4_oracle.c restates the same
// rules on the CPU.  Every global access is bounded by the frame's seek-table
// sizes (reads clamp into the frame, writes never pass dSize).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zsk_internal.h"

namespace zsk {

namespace {

constexpr uint32_t kLz4Magic = 0x184D2204u;
constexpr uint32_t kMinMatch = 4;
constexpr uint32_t kMfLimit = 12;
constexpr uint32_t kLastLiterals = 5;

enum : uint32_t { M_DONE = 0, M_BLKHDR = 1, M_SEQ = 2 };

__device__ __forceinline__ uint32_t align_bytes(uint32_t hi, uint32_t lo, uint32_t sh)
{
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// Per-group decode context.  Every member is uniform across the L lanes of
// a group but differs between groups: the compiler keeps it in VGPRs.
template <int L, int RING, int CM = 1, int DIAG = 0>
struct Group {
    static constexpr uint32_t CHUNK = 16 * L * CM;   // input refill / output flush size
    static constexpr uint32_t IWIN = 2 * CHUNK;   // input window (LDS)
    static constexpr uint32_t RMASK = RING - 1;
    static_assert((RING & (RING - 1)) == 0, "RING must be a power of two");
    static_assert(RING >= 64 * L, "RING too small for the flush slice");
    // match sources at distance <= NEAR are still in the ring
    static constexpr uint32_t NEAR = RING - 16 * L - 2 * L;

    uint32_t gl;                 // lane within group
    const uint8_t *cab;          // compressed frame base, aligned down to 16
    uint32_t s0;                 // misalignment: coord = offset + s0
    uint32_t clen, climit;       // compressed size; coord limit (16-aligned)
    uint8_t *obase;              // decoded frame base in HBM
    uint32_t dlen;
    bool oal;                    // obase 16-byte aligned
    uint32_t filled;             // window holds coords [filled - IWIN, filled)
    uint4 pf[CM];                // prefetched 16*CM B of chunk [filled, +CHUNK)
    uint8_t *ring;               // LDS: RING bytes
    uint8_t *iwin;               // LDS: IWIN + 16 (guard) bytes
    uint32_t flushed;            // decoded bytes stored to HBM

    __device__ __forceinline__ void load_chunk(uint32_t coord)
    {
#pragma unroll
        for (int k = 0; k < CM; k++) {
            uint32_t c = coord + 16 * (gl + L * k);
            c = c < climit ? c : 0;   // clamp inside the frame (bytes past
                                      // the frame are never parsed)
            pf[k] = *reinterpret_cast<const uint4 *>(cab + c);
        }
    }

    __device__ __forceinline__ void refill()
    {
#pragma unroll
        for (int k = 0; k < CM; k++) {
            uint32_t at = (filled & (IWIN - 1)) + 16 * (gl + L * k);
            *reinterpret_cast<uint4 *>(iwin + at) = pf[k];
            if (at == 0)   // mirror the window head past its end (2-dword reads)
                *reinterpret_cast<uint4 *>(iwin + IWIN) = pf[k];
        }
        filled += CHUNK;
        load_chunk(filled);
    }

    __device__ __forceinline__ void window_reset(uint32_t x)
    {
        filled = x & ~(CHUNK - 1);
        load_chunk(filled);
        refill();
        refill();
    }

    // make coords [x, x+need) readable (need <= CHUNK)
    __device__ __forceinline__ void ensure(uint32_t x, uint32_t need)
    {
        if (x + need > filled + CHUNK || x < filled - IWIN)
            window_reset(x);
        while (x + need > filled)
            refill();
    }

    // 4 bytes at coord x (window must hold [x, x+8))
    __device__ __forceinline__ uint32_t peek32(uint32_t x) const
    {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(iwin);
        uint32_t k = (x & (IWIN - 1)) >> 2;
        return align_bytes(w[k + 1], w[k], x & 3);
    }

    __device__ __forceinline__ uint32_t fetch32(uint32_t p)
    {
        ensure(p + s0, 8);
        return peek32(p + s0);
    }

    // ---- output side -------------------------------------------------------
    static constexpr uint32_t FSLICE = 16 * L;   // output flush slice

    __device__ __forceinline__ void flush_slice()
    {
        if (DIAG & 2) {   // diagnostic build: no output stores
            flushed += FSLICE;
            return;
        }
        uint32_t at = flushed + 16 * gl;
        uint4 v = *reinterpret_cast<const uint4 *>(ring + (at & RMASK));
        if (oal) {
            *reinterpret_cast<uint4 *>(obase + at) = v;
        } else {
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int b = 0; b < 16; b++)
                obase[at + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
        }
        flushed += FSLICE;
    }

    __device__ __forceinline__ void flush_upto(uint32_t op)
    {
        while (op - flushed >= FSLICE)
            flush_slice();
    }

    __device__ __forceinline__ void flush_tail(uint32_t op)
    {
        flush_upto(op);
        for (uint32_t p = flushed + gl; p < op; p += L)
            obase[p] = ring[p & RMASK];
        flushed = op;
    }

    // ---- fast path: 4 bytes per lane, one 4L-byte step ------------------
    // Write the `n` (< 4 once past the end) valid bytes of v to ring offsets
    // dop..dop+3; lanes' surplus bytes go to a per-frame dummy slot.
    __device__ __forceinline__ void ring_put4(uint32_t dop, uint32_t v, int32_t n)
    {
#pragma unroll
        for (int b = 0; b < 4; b++) {
            uint32_t at = b < n ? ((dop + b) & RMASK) : RING + IWIN + 16;
            ring[at] = (uint8_t)(v >> (8 * b));
        }
    }

    // literal step: bytes [c, c+4L) of the run at frame offset lsrc -> op
    __device__ __forceinline__ void lit_step(uint32_t lsrc, uint32_t op, uint32_t n, uint32_t c)
    {
        uint32_t j = c + 4 * gl;
        uint32_t x = lsrc + s0 + j;
        const uint32_t *w = reinterpret_cast<const uint32_t *>(iwin);
        uint32_t k = (x & (IWIN - 1)) >> 2;
        uint32_t v = align_bytes(w[k + 1], w[k], x & 3);
        ring_put4(op + j, v, (int32_t)n - (int32_t)j);
    }

    // match step: bytes [c, c+4L) of a match at distance off (>= 4L) -> op
    __device__ __forceinline__ void match_step(uint32_t op, uint32_t off, uint32_t n, uint32_t c)
    {
        uint32_t j = c + 4 * gl;
        uint32_t src = op - off + j;
        const uint32_t *r = reinterpret_cast<const uint32_t *>(ring);
        uint32_t k = (src & RMASK) >> 2;
        uint32_t v = align_bytes(r[(k + 1) & (RMASK >> 2)], r[k], src & 3);
        ring_put4(op + j, v, (int32_t)n - (int32_t)j);
    }

    // n literal bytes from frame offset ip to output offset op
    __device__ __forceinline__ void copy_literals(uint32_t ip, uint32_t op, uint32_t n)
    {
        for (uint32_t c = 0; c < n; c += L) {
            uint32_t x = ip + c + s0;
            ensure(x, L);
            uint8_t b = iwin[(x + gl) & (IWIN - 1)];
            if (c + gl < n)
                ring[(op + c + gl) & RMASK] = b;
            flush_upto(op + (n - c < L ? n : c + L));
        }
    }

    // n-byte match at distance off, written at output offset op
    __device__ __forceinline__ void copy_match(uint32_t op, uint32_t off, uint32_t n)
    {
        uint32_t c = 0;
        uint32_t eff = off;
        if (off < L) {
            // period-off pattern for the first L bytes, then a distance that
            // is a multiple of off and >= L (never overlaps within a step)
            uint32_t m = gl % off;
            uint8_t b = ring[(op - off + m) & RMASK];
            if (gl < n)
                ring[(op + gl) & RMASK] = b;
            flush_upto(op + (n < L ? n : L));
            c = L;
            eff = off * ((L + off - 1) / off);
        }
        const bool near = (DIAG & 1) ? true : eff <= NEAR;   // DIAG 1: ring only
        for (; c < n; c += L) {
            uint32_t src = op + c - eff + gl;
            uint8_t b = near ? ring[src & RMASK] : obase[src];
            if (c + gl < n)
                ring[(op + c + gl) & RMASK] = b;
            flush_upto(op + (n - c < L ? n : c + L));
        }
    }
};

// XXH32 constants (rare checksum paths)
constexpr uint32_t P1 = 0x9E3779B1u, P2 = 0x85EBCA77u, P3 = 0xC2B2AE3Du, P4 = 0x27D4EB2Fu,
                   P5 = 0x165667B1u;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r)
{
    return (x << r) | (x >> (32 - r));
}

// XXH32 (seed 0) over n bytes; get(i) returns the 4 bytes at i (LE).
template <typename Get>
__device__ uint32_t xxh32(uint32_t n, Get get)
{
    uint32_t acc, i = 0;
    if (n >= 16) {
        uint32_t a0 = P1 + P2, a1 = P2, a2 = 0, a3 = 0u - P1;
        for (; i + 16 <= n; i += 16) {
            a0 = rotl(a0 + get(i) * P2, 13) * P1;
            a1 = rotl(a1 + get(i + 4) * P2, 13) * P1;
            a2 = rotl(a2 + get(i + 8) * P2, 13) * P1;
            a3 = rotl(a3 + get(i + 12) * P2, 13) * P1;
        }
        acc = rotl(a0, 1) + rotl(a1, 7) + rotl(a2, 12) + rotl(a3, 18);
    } else {
        acc = P5;
    }
    acc += n;
    for (; i + 4 <= n; i += 4)
        acc = rotl(acc + get(i) * P3, 17) * P4;
    for (; i < n; i++)
        acc = rotl(acc + (get(i) & 0xFF) * P5, 11) * P1;
    acc ^= acc >> 15;
    acc *= P2;
    acc ^= acc >> 13;
    acc *= P3;
    acc ^= acc >> 16;
    return acc;
}

template <int L, int RING, int WAVES, int CM, int DIAG, bool FAST>
__global__ __launch_bounds__(64 * WAVES) void lz4_frames_kernel(const FrameDesc *__restrict__ desc,
                                                                uint32_t nframes,
                                                                const uint8_t *__restrict__ comp,
                                                                uint8_t *__restrict__ out,
                                                                int32_t *__restrict__ status,
                                                                uint32_t *__restrict__ fail_at)
{
    using G = Group<L, RING, CM, DIAG>;
    constexpr int GPW = 64 / L;                     // frames per wave
    constexpr uint32_t PER = RING + G::IWIN + 32;   // ring, window + guard, dummy
    __shared__ __attribute__((aligned(16))) uint8_t lds[WAVES * GPW * PER];

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t grp = lane / L;
    const uint32_t f = (blockIdx.x * WAVES + wave) * GPW + grp;
    const bool live = f < nframes;

    G g;
    g.gl = lane % L;
    FrameDesc d = live ? desc[f] : FrameDesc{0, 0, 0, 0};
    const uint8_t *cbase = comp + d.c_off;
    g.s0 = (uint32_t)(reinterpret_cast<uintptr_t>(cbase) & 15);
    g.cab = cbase - g.s0;
    g.clen = d.c_size;
    g.climit = (g.s0 + g.clen + 15) & ~15u;
    g.obase = out + d.d_off;
    g.dlen = d.d_size;
    g.oal = (reinterpret_cast<uintptr_t>(g.obase) & 15) == 0;
    uint8_t *base = lds + (wave * GPW + grp) * PER;
    g.ring = base;
    g.iwin = base + RING;
    g.flushed = 0;

    // ---- frame header (LZ4F_decodeHeader order, liblz4 1.9.3) ----------
    int32_t st = ST_OK;
    uint32_t mode = live ? M_BLKHDR : M_DONE;
    uint32_t ip = 0, op = 0, fail_op = 0;
    uint32_t block_ck = 0, indep = 1, content_ck = 0, csize_flag = 0, bsid = 4;
    uint32_t max_block = 65536;
    uint64_t content_size = 0;
    uint32_t iend = 0, oend = 0, floor_ = 0, bstart = 0;
    if (live) {
        g.window_reset(g.s0);
        if (g.clen < 7) {
            st = ST_HDR_INCOMPLETE;
        } else {
            uint32_t magic = g.fetch32(0);
            uint32_t dsc = g.fetch32(4);
            uint32_t flg = dsc & 0xFF, bd = (dsc >> 8) & 0xFF;
            block_ck = (flg >> 4) & 1;
            indep = (flg >> 5) & 1;
            csize_flag = (flg >> 3) & 1;
            content_ck = (flg >> 2) & 1;
            uint32_t dictid = flg & 1;
            uint32_t hdr = 7 + (csize_flag ? 8 : 0) + (dictid ? 4 : 0);
            bsid = (bd >> 4) & 7;
            if ((magic & 0xFFFFFFF0u) == 0x184D2A50u)
                st = ST_SHORT_FRAME;
            else if (magic != kLz4Magic)
                st = ST_FRAME_TYPE;
            else if ((flg >> 1) & 1)
                st = ST_RESERVED;
            else if (((flg >> 6) & 3) != 1)
                st = ST_VERSION;
            else if (g.clen < hdr)
                st = ST_HDR_INCOMPLETE;
            else if ((bd >> 7) & 1)
                st = ST_RESERVED;
            else if (bsid < 4)
                st = ST_MAXBLOCK;
            else if (bd & 15)
                st = ST_RESERVED;
            else {
                uint32_t hc = xxh32(hdr - 5, [&](uint32_t i) { return g.fetch32(4 + i); });
                if (((hc >> 8) & 0xFF) != (g.fetch32(hdr - 1) & 0xFF))
                    st = ST_HDR_CHECKSUM;
            }
            if (st == ST_OK) {
                if (csize_flag)
                    content_size = (uint64_t)g.fetch32(6) | ((uint64_t)g.fetch32(10) << 32);
                max_block = 1u << (8 + 2 * bsid);
                ip = hdr;
            }
        }
        if (st != ST_OK)
            mode = M_DONE;
    }

    // ---- blocks and sequences, all groups in lockstep ---------------------
    while (__builtin_amdgcn_ballot_w64(mode != M_DONE) != 0) {
        if (mode == M_BLKHDR) {
            fail_op = op;
            if (g.clen - ip < 4) {
                st = ST_TRUNCATED;
                mode = M_DONE;
            } else {
                uint32_t bh = g.fetch32(ip);
                ip += 4;
                uint32_t bsize = bh & 0x7FFFFFFFu;
                uint32_t need = bsize + (block_ck ? 4 : 0);
                if (bh == 0) {
                    mode = M_DONE;   // EndMark; suffix below
                } else if (bsize > max_block) {
                    st = ST_MAXBLOCK;
                    mode = M_DONE;
                } else if (g.clen - ip < need) {
                    st = ST_TRUNCATED;
                    mode = M_DONE;
                } else {
                    if (block_ck) {
                        uint32_t h = xxh32(bsize, [&](uint32_t i) { return g.fetch32(ip + i); });
                        if (h != g.fetch32(ip + bsize)) {
                            st = ST_BLOCK_CHECKSUM;
                            mode = M_DONE;
                        }
                    }
                    if (st == ST_OK && (bh & 0x80000000u)) {
                        if (op + bsize > g.dlen) {
                            st = ST_DST_OVERFLOW;
                            mode = M_DONE;
                        } else {
                            g.copy_literals(ip, op, bsize);
                            op += bsize;
                            ip += need;
                        }
                    } else if (st == ST_OK) {
                        iend = ip + bsize;
                        bstart = op;
                        oend = op + max_block;
                        floor_ = indep ? op : 0;
                        mode = M_SEQ;
                    }
                }
            }
        }
        bool slow = mode == M_SEQ;
        if (FAST && mode == M_SEQ) {
            // ---- fast path: the common sequence shape in one step --------
            // (no multi-byte length extensions, literals <= 4L bytes,
            // match <= 8L bytes at a near distance >= 4L, not the block's last
            // sequence, every bound satisfied).  Anything else re-runs the
            // same sequence through the general path below.
            if (ip + g.s0 + 6 * L > g.filled)
                g.refill();   // keep >= 6L bytes of input ahead
            const uint32_t a = g.peek32(ip + g.s0);
            const uint32_t tok = a & 0xFF, lit4 = tok >> 4, mln = tok & 15;
            const uint32_t b1 = (a >> 8) & 0xFF;
            const bool litx = lit4 == 15;
            const uint32_t lit = litx ? 15 + b1 : lit4;
            const uint32_t lsrc = ip + 1 + (litx ? 1 : 0);
            const uint32_t p = lsrc + lit;
            const uint32_t o = g.peek32(p + g.s0);
            const uint32_t off = o & 0xFFFF, b2 = (o >> 16) & 0xFF;
            const bool mlx = mln == 15;
            const uint32_t ml = (mlx ? 15 + b2 : mln) + kMinMatch;
            const uint32_t np = p + 2 + (mlx ? 1 : 0);
            const uint32_t mop = op + lit;
            const uint32_t nop = mop + ml;
            const bool ok = ip + g.s0 + 6 * L <= g.filled && ip + g.s0 >= g.filled - G::IWIN &&
                            (!litx || (b1 != 255 && iend - (ip + 1) > 15)) &&
                            (!mlx || (b2 != 255 && np < iend - (kLastLiterals - 1))) &&
                            lit <= 4 * L && ml <= 8 * L && ip < iend &&
                            op + lit <= oend - kMfLimit && iend - lsrc >= lit + 2 + 1 + kLastLiterals &&
                            off >= 4 * L && off <= G::NEAR && off <= mop - floor_ &&
                            nop <= oend - kLastLiterals && nop <= g.dlen;
            if (ok) {
                if (lit)
                    g.lit_step(lsrc, op, lit, 0);
                g.match_step(mop, off, ml, 0);
                if (ml > 4 * L)
                    g.match_step(mop, off, ml, 4 * L);
                op = nop;
                ip = np;
                g.flush_upto(op);
                slow = false;
            }
        }
        if (slow) {
            // one LZ4 sequence (LZ4_decompress_safe semantics, 1.9.3)
            int32_t e = ST_OK;
            bool last = false;
            if (ip >= iend) {
                e = ST_BLOCK_ERR;
            } else {
                uint32_t t = g.fetch32(ip);
                uint32_t tok = t & 0xFF;
                uint32_t lit = tok >> 4;
                uint32_t p = ip + 1;
                if (lit == 15) {
                    if (iend - p <= 15) {
                        e = ST_BLOCK_ERR;
                    } else {
                        uint32_t s;
                        do {
                            if (p >= iend) {
                                e = ST_BLOCK_ERR;
                                break;
                            }
                            s = g.fetch32(p++) & 0xFF;
                            lit += s;
                        } while (s == 255);
                    }
                }
                if (e == ST_OK) {
                    if (op + lit > oend - kMfLimit || iend - p < lit + 2 + 1 + kLastLiterals) {
                        // last sequence: literals only, exactly to the block end
                        if (iend - p != lit || op + lit > oend)
                            e = ST_BLOCK_ERR;
                        else if (op + lit > g.dlen)
                            e = ST_DST_OVERFLOW;
                        else {
                            g.copy_literals(p, op, lit);
                            op += lit;
                            ip = iend;
                            last = true;
                        }
                    } else if (op + lit > g.dlen) {
                        e = ST_DST_OVERFLOW;
                    } else {
                        if (lit)
                            g.copy_literals(p, op, lit);
                        p += lit;
                        op += lit;
                        uint32_t o = g.fetch32(p);
                        uint32_t off = o & 0xFFFF;
                        p += 2;
                        uint32_t ml = tok & 15;
                        if (ml == 15) {
                            uint32_t s;
                            do {
                                if (p >= iend) {
                                    e = ST_BLOCK_ERR;
                                    break;
                                }
                                s = g.fetch32(p++) & 0xFF;
                                ml += s;
                                if (p >= iend - (kLastLiterals - 1)) {
                                    e = ST_BLOCK_ERR;
                                    break;
                                }
                            } while (s == 255);
                        }
                        ml += kMinMatch;
                        if (e == ST_OK) {
                            if (off == 0 || off > op - floor_ || op + ml > oend - kLastLiterals)
                                e = ST_BLOCK_ERR;
                            else if (op + ml > g.dlen)
                                e = ST_DST_OVERFLOW;
                            else {
                                g.copy_match(op, off, ml);
                                op += ml;
                                ip = p;
                            }
                        }
                    }
                }
            }
            if (e != ST_OK) {
                if (e == ST_BLOCK_ERR) {
                    // liblz4: ERROR_GENERIC when it decodes the block straight
                    // into dst (room >= max block), else decompressionFailed
                    // via its tmp buffer.  Room = rest of the frame (the
                    // reference's cached path); the host re-derives it for
                    // no-cache reads from fail_at + the block size id.
                    bool direct = (g.dlen - bstart) >= max_block;
                    e = (direct ? (ST_GENERIC | ST_DIRECT_FLAG) : ST_DECOMPRESS_FAILED) |
                        ST_BLOCK_FAIL_FLAG | (int32_t)((bsid - 4) << ST_BSID_SHIFT);
                    fail_op = bstart;
                } else {
                    fail_op = op;
                }
                st = e;
                mode = M_DONE;
            } else if (last) {
                ip = iend + (block_ck ? 4 : 0);
                mode = M_BLKHDR;
            }
        }
    }

    // ---- suffix: flush, content size / checksum, dSize match --------------
    if (live) {
        if (st == ST_OK) {
            g.flush_tail(op);
            fail_op = op;
            if (csize_flag && content_size != op)
                st = ST_FRAME_SIZE;
            else if (content_ck) {
                if (g.clen - ip < 4) {
                    st = ST_TRUNCATED;
                } else {
                    __builtin_amdgcn_s_waitcnt(0);
                    const uint8_t *ob = g.obase;
                    const uint32_t n = op;
                    uint32_t h = xxh32(n, [&](uint32_t i) {
                        uint32_t v = 0;
                        for (int b = 0; b < 4; b++)
                            v |= (i + b < n ? (uint32_t)ob[i + b] : 0u) << (8 * b);
                        return v;
                    });
                    if (h != g.fetch32(ip))
                        st = ST_CONTENT_CHECKSUM;
                }
            }
            if (st == ST_OK && op != g.dlen)
                st = ST_SHORT_FRAME;
        }
        if (g.gl == 0) {
            status[f] = st;
            if (fail_at)
                fail_at[f] = fail_op;
        }
    }
}

template <int L, int RING, int WAVES, int CM = 1, int DIAG = 0, bool FAST = true>
int launch_variant(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                   uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream)
{
    constexpr uint32_t per_block = WAVES * (64 / L);
    dim3 grid((nframes + per_block - 1) / per_block);
    hipLaunchKernelGGL((lz4_frames_kernel<L, RING, WAVES, CM, DIAG, FAST>), grid, dim3(64 * WAVES), 0, stream,
                       d_desc, nframes, d_comp, d_out, d_status, d_fail_at);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace

// Tuning hook: explicit (lanes per frame, ring, waves) variants for
// scripts/kbench.py.
int launch_lz4_frames_variant(int variant, const FrameDesc *d_desc, uint32_t nframes,
                              const uint8_t *d_comp, uint8_t *d_out, int32_t *d_status,
                              hipStream_t stream)
{
    if (nframes == 0)
        return 0;
#define ZSK_V(L, R, W, CM, D, F) \
    launch_variant<L, R, W, CM, D, F>(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream)
    switch (variant) {
    case 0: return ZSK_V(16, 4096, 2, 1, 0, true);
    case 1: return ZSK_V(16, 2048, 2, 1, 0, true);
    case 2: return ZSK_V(16, 8192, 1, 1, 0, true);
    case 3: return ZSK_V(16, 2048, 2, 1, 0, false);
    case 4: return ZSK_V(8, 2048, 1, 1, 0, true);
    case 5: return ZSK_V(8, 4096, 1, 1, 0, true);
    case 6: return ZSK_V(32, 4096, 2, 1, 0, true);
    case 7: return ZSK_V(16, 4096, 1, 1, 0, true);
    case 8: return ZSK_V(8, 8192, 1, 1, 0, true);
    // diagnostic builds (wrong output, timing only): 1 = all matches from
    // the ring, 2 = no output stores, 3 = both
    case 10: return ZSK_V(16, 2048, 2, 1, 1, true);
    case 11: return ZSK_V(16, 2048, 2, 1, 2, true);
    case 12: return ZSK_V(16, 2048, 2, 1, 3, true);
    case 20: return launch_lz4_wave(0, d_desc, nframes, d_comp, d_out, d_status, nullptr, stream);
    case 21: return launch_lz4_wave(1, d_desc, nframes, d_comp, d_out, d_status, nullptr, stream);
    case 22: return launch_lz4_wave(2, d_desc, nframes, d_comp, d_out, d_status, nullptr, stream);
    case 50: return launch_lz4_lane(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream);
    case 51: return launch_lz4_lane(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream, 1);
    case 54: return launch_lz4_lane(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream, 4);
    case 53: return launch_lz4_lane(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream, 3);
    case 30: return launch_lz4_frames(d_desc, nframes, d_comp, d_out, d_status, nullptr, stream);
    case 31: return launch_lz4_split_stages(3, 0x800, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 32: return launch_lz4_split_stages(7, 0x1800, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 33: return launch_lz4_split_stages(2, 0x800, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 36: return launch_lz4_split_stages(15, 0xA01, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 35: return launch_lz4_split_stages(15, 0x1800, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 37: return launch_lz4_split_stages(15, 0xA03, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 39: return launch_lz4_split_stages(15, 0x603, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 61: return launch_lz4_split_stages(15, 0, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 62: return launch_lz4_split_stages(7, 0, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 63: return launch_lz4_split_stages(4, 0x205, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 64: return launch_lz4_split_stages(4, 0x206, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 65: return launch_lz4_split_stages(4, 0x207, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 66: return launch_lz4_split_stages(4, 0x204, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 68: return launch_lz4_split_stages(4, 0x208, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 67: return launch_lz4_split_stages(4, 0x203, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 69: return launch_lz4_split_stages(4, 0x209, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 70: return launch_lz4_split_stages(4, 0x20A, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 71: return launch_lz4_split_stages(15, 0x209, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 72: return launch_lz4_split_stages(15, 0x20A, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 73: return launch_lz4_split_stages(15, 0x400, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 74: return launch_lz4_split_stages(2, 0x400, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 75: return launch_lz4_split_stages(15, 0x20B, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 76: return launch_lz4_split_stages(4, 0x20B, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 77: return launch_lz4_split_stages(15, 0x20C, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 79: return launch_lz4_split_stages(15, 0x20D, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 78: return launch_lz4_split_stages(15, 0x204, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 60: return launch_lz4_split_stages(2, 0, d_desc, nframes, d_comp, d_out, d_status, stream);
    // parse A/B: 80/81 = split decoder with the chunk / lane-per-frame (lean)
    // parse for every frame, 82/83 = plan + that parse only
    case 80: return launch_lz4_split_stages(15, 0x4000, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 81: return launch_lz4_split_stages(15, 0x2000, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 82: return launch_lz4_split_stages(3, 0x4000, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 83: return launch_lz4_split_stages(3, 0x2000, d_desc, nframes, d_comp, d_out, d_status, stream);
    // 85/86 = the split decoder / plan + parse with the older lz4_scan_kernel
    // for every frame; 87/88 = plan + lz4_lean_kernel diagnostics (no item
    // stores / every item to slot 0); 89 = split decoder, older scan for the
    // frames the lane-per-frame parse takes by default
    case 85: return launch_lz4_split_stages(15, 0xA20D, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 86: return launch_lz4_split_stages(3, 0xA000, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 87: return launch_lz4_split_stages(3, 0x12000, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 88: return launch_lz4_split_stages(3, 0x22000, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 89: return launch_lz4_split_stages(15, 0x8000, d_desc, nframes, d_comp, d_out, d_status, stream);
    // 84 = execute v13 alone over the items the previous launch left
    // 90 = execute v13 with section timers (wave cycles per section; diagnostic)
    case 90: return launch_lz4_split_stages(4, 0x20E, d_desc, nframes, d_comp, d_out, d_status, stream);
    // 91 = split decoder with execute v15 (= the default), by version number
    case 91: return launch_lz4_split_stages(15, 0x20F, d_desc, nframes, d_comp, d_out, d_status, stream);
    // 93-96 = execute v15 diagnostics alone: no rounds / no round 0 / no flush / no piece loads
    case 93: return launch_lz4_split_stages(4, 0x21B, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 94: return launch_lz4_split_stages(4, 0x21C, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 95: return launch_lz4_split_stages(4, 0x21D, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 96: return launch_lz4_split_stages(4, 0x21E, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 97: return launch_lz4_split_stages(4, 0x20F, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 98: return launch_lz4_split_stages(15, 0x210, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 99: return launch_lz4_split_stages(15, 0x211, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 100: return launch_lz4_split_stages(3, 0x42000, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 105: return launch_lz4_split_stages(3, 0x102000, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 104: return launch_lz4_split_stages(3, 0x82000, d_desc, nframes, d_comp, d_out, d_status, stream);
    // 101 = execute v17 alone with its flush's stage reads but no stores (diagnostic)
    case 101: return launch_lz4_split_stages(4, 0x21F, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 106: return launch_lz4_split_stages(4, 0x211, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 84: return launch_lz4_split_stages(4, 0x20D, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 38: return launch_lz4_split_stages(7, 0xA03, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 34: return launch_lz4_split_stages(15, 0xA00, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 40: return launch_lz4_split_stages(7, 0x1801, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 41: return launch_lz4_split_stages(7, 0x1802, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 44: return launch_lz4_split_stages(7, 0x1810, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 45: return launch_lz4_split_stages(7, 0x1906, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 46: return launch_lz4_split_stages(7, 0x1908, d_desc, nframes, d_comp, d_out, d_status, stream);
    case 43: return launch_lz4_split_stages(7, 0x1808, d_desc, nframes, d_comp, d_out, d_status, stream);
    default: return -1;
    }
#undef ZSK_V
}

}   // namespace zsk
