// lz4_chunk.hip — parse phase of the two-phase LZ4 decoder, one WAVE per
// frame, the LZ4 token chain split over the wave's 64 lanes (gfx950).
//
// The lane-per-frame parse (lz4_scan.hip) walks each frame's ~1,500-token
// chain serially: 65,536 frames = one wave per SIMD, every step a dependent
// LDS round trip.  Here a frame's compressed block is cut into 64 chunks and
// every lane parses one, so a frame's chain takes ~25 steps instead of
// ~1,500 and there are as many waves as frames to hide the latency.
//
// A chunk's true first token is unknown until the chunk before it is parsed,
// so each block goes through three passes over the same bytes:
//
//   1. speculate: lane j parses from its chunk start s_j as if a token began
//      there, until it passes its chunk end, marking every token position it
//      visits in a per-lane bitmap (LDS, the chunk's first kMap bytes).  An LZ4
//      token chain started at a wrong byte joins the true chain after a few
//      tokens (it lands on a true token start), and from there on the two are
//      the same chain.
//   2. join: lane j continues its own chain past its exit e_j until it lands
//      on a position another lane visited (bit set) — y_j — or on the block
//      end.  If lane j's chain is the true one, y_j is a true token and the
//      lane whose chunk holds y_j (its owner) is true from y_j on.  Walking
//      owners from lane 0 (whose start is the block start) gives every lane's
//      true range [entry_j, y_j): usually lane j+1 starts where lane j stops.
//   3. count, then emit: each true lane re-parses its range counting output
//      bytes and items; wave prefix sums give its absolute output position and
//      item slot; a last pass parses the range again with every liblz4 rule
//      (same checks, same order as lz4_scan.hip's slow step and
//      oracle/lz4_oracle.c decode_block) and writes the items.
//
// Passes 1-2 never validate: a speculative chain is arbitrary bytes.  They
// follow liblz4's token/offset/length-extension transitions with the
// input-side end rule only (a literal run reaching within 8 bytes of the block
// end ends the block), which makes the same moves as liblz4 on every sequence
// liblz4 accepts; where the two could differ, pass 3 reports the error liblz4
// reports.  Correctness never depends on the speculation succeeding: a chain
// that does not join just makes its left neighbour parse further.
//
// One-frame route (ONE, batches of <= 64 frames): one frame per workgroup,
// staged whole in LDS, and pass 1 records each lane's first tokens with the
// counts before them so the count pass is skipped (below).  Its frames of
// more than 64 KiB: each 64 KiB block a workgroup of lz4_job_parse_kernel
// (below), accepted or re-parsed by the one-frame kernel.
//
// Output: the items of lz4_scan.hip (8 bytes per sequence, two when a run is
// longer than the small form holds) at rec_base[f], without the padding item
// the older execute kernels needed (seq_exec.hip keeps an extended pair
// together itself), nitems[f], status[f], fail_at[f].
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lz4_dev.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4d;

constexpr uint32_t kItemExt = 0x80000000u;
constexpr uint32_t kItemPos = 0x3FFFFFFFu;
constexpr uint32_t kCW = 4;                 // waves (frames) per workgroup
constexpr uint32_t kMap = 512;              // token-map bits per lane (chunk prefix)
constexpr uint32_t kMapW = kMap / 32;       // dwords per lane
constexpr uint32_t kMinChunk = 256;         // shortest chunk worth a lane
constexpr uint32_t kNone = 0xFFFFFFFFu;

// The frame's compressed bytes through a 64-byte per-lane window in LDS:
// frame offset x is resource byte x + s0; the window holds resource bytes
// [base, base + 64), base 16-aligned, refilled with four 16-byte loads issued
// together (a sequence spans ~21 bytes on the synthetic, so a refill serves
// about three; the 16-byte register window it replaces reloaded, and waited,
// about twice per sequence).  Loads past the span read 0 (dword range checks).
struct Src {
    __amdgpu_buffer_rsrc_t r;
    uint32_t s0;
    bool staged;     // one-frame route: the frame is staged whole in LDS at `lds`
    uint32_t lds;
};

struct Win {
    uint32_t lds;    // this lane's window (64 bytes of LDS)
    uint32_t base;
};

template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T *lp(uint32_t a)
{
    return (__attribute__((address_space(3))) T *)(uintptr_t)a;
}

// KS 1: the frame is known to be staged (the one-frame route's parse
// instantiates the block parse both ways, so its hot loops carry no test)
template <int KS = 0>
__device__ __forceinline__ uint32_t rd4(const Src &S, Win &W, uint32_t x)
{
    if (KS == 1 || S.staged) {   // (wave-uniform) the frame staged whole: one LDS round trip
        const uint32_t a = S.lds + (x & ~3u);
        return __builtin_amdgcn_alignbyte(*lp<uint32_t>(a + 4), *lp<uint32_t>(a), x & 3);
    }
    const uint32_t rx = x + S.s0;
    if (rx - W.base > 59u) {
        W.base = rx & ~15u;
        u32x4 v[4];
#pragma unroll
        for (int i = 0; i < 4; i++)
            v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(S.r, W.base + 16 * i, 0, 0));
#pragma unroll
        for (int i = 0; i < 4; i++)
            *lp<u32x4>(W.lds + 16 * i) = v[i];
    }
    const uint32_t o = rx - W.base, a = W.lds + (o & ~3u);
    return __builtin_amdgcn_alignbyte(*lp<uint32_t>(a + 4), *lp<uint32_t>(a), o & 3);
}

template <int KS = 0>
__device__ __forceinline__ uint32_t rd1(const Src &S, Win &W, uint32_t x)
{
    return rd4<KS>(S, W, x) & 0xFF;
}

// One sequence of a chain, no validation (passes 1, 2 and the count).
// Advances p to the next token (the block end after a literals-only last
// sequence or when the bytes cannot be a sequence) and adds the sequence's
// output bytes and items.
// (t4: the four bytes at p, read by the caller)
template <int KS = 0>
__device__ __forceinline__ void skel_at(const Src &S, Win &W, uint32_t &p, uint32_t iend, uint32_t &out,
                                        uint32_t &nitem, uint32_t t4)
{
    const uint32_t tok = t4 & 0xFF;
    uint32_t lit = tok >> 4, pp = p + 1;
    if (lit == 15) {
        uint32_t e = (t4 >> 8) & 0xFF;
        pp++;
        lit += e;
        while (e == 255 && pp < iend) {
            e = rd1<KS>(S, W, pp);
            pp++;
            lit += e;
        }
    }
    // liblz4's input-side end rule (ip + lit > iend - (2 + 1 + LASTLITERALS)):
    // a literals-only last sequence (no early exit: one join for the wave)
    const bool endr = pp >= iend || iend - pp < lit + 8;
    uint32_t q = pp + lit;
    uint32_t ml = tok & 15;
    if (!endr && ml == 15) {
        uint32_t e = (rd4<KS>(S, W, q) >> 16) & 0xFF;
        q += 3;
        ml += e;
        while (e == 255 && q < iend) {
            e = rd1<KS>(S, W, q);
            q++;
            ml += e;
        }
    } else {
        q += 2;
    }
    ml = endr ? 0 : ml + kMinMatch;
    out += lit + ml;
    nitem += (lit > 255 || ml > 258) ? 2 : 1;
    p = endr || q >= iend ? iend : q;
}

template <int KS = 0>
__device__ __forceinline__ void skel(const Src &S, Win &W, uint32_t &p, uint32_t iend, uint32_t &out,
                                     uint32_t &nitem)
{
    skel_at<KS>(S, W, p, iend, out, nitem, rd4<KS>(S, W, p));
}

struct Blk {
    uint32_t ib, iend;     // compressed block [ib, iend) (frame offsets)
    uint32_t bop, oend;    // output position of the block, + max block size
    uint32_t floor_;       // lowest match source (block start if independent)
    uint32_t dlen;
};

// the frame's status for a failure inside block B (lz4_scan.hip fail_block)
__device__ __forceinline__ int32_t block_fail(const Blk &B, uint32_t bsid, uint32_t max_block)
{
    const bool direct = (B.dlen - B.bop) >= max_block;
    const int32_t bits = (int32_t)((bsid - 4) << ST_BSID_SHIFT);
    return (direct ? (ST_GENERIC | ST_DIRECT_FLAG) : ST_DECOMPRESS_FAILED) | ST_BLOCK_FAIL_FLAG | bits;
}

__device__ __forceinline__ void put_item(uint64_t *it, uint32_t &k, uint32_t lsrc, uint32_t lit,
                                         uint32_t off, uint32_t ml)
{
    // one store always, the extended pair's second only when needed (no
    // two-way branch in the emit loop)
    const bool ext = lit > 255 || ml > 258;
    it[k] = ext ? (((uint64_t)off << 32) | (lsrc | kItemExt))
                : (((uint64_t)(off | (lit << 16) | ((ml ? ml - 3 : 0) << 24)) << 32) | lsrc);
    if (ext)
        it[k + 1] = ((uint64_t)ml << 32) | lit;
    k += ext ? 2 : 1;
}

// Pass 3: the validated parse of a true range [p, y) from output position op,
// items from slot k.  Returns -1, or the status of the first failing rule
// (ST_BLOCK_ERR for a block failure, ST_DST_OVERFLOW), in liblz4's order.
// A sequence's rules fold into one status and one exit from the loop (fewer
// divergent exits for the wave to track).
template <int KS = 0>
__device__ __forceinline__ int32_t emit_range(const Src &S, Win &W, const Blk &B, uint32_t p,
                                              uint32_t y, uint32_t op, uint64_t *it, uint32_t k)
{
    const uint32_t iend = B.iend;
    int32_t st = -1;
    while (p < y) {
        const uint32_t t4 = rd4<KS>(S, W, p);
        const uint32_t tok = t4 & 0xFF;
        p++;
        uint32_t lit = tok >> 4;
        if (lit == 15) {
            if (iend - p <= 15) {
                st = ST_BLOCK_ERR;
                break;
            }
            uint32_t e = (t4 >> 8) & 0xFF;
            p++;
            lit += e;
            while (e == 255 && p < iend) {
                e = rd1<KS>(S, W, p);
                p++;
                lit += e;
            }
            if (e == 255) {   // the length bytes run past the block
                st = ST_BLOCK_ERR;
                break;
            }
        }
        if (op + lit > B.oend - kMfLimit || iend - p < lit + 2 + 1 + kLastLiterals) {
            // the block's last sequence: literals only, ending the block
            st = (iend - p != lit || op + lit > B.oend) ? ST_BLOCK_ERR : op + lit > B.dlen ? ST_DST_OVERFLOW : -1;
            if (st < 0)
                put_item(it, k, p, lit, 0, 0);
            break;
        }
        const uint32_t lsrc = p;
        const uint32_t mb = op + lit;
        p += lit;
        const uint32_t o4 = rd4<KS>(S, W, p);
        const uint32_t off = o4 & 0xFFFF;
        p += 2;
        uint32_t ml = tok & 15;
        bool bad = false;
        if (ml == 15) {
            uint32_t e = (o4 >> 16) & 0xFF;
            for (bool first = true;; first = false) {
                if (p >= iend) {
                    bad = true;
                    break;
                }
                if (!first)
                    e = rd1<KS>(S, W, p);
                p++;
                ml += e;
                if (p >= iend - (kLastLiterals - 1)) {
                    bad = true;
                    break;
                }
                if (e != 255)
                    break;
            }
        }
        ml += kMinMatch;
        // the literals' output room first (checked before the offset is
        // read), then the match length bytes, the offset, the match's room
        st = mb > B.dlen                        ? ST_DST_OVERFLOW
             : bad                              ? ST_BLOCK_ERR
             : off > mb - B.floor_              ? ST_BLOCK_ERR
             : off == 0                         ? ST_NOT_RUN   // liblz4 writes zeros: the wave kernel decodes the frame
             : mb + ml > B.oend - kLastLiterals ? ST_BLOCK_ERR
             : mb + ml > B.dlen                 ? ST_DST_OVERFLOW
                                                : -1;
        if (st >= 0)
            break;
        put_item(it, k, lsrc, lit, off, ml);
        op = mb + ml;
    }
    return st;
}

// One-frame route: pass 1 records, for each of a lane's first kRec visited
// tokens, (position in the chunk, output bytes and items counted before it);
// a true range always starts at a position its lane visited (the chunk start,
// or where the lane before stopped on this lane's mark), so its count is the
// lane's total through pass 2 minus the record at its entry -- no count pass
// (a lane whose entry is past its records counts as before).
constexpr uint32_t kRec = 64;
// The one-frame route parses over all OW waves of its workgroup: lane j of
// 64 OW takes chunk j (at least 32 KiB / (64 OW) bytes), 8192 / (64 OW)
// records each (OW 4: 128-byte chunks, 32 records; OW 8: 64 and 16)
template <uint32_t OW>
constexpr uint32_t one_min_chunk() { return 32768 / (64 * OW); }
template <uint32_t OW>
constexpr uint32_t one_rec() { return 8192 / (64 * OW); }
constexpr uint32_t kOneMapW = 4;   // map dwords per lane: a 128-bit chunk prefix

#ifdef ZSK_TUNING
// tuning builds: the one-frame route's phase cycles ([0] staging, [1]
// header, [2] pass 1, [3] pass 2 + owners, [4] count, [5] emit, [6] rest) and
// per-block wave-max iteration counts ([8] pass 1, [9] pass 2, [10] emit),
// [12] blocks; printed by launch_lz4_chunk under ZSEEK_CHUNK_TIMERS
__device__ unsigned long long g_ctime[16];
#define ZSK_CT(i)                                                             \
    if (ONE) {                                                                \
        const uint64_t tn_ = __builtin_readcyclecounter();                    \
        if (lane == 0)                                                        \
            atomicAdd(&g_ctime[i], (unsigned long long)(tn_ - tmark_));       \
        tmark_ = tn_;                                                         \
    }
#define ZSK_CN(i, v)                                                          \
    if (ONE) {                                                                \
        const uint32_t m_ = wave_incl_max(v);                                 \
        if (lane == 63)                                                       \
            atomicAdd(&g_ctime[i], (unsigned long long)m_);                   \
    }
#else
#define ZSK_CT(i)
#define ZSK_CN(i, v)
#endif

// One compressed block over the wave.  Returns -1 (block done: *op and *k
// advanced) or a frame status.
// ONE: the workgroup's kOneLanes lanes (lane = thread index) take the block,
// the wave-wide steps (owners, scans, the first failure) going through LDS
// scratch at `coll` (3 x 256 + 16 words) with workgroup barriers.
template <bool ONE, int KS = 0, uint32_t OW = 4>
__device__ int32_t chunk_block(const Src &S, Win &W, const Blk &B, uint32_t lane, uint32_t mapbase,
                               uint64_t *it, uint32_t &k, uint32_t cap, uint32_t &op, uint32_t recbase,
                               uint32_t coll, uint32_t lead)
{
    constexpr uint32_t NL = ONE ? 64 * OW : 64;
    constexpr uint32_t kR = ONE ? one_rec<OW>() : kRec;
    constexpr int LG = ONE ? (OW == 8 ? 9 : 8) : 6;   // log2 NL
    const uint32_t bsize = B.iend - B.ib;
    // chunking: C bytes per lane (>= the minimum chunk), nl lanes
    uint32_t C = (bsize + NL - 1) / NL;
    C = C < (ONE ? one_min_chunk<OW>() : kMinChunk) ? (ONE ? one_min_chunk<OW>() : kMinChunk) : (C + 3) & ~3u;
    const uint32_t nl = (bsize + C - 1) / C;
    // LDS scratch of the ONE route's workgroup steps
    auto cw = [&](uint32_t i) { return lp<uint32_t>(coll + 4 * i); };   // word i
    constexpr uint32_t cY = 0, cN = NL, cE = 2 * NL, cWS = 3 * NL, cM = cWS + 8, cBad = cM + 1, cFirst = cM + 2;
    auto sync = [&]() {
        if constexpr (ONE)
            __syncthreads();
        else
            wave_lds_sync();
    };
    // inclusive sum over the NL lanes, and the total
    auto scan = [&](uint32_t v, uint32_t &total) -> uint32_t {
        const uint32_t inc = wave_incl_add(v);
        if constexpr (!ONE) {
            total = lane_val(inc, 63);
            return inc;
        } else {
            if ((lane & 63) == 63)
                *cw(cWS + (lane >> 6)) = inc;
            __syncthreads();
            uint32_t before = 0, tot = 0;
            for (uint32_t q = 0; q < NL / 64; q++) {
                const uint32_t x = *cw(cWS + q);
                before += q < (lane >> 6) ? x : 0;
                tot += x;
            }
            __syncthreads();
            total = tot;
            return before + inc;
        }
    };
    const uint32_t s = B.ib + lane * C;
    const uint32_t t = s + C < B.iend ? s + C : B.iend;
    const bool act = lane < nl;
    constexpr uint32_t MW = ONE ? kOneMapW : kMapW;   // map dwords per lane
    const uint32_t mlen = C < 32 * MW ? C : 32 * MW;
    const uint32_t mymap = mapbase + lane * (MW * 4);

    uint32_t entry = kNone, y = B.iend;
    uint32_t tout = 0, tnit = 0, nrec = 0;   // ONE: counts from s through pass 2, records
    const uint32_t myrec = recbase + lane * (kR * 8);
#ifdef ZSK_TUNING
    uint64_t tmark_ = __builtin_readcyclecounter();
    uint32_t n1_ = 0, n2_ = 0;
#endif
    if (nl == 1) {
        entry = lane == 0 ? B.ib : kNone;
    } else {
        // pass 1: speculate over the own chunk, marking visited tokens
#pragma unroll
        for (uint32_t i = 0; i < MW; i += 4)
            *lp<u32x4>(mymap + 4 * i) = (u32x4){0, 0, 0, 0};
        sync();
        // (ONE) pass 1 starts `lead` bytes before the chunk, so its chain has
        // usually met the true one when it enters the chunk and pass 2's join
        // after the chunk is short; the lead-in marks and records nothing
        uint32_t p = (ONE && lane > 0) ? (s - B.ib > lead ? s - lead : B.ib) : s;
        if (act) {
            while (p < t) {
                const uint32_t r = p - s;
                const bool in = r < mlen;
                // (no branches: outside the map an OR of 0 into its first
                // word; every position stored, counted only inside the chunk
                // -- a lead-in position's record sits in slot 0 until the
                // chunk's first overwrites it -- the slot saturating at the
                // last, a later record, a consistent pair in ascending
                // order, overwriting it)
                __hip_atomic_fetch_or(lp<uint32_t>(mymap + 4 * (in ? r >> 5 : 0u)), in ? 1u << (r & 31) : 0u,
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                if (ONE) {
                    *lp<uint64_t>(myrec + 8 * (nrec < kR ? nrec : kR - 1)) =
                        ((uint64_t)tout << 32) | (tnit << 16) | (r & 0xFFFF);
                    nrec += r < C && nrec < kR ? 1u : 0u;
                }
                skel<KS>(S, W, p, B.iend, tout, tnit);
#ifdef ZSK_TUNING
                n1_++;
#endif
            }
        }
        sync();
        ZSK_CT(2)
        // pass 2: continue to the first position another lane visited (the
        // chunk by a reciprocal multiply, not a division; the map word and
        // the token read together, one round trip)
        // (ceil(2^32 / C) for C >= 2, in 32 bits: a 64-bit quotient made
        // the loop's multiply a 64-bit one)
        const uint32_t mC = 0xFFFFFFFFu / C + 1u;
        if (act) {
            while (p < B.iend) {
                const uint32_t x = p - B.ib;
                uint32_t c = __umulhi(x, mC);
                c -= c * C > x ? 1u : 0u;
                const uint32_t r = x - c * C;
                const uint32_t mw = *lp<uint32_t>(mapbase + c * (MW * 4) + 4 * ((r < mlen ? r : 0u) >> 5));
                const uint32_t t4 = rd4<KS>(S, W, p);
                if (r < mlen && ((mw >> (r & 31)) & 1))
                    break;
                skel_at<KS>(S, W, p, B.iend, tout, tnit, t4);
#ifdef ZSK_TUNING
                n2_++;
#endif
            }
        }
        y = p;
#ifdef ZSK_TUNING
        if (ONE)
            __syncthreads();
        ZSK_CT(11)
#endif
        // owners: lane j's successor is the lane whose chunk holds y_j
        const uint32_t nxt = act ? (y >= B.iend ? NL : (y - B.ib) / C) : NL;
        if constexpr (!ONE) {
            const uint64_t ends = __ballot(act && nxt == 64);
            const uint32_t m = (uint32_t)__builtin_ctzll(ends | (1ull << 63));   // first lane ending the block
            const uint64_t bad = __ballot(lane < m && nxt != lane + 1);
            if (bad == 0 && (ends >> m) & 1) {
                // the usual case: lanes 0..m, each starting where the previous stops
                const uint32_t yp = dpp_prev(y, B.ib);
                entry = lane <= m ? (lane == 0 ? B.ib : yp) : kNone;
            } else {
                // follow the owner chain from lane 0
                uint32_t j = 0, x = B.ib;
                for (;;) {
                    if (lane == j)
                        entry = x;
                    const uint32_t yj = lane_val(y, (int)j);
                    const uint32_t nj = lane_val(nxt, (int)j);
                    if (nj >= 64)
                        break;
                    x = yj;
                    j = nj;
                }
            }
        } else {
            // the same over the workgroup: y and successors in LDS, the first
            // lane ending the block by atomicMin, any break in 0..m by atomicOr
            *cw(cY + lane) = y;
            *cw(cN + lane) = nxt;
            *cw(cE + lane) = kNone;
            if (lane == 0) {
                *cw(cM) = NL;
                *cw(cBad) = 0;
            }
            __syncthreads();
            if (act && nxt == NL)
                __hip_atomic_fetch_min(cw(cM), lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __syncthreads();
            const uint32_t m = *cw(cM);
            if (lane < m && nxt != lane + 1)
                __hip_atomic_fetch_or(cw(cBad), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __syncthreads();
            if (*cw(cBad) == 0 && m < NL) {
                entry = lane <= m ? (lane == 0 ? B.ib : *cw(cY + lane - 1)) : kNone;
            } else {
#ifdef ZSK_TUNING
                if (lane == 0)
                    atomicAdd(&g_ctime[13], 1ull);
#endif
                // the owner chain from lane 0 by pointer jumping (successors
                // only increase): J_r = 2^r successor steps; a lane on the
                // chain at distance d marks the lane at d + 2^r, top bit
                // first, so every distance is reached; then each chain lane
                // gives its successor the entry it stopped at
                uint32_t J[LG];
                J[0] = nxt;
                for (int r = 1; r < LG; r++) {
                    *cw(cE + lane) = J[r - 1];
                    __syncthreads();
                    J[r] = J[r - 1] < NL ? *cw(cE + J[r - 1]) : NL;
                    __syncthreads();
                }
                *cw(cE + lane) = lane == 0 ? 1u : 0u;   // on the chain
                __syncthreads();
                for (int r = LG - 1; r >= 0; r--) {
                    const bool on = *cw(cE + lane) != 0;
                    __syncthreads();
                    if (on && J[r] < NL)
                        *cw(cE + J[r]) = 1u;
                    __syncthreads();
                }
                const bool on = *cw(cE + lane) != 0;
                __syncthreads();
                *cw(cE + lane) = lane == 0 ? B.ib : kNone;
                __syncthreads();
                if (on && nxt < NL)
                    *cw(cE + nxt) = y;
                __syncthreads();
                entry = *cw(cE + lane);
            }
            __syncthreads();
        }
    }
    ZSK_CT(3)
    const bool tru = entry != kNone;
    // count: output bytes and items of the true range
    uint32_t out = 0, nit = 0;
    bool counted = false;
    if (ONE && tru && nl > 1) {
        // the record at entry: positions ascend, binary search
        const uint32_t re = entry - s;
        uint32_t lo = 0, hi = nrec;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint32_t)(*lp<uint64_t>(myrec + 8 * mid) & 0xFFFF) < re)
                lo = mid + 1;
            else
                hi = mid;
        }
        if (lo < nrec) {
            const uint64_t e = *lp<uint64_t>(myrec + 8 * lo);
            if ((uint32_t)(e & 0xFFFF) == re) {
                out = tout - (uint32_t)(e >> 32);
                nit = tnit - (uint32_t)((e >> 16) & 0xFFFF);
                counted = true;
            }
        }
    }
    if (tru && !counted) {
        uint32_t p = entry;
        while (p < y)
            skel<KS>(S, W, p, B.iend, out, nit);
    }
    ZSK_CT(4)
    uint32_t otot, ktot;
    const uint32_t oinc = scan(out, otot), kinc = scan(nit, ktot);
    if (k + ktot > cap)
        return ST_NOT_RUN;
    // emit: the validated parse, items in place
    int32_t st = -1;
    if (tru)
        st = emit_range<KS>(S, W, B, entry, y, op + oinc - out, it, k + kinc - nit);
#ifdef ZSK_TUNING
    ZSK_CT(5)
    ZSK_CN(8, n1_)
    ZSK_CN(9, n2_)
    if (ONE && lane == 0)
        atomicAdd(&g_ctime[12], 1ull);
    if constexpr (ONE) {   // the workgroup-max iterations of passes 1 and 2
        __shared__ uint32_t wmax_[2];
        if (lane == 0)
            wmax_[0] = wmax_[1] = 0;
        __syncthreads();
        atomicMax(&wmax_[0], n1_);
        atomicMax(&wmax_[1], n2_);
        __syncthreads();
        if (lane == 0) {
            atomicAdd(&g_ctime[14], (unsigned long long)wmax_[0]);
            atomicAdd(&g_ctime[15], (unsigned long long)wmax_[1]);
        }
    }
#endif
    if constexpr (!ONE) {
        const uint64_t fails = __ballot(st >= 0);
        if (fails) {
            const int32_t fs = (int32_t)lane_val((uint32_t)st, __builtin_ctzll(fails));
            return fs;
        }
    } else {
        // the first failing lane's status (lane order = block order)
        if (lane == 0)
            *cw(cFirst) = NL;
        *cw(cE + lane) = (uint32_t)st;
        __syncthreads();
        if (st >= 0)
            __hip_atomic_fetch_min(cw(cFirst), lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __syncthreads();
        const uint32_t first = *cw(cFirst);
        const int32_t fs = first < NL ? (int32_t)*cw(cE + first) : -1;
        __syncthreads();
        if (first < NL)
            return fs;
    }
    op += otot;
    k += ktot;
    return -1;
}

__device__ __forceinline__ uint32_t hdr_xxh32(const Src &S, Win &W, uint32_t n)
{
    // XXH32(frame descriptor bytes [4, 4 + n), seed 0), n < 16
    uint32_t acc = 0x165667B1u + n;
    uint32_t i = 0;
    for (; i + 4 <= n; i += 4) {
        acc += rd4(S, W, 4 + i) * 0xC2B2AE3Du;
        acc = ((acc << 17) | (acc >> 15)) * 0x27D4EB2Fu;
    }
    for (; i < n; i++) {
        acc += rd1(S, W, 4 + i) * 0x165667B1u;
        acc = ((acc << 11) | (acc >> 21)) * 0x9E3779B1u;
    }
    acc ^= acc >> 15;
    acc *= 0x85EBCA77u;
    acc ^= acc >> 13;
    acc *= 0xC2B2AE3Du;
    acc ^= acc >> 16;
    return acc;
}

// ONE (the one-frame route, small batches: DESIGN.md §3): one frame per
// workgroup; its kOneWaves waves stage the compressed frame in LDS (the same
// bytes the window reads, zeros past the resource), then wave 0 parses it
// with every read an LDS round trip instead of an HBM / L2 one.  A frame too
// big for the stage is parsed through the window as usual.
constexpr uint32_t kOneStage = 65536 + 1024;   // bytes: frames of <= kOneStage - 64 compressed
constexpr uint32_t kWinQ = 4;                  // window: 16-byte pieces per lane

// frame f's first item slot when the batch's frames lie in order (the plan's
// direct layout)
__device__ __forceinline__ uint64_t solo_slots(const FrameDesc *__restrict__ desc, uint32_t f)
{
    return (((desc[f].c_off - desc[0].c_off) >> 3) + 40ull * f + 3) & ~3ull;
}

template <bool ONE, uint32_t OW = 4>
__global__ __launch_bounds__(64 * (ONE ? OW : kCW)) void lz4_chunk_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    const uint64_t *__restrict__ rec_base, uint64_t capacity, uint64_t *__restrict__ items,
    uint32_t *__restrict__ nitems, int32_t *__restrict__ status, uint32_t *__restrict__ fail_at,
    uint32_t min_csize, uint32_t *__restrict__ bfirst, const uint32_t *__restrict__ bcount,
    const BlockJob *__restrict__ jobs, const BlockRes *__restrict__ jres, const uint32_t *__restrict__ njobs,
    uint32_t min_jobs, uint64_t *__restrict__ solo_total, uint32_t per_wave, uint32_t lead)
{
    constexpr uint32_t kOneWaves = OW;
    constexpr uint32_t kOneLanes = 64 * OW;
    // (ONE: the staged frame and the window share LDS -- a frame reads one
    // or the other)
    constexpr uint32_t nsw = ONE ? (kOneStage / 16 > kOneLanes * kWinQ ? kOneStage / 16 : kOneLanes * kWinQ)
                                 : kCW * 64 * kWinQ;
    __shared__ __attribute__((aligned(16))) uint32_t maps[ONE ? kOneLanes * kOneMapW : kCW * 64 * kMapW];
    __shared__ __attribute__((aligned(16))) u32x4 stw[nsw];
    __shared__ __attribute__((aligned(16))) uint64_t recs[ONE ? kOneLanes * one_rec<OW>() : 1];
    __shared__ uint32_t coll[ONE ? 3 * kOneLanes + 16 : 1];
    u32x4 *const stage = stw, *const wins = stw;
    const uint32_t lane = ONE ? threadIdx.x : threadIdx.x & 63;   // ONE: the workgroup's lanes
    const uint32_t w = ONE ? 0 : threadIdx.x >> 6;
    // one frame (wave-uniform f); a return ends that frame
    auto frame = [&](const uint32_t f) {
    const FrameDesc d = desc[f];
#ifdef ZSK_TUNING
    uint64_t tmark_ = __builtin_readcyclecounter();
    const uint64_t tstart_ = tmark_;
#endif
    bool staged = false;
    if constexpr (ONE) {
        staged = d.c_size + 64 <= kOneStage && d.c_size >= min_csize;
        if (staged) {
            const Span sp = make_span(comp + d.c_off, d.c_size);
            const uint32_t np = (d.c_size + 64) / 16;
            for (uint32_t i0 = 0; i0 < np; i0 += 4 * 64 * kOneWaves) {
                u32x4 v[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t i = i0 + 64 * kOneWaves * j + threadIdx.x;
                    v[j] = load16u(sp.r, i < np ? sp.s0 + 16 * i : 0x80000000u);
                }
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t i = i0 + 64 * kOneWaves * j + threadIdx.x;
                    if (i < np)
                        stage[i] = v[j];
                }
            }
        }
        __syncthreads();
        // a batch whose frames the caller laid out in order launches no plan
        // kernel (solo_total != null): each workgroup writes its frame's slot
        // offset by the plan's in-order formula (lz4_plan_direct_kernel), the
        // last frame's the total the plan would report; status and fail_at
        // are written below whatever happens
        if (solo_total && lane == 0) {
            const uint64_t r = solo_slots(desc, f);
            const_cast<uint64_t *>(rec_base)[f] = r;
            if (f + 1 == n)
                *solo_total = r + slots_of(d.c_size);
        }
        ZSK_CT(0)
    }
    if (uni(d.c_size) < min_csize)
        return;   // lz4_scan_kernel's frame
    if (bfirst) {
        // block route: the frame's jobs (lane j: job j) are its parse when
        // every one reached its next header with every rule met, each block
        // but the last decoding to exactly the maximum block size (so the
        // speculative offsets were the real ones) and the last ending at
        // dSize; otherwise this kernel parses the frame and the execute reads
        // its items from rec_base (the job list is dropped)
        const uint32_t j0 = uni(bfirst[f]);
        if (j0 != kNoJob) {
            // (ONE: wave 0 decides, the workgroup follows -- a re-parse needs
            // every wave)
            bool take = false;
            if (!ONE || threadIdx.x < 64) {
                const uint32_t l64 = threadIdx.x & 63;
                const uint32_t nb = uni(bcount[f]);
                bool bad = uni(*njobs) < min_jobs || nb == 0 || nb > 64;
                uint32_t k = 0;
                if (!bad && l64 < nb) {
                    const BlockJob J = jobs[j0 + l64];
                    const BlockRes R = jres[j0 + l64];
                    const uint32_t mb = 1u << (8 + 2 * (J.info & 0xFF));
                    const uint32_t end = l64 + 1 == nb ? d.d_size : J.bop + mb;
                    k = R.n;
                    bad = J.f != f || R.st != ST_OK || R.op != end || R.n == 0;
                }
                take = __ballot(bad) == 0;
                const uint32_t total = wave_incl_add(k);
                if (l64 == 63) {
                    if (take) {
                        status[f] = ST_OK;
                        nitems[f] = total;
                        if (fail_at)
                            fail_at[f] = 0;
                    } else if (!ONE) {
                        bfirst[f] = kNoJob;
                    }
                }
            }
            if constexpr (ONE) {
                // (the job list dropped only once every wave has read it: a
                // wave reading kNoJob would skip these barriers)
                if (threadIdx.x == 0)
                    coll[3 * kOneLanes + 15] = take ? 1u : 0u;
                __syncthreads();
                take = coll[3 * kOneLanes + 15] != 0;
                __syncthreads();
                if (!take && threadIdx.x == 0)
                    bfirst[f] = kNoJob;
            }
            if (take)
                return;
        }
    }
    const uint64_t rb0 = (ONE && solo_total) ? solo_slots(desc, f) : rec_base[f];
    const uint32_t cap = slots_of(d.c_size);
    const uint32_t clen = d.c_size, dlen = d.d_size;
    const uint32_t mapbase = (uint32_t)(uintptr_t)(maps) + w * (64 * kMapW * 4);
    uint64_t *it = items + rb0;
    Src S;
    {
        const Span sp = make_span(comp + d.c_off, clen);
        S.r = sp.r;
        S.s0 = sp.s0;
        S.staged = staged;
        S.lds = (uint32_t)(uintptr_t)stage;
    }
    Win W;
    W.base = 0x80000000u;   // no resource byte is within 59 of it: the first read refills
    W.lds = (uint32_t)(uintptr_t)(wins) + 64 * threadIdx.x;
    uint32_t op = 0, k = 0, fail_op = 0;
    int32_t st = ST_OK;
    do {
        if (rb0 + cap > capacity || clen > kItemPos) {
            st = ST_NOT_RUN;
            break;
        }
        // frame header (LZ4F_decodeHeader order; lz4_scan.hip hdr_status)
        if (clen < 7) {
            st = ST_HDR_INCOMPLETE;
            break;
        }
        const uint32_t magic = rd4(S, W, 0);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            st = ST_SHORT_FRAME;
            break;
        }
        if (magic != kLz4Magic) {
            st = ST_FRAME_TYPE;
            break;
        }
        const uint32_t fb = rd4(S, W, 4);
        const uint32_t flg = fb & 0xFF, bd = (fb >> 8) & 0xFF;
        if (flg & 0x14) {   // block / content checksums: the wave kernel verifies them
            st = ST_NOT_RUN;
            break;
        }
        if ((flg >> 1) & 1) {
            st = ST_RESERVED;
            break;
        }
        if (((flg >> 6) & 3) != 1) {
            st = ST_VERSION;
            break;
        }
        const uint32_t csz = (flg >> 3) & 1;
        const uint32_t hdr = 7 + (csz ? 8 : 0) + ((flg & 1) ? 4 : 0);
        if (clen < hdr) {
            st = ST_HDR_INCOMPLETE;
            break;
        }
        const uint32_t bsid = (bd >> 4) & 7;
        if ((bd >> 7) & 1) {
            st = ST_RESERVED;
            break;
        }
        if (bsid < 4) {
            st = ST_MAXBLOCK;
            break;
        }
        if (bd & 15) {
            st = ST_RESERVED;
            break;
        }
        if (((hdr_xxh32(S, W, hdr - 5) >> 8) & 0xFF) != rd1(S, W, hdr - 1)) {
            st = ST_HDR_CHECKSUM;
            break;
        }
        const uint32_t indep = (flg >> 5) & 1;
        const uint64_t csize = csz ? ((uint64_t)rd4(S, W, 6) | ((uint64_t)rd4(S, W, 10) << 32)) : 0;
        const uint32_t max_block = 1u << (8 + 2 * bsid);
        uint32_t ip = hdr;
        ZSK_CT(1)
        st = -1;
        while (st < 0) {
            fail_op = op;
            if (clen - ip < 4) {
                st = ST_TRUNCATED;
                break;
            }
            const uint32_t bh = rd4(S, W, ip);
            ip += 4;
            if (bh == 0) {
                if (csz && csize != op)
                    st = ST_FRAME_SIZE;
                else
                    st = op != dlen ? ST_SHORT_FRAME : ST_OK;
                break;
            }
            const uint32_t bsize = bh & 0x7FFFFFFFu;
            if (bsize > max_block) {
                st = ST_MAXBLOCK;
                break;
            }
            if (clen - ip < bsize) {
                st = ST_TRUNCATED;
                break;
            }
            Blk B;
            B.ib = ip;
            B.iend = ip + bsize;
            B.bop = op;
            B.oend = op + max_block;
            B.floor_ = indep ? op : 0;
            B.dlen = dlen;
            if (bh & 0x80000000u) {
                // stored block: one literal run
                if (op + bsize > dlen) {
                    st = ST_DST_OVERFLOW;
                    break;
                }
                const uint32_t nk = bsize > 255 ? 2 : 1;
                if (k + nk > cap) {
                    st = ST_NOT_RUN;
                    break;
                }
                if (lane == 0) {
                    uint32_t kk = k;
                    put_item(it, kk, ip, bsize, 0, 0);
                }
                k += nk;
                op += bsize;
                ip += bsize;
                continue;
            }
            if (bsize == 0) {
                st = block_fail(B, bsid, max_block);
                break;
            }
            // (ONE: a staged frame's parse without the staged test per read)
            const int32_t bs =
                ONE && S.staged
                    ? chunk_block<ONE, 1, OW>(S, W, B, lane, mapbase, it, k, cap, op, (uint32_t)(uintptr_t)recs,
                                              (uint32_t)(uintptr_t)coll, lead)
                    : chunk_block<ONE, 0, OW>(S, W, B, lane, mapbase, it, k, cap, op, (uint32_t)(uintptr_t)recs,
                                              (uint32_t)(uintptr_t)coll, lead);
            if (bs == ST_BLOCK_ERR)
                st = block_fail(B, bsid, max_block);
            else if (bs >= 0)
                st = bs;
            ip = B.iend;
        }
    } while (false);
#ifdef ZSK_TUNING
    if (ONE && lane == 0)
        atomicAdd(&g_ctime[7], (unsigned long long)(__builtin_readcyclecounter() - tstart_));
#endif
    if (lane == 0) {
        status[f] = st;
        nitems[f] = k;
        if (fail_at)
            fail_at[f] = fail_op;
    }
    };
    if constexpr (ONE) {
        if (blockIdx.x < n)
            frame(blockIdx.x);
    } else {
        // per_wave consecutive frames per wave, their sizes read at once: the
        // ones of this route are parsed in turn (a batch whose frames all
        // take another parse costs one descriptor load per wave, not one
        // wave per frame)
        const uint32_t f0 = uni((blockIdx.x * kCW + w) * per_wave);
        if (f0 >= n)
            return;
        for (uint64_t todo = __ballot(lane < per_wave && f0 + lane < n && desc[f0 + lane].c_size >= min_csize);
             todo; todo &= todo - 1)
            frame(f0 + (uint32_t)__builtin_ctzll(todo));
    }
}

// The one-frame route for a frame of linked 64 KiB blocks (round 6, verdict
// r05 item 7): a 1 MiB frame's 16 blocks went through one workgroup in turn
// (~880 us of parse per miss).  Here the block plan's jobs (one per block,
// lz4_block_plan_kernel) are parsed by a workgroup each, concurrently: the
// block staged in LDS, the one-frame route's chunk parse (chunk_block<true>)
// at the job's speculative output offset j x 64 KiB, its items into the job's
// slots, its result into jres -- what the lean parse's block mode gives the
// block route.  lz4_chunk_kernel<true> then accepts the frame's jobs or
// re-parses the frame (exact status and fail_at) as for the block route.
template <uint32_t OW>
__global__ __launch_bounds__(64 * OW) void lz4_job_parse_kernel(const FrameDesc *__restrict__ desc,
                                                               const uint8_t *__restrict__ comp,
                                                               const uint64_t *__restrict__ rec_base,
                                                               uint64_t capacity, uint64_t *__restrict__ items,
                                                               const BlockJob *__restrict__ jobs,
                                                               BlockRes *__restrict__ jres,
                                                               const uint32_t *__restrict__ njobs, uint32_t lead)
{
    constexpr uint32_t kOneLanes = 64 * OW;
    constexpr uint32_t nsw = kOneStage / 16 > kOneLanes * kWinQ ? kOneStage / 16 : kOneLanes * kWinQ;
    __shared__ __attribute__((aligned(16))) uint32_t maps[kOneLanes * kOneMapW];
    __shared__ __attribute__((aligned(16))) u32x4 stw[nsw];
    __shared__ __attribute__((aligned(16))) uint64_t recs[kOneLanes * one_rec<OW>()];
    __shared__ uint32_t coll[3 * kOneLanes + 16];
    const uint32_t j = blockIdx.x, lane = threadIdx.x;
    if (j >= (uint32_t)__builtin_amdgcn_readfirstlane(*njobs))
        return;
    const BlockJob J = jobs[j];
    if (J.f == kNoJob)
        return;
    const FrameDesc d = desc[J.f];
    const uint32_t ib = J.hpos + 4, iend = J.stop;
    const Span sp = make_span(comp + d.c_off, d.c_size);
    // the block [ib & ~3, iend + 64) staged: frame offset x at stage byte
    // x - (ib & ~3) (chunk_block's staged reads take the frame offset)
    const uint32_t a0 = ib & ~3u, np = (iend + 64 - a0 + 15) / 16;
    const bool staged = np * 16 <= kOneStage;
    if (staged) {
        for (uint32_t i0 = 0; i0 < np; i0 += 4 * kOneLanes) {
            u32x4 v[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t i = i0 + kOneLanes * q + lane;
                v[q] = load16u(sp.r, i < np ? sp.s0 + a0 + 16 * i : 0x80000000u);
            }
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t i = i0 + kOneLanes * q + lane;
                if (i < np)
                    stw[i] = v[q];
            }
        }
    }
    __syncthreads();
    Src S;
    S.r = sp.r;
    S.s0 = sp.s0;
    S.staged = staged;
    S.lds = (uint32_t)(uintptr_t)stw - a0;
    Win W;
    W.base = 0x80000000u;
    W.lds = (uint32_t)(uintptr_t)(stw) + 64 * lane;
    const uint32_t bsid = J.info & 0xFF, max_block = 1u << (8 + 2 * bsid);
    const bool indep = (J.info >> 8) & 1;
    const uint32_t bh = load16u(sp.r, sp.s0 + J.hpos).x, bsize = bh & 0x7FFFFFFFu;
    uint64_t *it = items + rec_base[J.f] + J.slot_off;
    const uint32_t cap = J.slot_cap;
    uint32_t op = J.bop, k = 0;
    int32_t st;
    Blk B;
    B.ib = ib;
    B.iend = iend;
    B.bop = op;
    B.oend = op + max_block;
    B.floor_ = indep ? op : 0;
    B.dlen = d.d_size;
    if (rec_base[J.f] + J.slot_off + cap > capacity || ib + bsize != iend) {
        st = ST_NOT_RUN;
    } else if (bh & 0x80000000u) {   // stored block: one literal run
        const uint32_t nk = bsize > 255 ? 2 : 1;
        st = op + bsize > d.d_size ? ST_DST_OVERFLOW : nk > cap ? ST_NOT_RUN : ST_OK;
        if (st == ST_OK) {
            if (lane == 0)
                put_item(it, k, ib, bsize, 0, 0);
            k = nk;
            op += bsize;
        }
    } else if (bsize == 0) {
        st = block_fail(B, bsid, max_block);
    } else {
        const int32_t bs = staged ? chunk_block<true, 1, OW>(S, W, B, lane, (uint32_t)(uintptr_t)maps, it, k, cap, op,
                                                            (uint32_t)(uintptr_t)recs, (uint32_t)(uintptr_t)coll, lead)
                                  : chunk_block<true, 0, OW>(S, W, B, lane, (uint32_t)(uintptr_t)maps, it, k, cap, op,
                                                            (uint32_t)(uintptr_t)recs, (uint32_t)(uintptr_t)coll, lead);
        st = bs < 0 ? ST_OK : bs == ST_BLOCK_ERR ? block_fail(B, bsid, max_block) : bs;
    }
    if (lane == 0)
        jres[j] = BlockRes{k, op, st, 0};
}

}   // namespace

// the one-frame parse's lead-in (bytes before each chunk): env ZSEEK_ONE_LEAD
// (tuning), default kOneLead
constexpr uint32_t kOneLead = 64;
// the one-frame parse's waves: 8 (64-byte chunks), or 4 (128-byte chunks,
// the round-4 shape) under env ZSEEK_ONE_WAVES=4.  Per frame (tuning timers,
// 64 KiB frames, lead 64): 119.8K cycles at 4 waves, 108.9K at 8 (pass 1
// 27.5K -> 24.4K, emit 33.5K -> 22.8K), 106.8K at 16 (each step slower:
// pass 2 + owners stays ~35K) -- not kept
constexpr uint32_t kOneWavesDef = 8;
static uint32_t one_waves()
{
    static const uint32_t v = [] {
        const char *e = getenv("ZSEEK_ONE_WAVES");
        return e && atoi(e) == 4 ? 4u : kOneWavesDef;
    }();
    return v;
}

uint32_t one_lead()
{
    static const uint32_t v = [] {
        const char *e = getenv("ZSEEK_ONE_LEAD");
        return e ? (uint32_t)atoi(e) : kOneLead;
    }();
    return v;
}

int launch_lz4_job_parse(const FrameDesc *d_desc, const uint8_t *d_comp, const uint64_t *rec_base, uint64_t capacity,
                         uint64_t *items, const SplitScratch *s, uint32_t jobs, hipStream_t stream)
{
    if (jobs == 0)
        return 0;
    hipLaunchKernelGGL((lz4_job_parse_kernel<8>), dim3(jobs), dim3(64 * 8), 0, stream, d_desc, d_comp, rec_base,
                       capacity, items, s->jobs, s->jres, s->njobs, one_lead());
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_lz4_chunk(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                     const uint64_t *rec_base, uint64_t capacity, uint64_t *items, uint32_t *nitems,
                     int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream, uint32_t min_csize,
                     SplitScratch *blk, uint32_t min_jobs, bool one, uint64_t *solo_total)
{
    if (nframes == 0)
        return 0;
    if (one) {
        // (blk: the big frames' jobs, lz4_job_parse_kernel's results)
        if (one_waves() == 8)
            hipLaunchKernelGGL((lz4_chunk_kernel<true, 8>), dim3(nframes), dim3(64 * 8), 0, stream, d_desc, nframes,
                               d_comp, rec_base, capacity, items, nitems, d_status, d_fail_at, min_csize,
                               blk ? blk->bfirst : nullptr, blk ? blk->bcount : nullptr, blk ? blk->jobs : nullptr,
                               blk ? blk->jres : nullptr, blk ? blk->njobs : nullptr, min_jobs,
                               solo_total, 1u, one_lead());
        else
            hipLaunchKernelGGL((lz4_chunk_kernel<true, 4>), dim3(nframes), dim3(64 * 4), 0, stream, d_desc, nframes,
                               d_comp, rec_base, capacity, items, nitems, d_status, d_fail_at, min_csize,
                               blk ? blk->bfirst : nullptr, blk ? blk->bcount : nullptr, blk ? blk->jobs : nullptr,
                               blk ? blk->jres : nullptr, blk ? blk->njobs : nullptr, min_jobs,
                               solo_total, 1u, one_lead());
#ifdef ZSK_TUNING
        if (getenv("ZSEEK_CHUNK_TIMERS")) {
            unsigned long long z[16];
            (void)hipStreamSynchronize(stream);
            (void)hipMemcpyFromSymbol(z, HIP_SYMBOL(g_ctime), sizeof(z), 0, hipMemcpyDeviceToHost);
            static unsigned long long acc[16];
            static int calls = 0;
            for (int i = 0; i < 16; i++)
                acc[i] += z[i];
            memset(z, 0, sizeof(z));
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_ctime), z, sizeof(z), 0, hipMemcpyHostToDevice);
            if (++calls % 100 == 0) {
                const double nf = (double)calls, nb = (double)(acc[12] ? acc[12] : 1);
                fprintf(stderr,
                        "chunk one-route cycles per frame: stage %.0f hdr %.0f pass1 %.0f pass2+own %.0f count %.0f "
                        "emit %.0f total %.0f | per block wave-max iters: pass1 %.1f pass2 %.1f (%d frames) | pass2 "
                        "alone %.0f, owner jumps in %.2f of blocks, workgroup-max iters pass1 %.1f pass2 %.1f\n",
                        acc[0] / nf, acc[1] / nf, acc[2] / nf, acc[3] / nf + acc[11] / nf, acc[4] / nf, acc[5] / nf,
                        acc[7] / nf, acc[8] / nb, acc[9] / nb, calls, acc[11] / nf, acc[13] / nb, acc[14] / nb,
                        acc[15] / nb);
            }
        }
#endif
    } else {
        // frames per wave: >= 16,384 waves whatever the batch (every frame may
        // take this parse), at most 64
        const uint32_t per = min(64u, max(1u, nframes / 16384));
        const uint32_t waves = (nframes + per - 1) / per;
        hipLaunchKernelGGL(lz4_chunk_kernel<false>, dim3((waves + kCW - 1) / kCW), dim3(64 * kCW), 0, stream,
                           d_desc, nframes, d_comp, rec_base, capacity, items, nitems, d_status, d_fail_at,
                           min_csize, blk ? blk->bfirst : nullptr, blk ? blk->bcount : nullptr,
                           blk ? blk->jobs : nullptr, blk ? blk->jres : nullptr, blk ? blk->njobs : nullptr,
                           min_jobs, nullptr, per, 0u);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk
