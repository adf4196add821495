// seq_exec.hip — the execute phase's launchers and the one-frame route's
// executes (gfx950): seq_exec_frame_kernel (a frame of <= 64 KiB staged whole
// in LDS per workgroup) and seq_exec_big_kernel (bigger frames through a
// sliding 64 KiB window).  The throughput kernel seq_exec_kernel<OUTB, SEG> and its
// helpers live in seq_exec_dev.h (shared with seq_exec_seg.hip and the
// tuning build's seq_exec_tune.hip, which holds the diagnostic variants).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "lz4_wave_dev.h"   // the one-frame execute decodes its batch's hand-offs
#include "seq_exec_dev.h"

namespace zsk {

namespace {

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

// 1..64 bytes between disjoint LDS ranges with whole-width writes only:
// 16-byte pieces from the start plus one ending at n (overlapping pieces
// rewrite equal bytes), two 8- or 4-byte ones below 16 bytes -- no per-piece
// partial-store branches (reads may run past the source: the arrays have
// slack)
__device__ __forceinline__ void scopy(uint32_t dst, uint32_t src, uint32_t n)
{
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
}

// n bytes from LDS src to LDS dst, dst - src >= step or the ranges apart: up
// to four 16-byte pieces read before they are written (a piece's source was
// written at least `step` bytes earlier)
__device__ __forceinline__ void lcopy(uint32_t dst, uint32_t src, uint32_t n, uint32_t step)
{
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
}

__global__ __launch_bounds__(kFT) void seq_exec_frame_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ rec_base, const uint64_t *__restrict__ items, const uint32_t *__restrict__ nitems,
    int32_t *__restrict__ status, uint32_t *__restrict__ fail_at, uint32_t stop_last, uint32_t handoff,
    const uint8_t *__restrict__ lit, const HostPost post)
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
        if (handoff && wv == 0) {
            lz4w::wave_frame<4096>(desc, f, comp, out, status, fail_at, ob);
            if (post.h_flag) {
                // (post: wave 0's decoded bytes, from HBM, then its status)
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
                const uint8_t *src = out + d.d_off + post.h_from;
                const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3);
                for (uint32_t c = lane; 16 * c < post.h_len; c += 64) {
                    const uint32_t *a = reinterpret_cast<const uint32_t *>(src - sh) + 4 * c;
                    uint32_t w[5];
#pragma unroll
                    for (int k = 0; k < 5; k++)
                        w[k] = a[k];
                    u32x4 v;
                    v.x = __builtin_amdgcn_alignbyte(w[1], w[0], sh);
                    v.y = __builtin_amdgcn_alignbyte(w[2], w[1], sh);
                    v.z = __builtin_amdgcn_alignbyte(w[3], w[2], sh);
                    v.w = __builtin_amdgcn_alignbyte(w[4], w[3], sh);
                    reinterpret_cast<u32x4 *>(post.h_out)[c] = v;
                }
                if (lane == 0) {
                    post.h_status[0] = (uint32_t)status[f];
                    post.h_status[1] = fail_at ? fail_at[f] : 0u;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                if (lane == 0)
                    __hip_atomic_store(post.h_flag, post.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
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
    if (post.h_flag) {
        // a lone frame's results to the host from the staged output (the
        // request's bytes; past E they are whatever LDS holds, as HBM's would
        // be), then the flag once every wave's stores are complete
        for (uint32_t c = t; 16 * c < post.h_len; c += kFT)
            reinterpret_cast<u32x4 *>(post.h_out)[c] = lds16(ob0 + post.h_from + 16 * c);
        if (t == 0) {
            post.h_status[0] = (uint32_t)status[f];
            post.h_status[1] = fail_at ? fail_at[f] : 0u;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (t == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __hip_atomic_store(post.h_flag, post.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
#ifdef ZSK_TUNING
    __syncthreads();
    ZSK_FT(4)
#endif
}
#undef ZSK_FT

// ---- the one-frame route's execute for frames of more than 64 KiB ----
// (round 6, verdict r05 item 7: a 1 MiB frame's execute on one wave took
// ~890 us per miss).  One frame per 1,024-thread workgroup, as
// seq_exec_frame_kernel, through a sliding window: LDS holds the 64 KiB of
// output before the window (every byte final: LZ4's offsets reach 65,535
// back) and the window itself, 64 KiB at frame offset H.  A batch of 2,048
// items is placed by the same workgroup scan and cut before the first item
// that would end past the window; literal runs are copied from HBM (the
// compressed frame does not fit beside the window), matches resolve in the
// per-wave passes over the window's done bits, a source byte before H
// always ready.  Then the window's bytes go out and it slides to the first
// byte not decoded (the 64 KiB before it moved down as the new history).
// Items: contiguous (rec_base[f]), or -- a frame the block route accepted
// (bfirst[f] != kNoJob, the job parse of lz4_chunk.hip) -- job by job, item
// index i mapped onto its job's slots through a table of the jobs' first
// indices.  A frame no window can take (an item longer than 64 KiB: blocks
// over 64 KiB) and the batch's hand-offs (ST_NOT_RUN) are decoded by the
// wave decoder on wave 0 instead.
constexpr uint32_t kBWin = 65536;

#ifdef ZSK_TUNING
// tuning builds: seq_exec_big_kernel's phase cycles (thread 0): [0] init,
// [1] items + scans, [2] cut + literal runs, [3] match passes, [4] slides,
// [5] last output; [6] slides, [7] batches, [8] frames (ZSEEK_BIG_TIMERS)
__device__ unsigned long long g_btime[9];
#define ZSK_BT(i)                                                             \
    {                                                                         \
        const uint64_t tn_ = __builtin_readcyclecounter();                    \
        if (t == 0)                                                           \
            atomicAdd(&g_btime[i], (unsigned long long)(tn_ - tmark_));       \
        tmark_ = tn_;                                                         \
    }
#define ZSK_BC(i)                                                             \
    if (t == 0)                                                               \
        atomicAdd(&g_btime[i], 1ull);
#else
#define ZSK_BT(i)
#define ZSK_BC(i)
#endif

__global__ __launch_bounds__(kFT) void seq_exec_big_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ rec_base, const uint64_t *__restrict__ items, const uint32_t *__restrict__ nitems,
    int32_t *__restrict__ status, uint32_t *__restrict__ fail_at, uint32_t stop_last, uint32_t handoff,
    const uint32_t *__restrict__ bfirst, const uint32_t *__restrict__ bcount, const BlockJob *__restrict__ jobs,
    const BlockRes *__restrict__ jres, uint32_t skip_jobs)
{
    __shared__ __attribute__((aligned(16))) uint8_t ob[2 * kBWin + 80];
    __shared__ uint32_t done[kBWin / 32 + 2];
    __shared__ uint32_t wsum[kFT / 64];
    __shared__ uint32_t jtab[2 * kMaxBlockJobs];   // per job: its first item index, slot offset - that index
    __shared__ uint32_t cut_i, cut_op, hi_end;
    const uint32_t f = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (f >= n)
        return;
    const FrameDesc d = desc[f];
    if (d.d_size <= kFMax)
        return;   // seq_exec_frame_kernel's frame
    // (a frame the block route accepted whose jobs are all below skip_jobs
    // is seq_exec_blocks_kernel's)
    if (skip_jobs && bfirst) {
        const uint32_t bf = __builtin_amdgcn_readfirstlane(bfirst[f]);
        if (bf != kNoJob && bf + (uint32_t)__builtin_amdgcn_readfirstlane(bcount[f]) <= skip_jobs)
            return;
    }
    // the windowed execute; false: stuck (an item longer than the window)
    auto window_frame = [&]() -> bool {
#ifdef ZSK_TUNING
        uint64_t tmark_ = __builtin_readcyclecounter();
#endif
        const uint32_t j0 = bfirst ? __builtin_amdgcn_readfirstlane(bfirst[f]) : kNoJob;
        const uint32_t nj = j0 != kNoJob ? __builtin_amdgcn_readfirstlane(bcount[f]) : 0u;
        uint32_t nit;
        if (nj) {
            if (wv == 0) {
                uint32_t so = 0, k = 0;
                if (lane < nj) {
                    so = jobs[j0 + lane].slot_off;
                    k = jres[j0 + lane].n;
                }
                const uint32_t inc = wave_incl_add(k);
                if (lane < nj) {
                    jtab[2 * lane] = inc - k;
                    jtab[2 * lane + 1] = so - (inc - k);
                }
                if (lane == 63)
                    wsum[0] = inc;
            }
            __syncthreads();
            nit = wsum[0];
        } else {
            nit = nitems[f];
        }
        // item index -> slot (relative to rec_base[f]): the last job starting at
        // or before i (job starts ascend: an accepted job has items)
        auto slot = [&](uint32_t i) -> uint32_t {
            if (nj == 0)
                return i;
            uint32_t lo = 0, hi = nj;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (jtab[2 * mid] <= i)
                    lo = mid;
                else
                    hi = mid;
            }
            return i + jtab[2 * lo + 1];
        };
        const uint32_t stop = f + 1 == n ? min(stop_last, d.d_size) : d.d_size;
        const uint64_t *it = items + rec_base[f];
        const Span lsp = make_span(comp + d.c_off, d.c_size);
        uint8_t *o = out + d.d_off;
        const uint32_t ob0 = (uint32_t)(uintptr_t)ob, C = ob0 + kBWin;   // window byte x at C + x - H
        for (uint32_t i = t; i < kBWin / 32 + 2; i += kFT)
            done[i] = 0;
        if (t == 0)
            hi_end = 0;
        __syncthreads();
        ZSK_BT(0)
        ZSK_BC(8)

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
        auto mark = [&](uint32_t a, uint32_t len) {   // window bytes [a, a + len) written
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            for (const uint32_t e = a + len; a < e;) {
                const uint32_t b0 = a & 31, nb = min(32 - b0, e - a);
                __hip_atomic_fetch_or(&done[a >> 5], nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1) << b0, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                a += nb;
            }
        };
        auto ready = [&](uint32_t a, uint32_t len) -> bool {   // window bytes
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
        // frame bytes [a, e) of the window out: a byte head to 16-byte
        // alignment, whole 16-byte stores, a byte tail
        auto put_out = [&](uint32_t H, uint32_t a, uint32_t e) {
            if (e <= a)
                return;
            const uint32_t head = min(e - a, (uint32_t)((16 - ((uintptr_t)(o + a) & 15)) & 15));
            const uint32_t w = kBWin + a - H;
            if (t < head)
                o[a + t] = ob[w + t];
            const uint32_t nchunks = (e - a - head) / 16;
            for (uint32_t c = t; c < nchunks; c += kFT)
                *reinterpret_cast<u32x4 *>(o + a + head + 16 * c) = lds16(ob0 + w + head + 16 * c);
            const uint32_t tail0 = head + 16 * nchunks;
            if (tail0 + t < e - a)
                o[a + tail0 + t] = ob[w + tail0 + t];
        };

        uint32_t H = 0, P = 0, w0 = 0;   // window start, bytes decoded, next item
        bool stuck = false;
        while (w0 < nit && P < stop) {
            if (t == 0) {
                cut_i = 0xFFFFFFFFu;
                cut_op = 0xFFFFFFFFu;
            }
            uint32_t lit[2], ml[2], off[2], src[2], op[2], tot[2], idx[2];
            for (int j = 0; j < 2; j++) {
                const uint32_t i = w0 + j * kFT + t;
                idx[j] = i;
                lit[j] = ml[j] = off[j] = src[j] = 0;
                if (i < nit) {
                    const uint32_t si = slot(i);
                    const uint64_t cur = it[si];
                    const uint32_t c0 = (uint32_t)cur, c1 = (uint32_t)(cur >> 32);
                    const bool second = i > 0 && ((uint32_t)it[slot(i - 1)] & kItemExt);   // an extended item's second half
                    if (!second) {
                        src[j] = c0 & kItemPos;
                        if (c0 & kItemExt) {
                            const uint64_t nx = it[si + 1];
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
            ZSK_BT(1)
            ZSK_BC(7)
            op[0] = P + x0;
            op[1] = P + tot[0] + x1;
            // the cut: the first item ending past the window (ops ascend with the
            // index, so the smallest index and op are the same item's)
            for (int j = 0; j < 2; j++) {
                const bool over = lit[j] + ml[j] != 0 && op[j] + lit[j] + ml[j] > H + kBWin;
                const uint64_t ov = __ballot(over);
                if (ov && lane == (uint32_t)__builtin_ctzll(ov)) {
                    atomicMin(&cut_i, idx[j]);
                    atomicMin(&cut_op, op[j]);
                }
            }
            __syncthreads();
            const uint32_t ci = cut_i, lim = min(cut_op, stop);
            bool pend[2];
            for (int j = 0; j < 2; j++) {
                const bool on = op[j] < lim && lit[j] + ml[j] != 0;
                const uint32_t L = on ? lit[j] : 0;
                const uint32_t dst = C + op[j] - H;
                const bool coop = L > kFLong;   // (as seq_exec_frame_kernel)
                for (uint64_t lm = __ballot(coop); lm; lm &= lm - 1) {
                    const int q = (int)__builtin_ctzll(lm);
                    const uint32_t d0 = lane_val(dst, q), s = lane_val(src[j], q), nq = lane_val(L, q);
                    for (uint32_t k = 16 * lane; k < nq; k += 1024)
                        lds_put(d0 + k, load16u(lsp.r, lsp.s0 + s + k), min(16u, nq - k));
                }
                if (!coop && L) {
                    // up to 64 bytes per step, four 16-byte loads in flight
                    for (uint32_t k = 0; k < L; k += 64) {
                        u32x4 v[4];
    #pragma unroll
                        for (uint32_t q = 0; q < 4; q++)
                            v[q] = load16u(lsp.r, k + 16 * q < L ? lsp.s0 + src[j] + k + 16 * q : kBad);
    #pragma unroll
                        for (uint32_t q = 0; q < 4; q++)
                            if (k + 16 * q < L)
                                lds_put(dst + k + 16 * q, v[q], min(16u, L - k - 16 * q));
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                for (uint64_t lm = __ballot(coop); lm; lm &= lm - 1) {
                    const int q = (int)__builtin_ctzll(lm);
                    const uint32_t a = lane_val(op[j], q) - H, e = a + lane_val(L, q) - 1;
                    for (uint32_t g = (a >> 5) + lane; g <= e >> 5; g += 64) {
                        const uint32_t lo = g == a >> 5 ? a & 31 : 0, hi = g == e >> 5 ? e & 31 : 31;
                        const uint32_t m = hi - lo == 31 ? 0xFFFFFFFFu : ((1u << (hi - lo + 1)) - 1) << lo;
                        __hip_atomic_fetch_or(&done[g], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                if (!coop && L)
                    mark(op[j] - H, L);
                pend[j] = on && ml[j] != 0;
            }
            {
                const bool on0 = op[0] < lim && lit[0] + ml[0] != 0, on1 = op[1] < lim && lit[1] + ml[1] != 0;
                const uint32_t e = max(on0 ? op[0] + lit[0] + ml[0] : 0u, on1 ? op[1] + lit[1] + ml[1] : 0u);
                const uint32_t we = wave_incl_max(e);
                if (lane == 63 && we)
                    atomicMax(&hi_end, we);
            }
            __syncthreads();
            ZSK_BT(2)
            for (uint32_t pass = 0;; pass++) {
                bool moved = false;
                for (int j = 0; j < 2; j++) {
                    if (!pend[j])
                        continue;
                    const uint32_t mb = op[j] + lit[j], ov = off[j], m = ml[j];
                    // the source's first min(off, ml) bytes: those before H are final
                    const uint32_t s0 = mb - ov, s1 = s0 + (ov >= m ? m : ov);
                    if (s1 > H && !ready(s0 > H ? s0 - H : 0u, s1 - (s0 > H ? s0 : H)))
                        continue;
                    const uint32_t db = C + mb - H, sb = db - ov;
                    if (ov >= m && m <= 128) {
                        scopy(db, sb, min(m, 64u));
                        if (m > 64)
                            scopy(db + 64, sb + 64, m - 64);
                    } else if (ov >= m || ov >= 16) {
                        lcopy(db, sb, m, ov >= m ? 64u : min(64u, ov & ~15u));
                    } else {
                        const uint32_t e = ov * ((16 + ov - 1) / ov);
                        const uint32_t h = min(e, m);
                        for (uint32_t k = 0; k < h; k++) {
                            *lp<uint8_t>(db + k) = *lp<uint8_t>(sb + k);
                            wave_lds_sync();
                        }
                        for (uint32_t k = h; k < m; k += 16) {
                            lds_put(db + k, lds16(db + k - e), min(16u, m - k));
                            wave_lds_sync();
                        }
                    }
                    mark(mb - H, m);
                    pend[j] = false;
                    moved = true;
                }
                if (!__any(pend[0] || pend[1]) || pass > (1u << 22))
                    break;
                if (!__any(moved))
                    __builtin_amdgcn_s_sleep(1);
            }
            __syncthreads();
            ZSK_BT(3)
            const uint32_t P1 = ci != 0xFFFFFFFFu ? min(cut_op, P + tot[0] + tot[1]) : P + tot[0] + tot[1];
            if (ci != 0xFFFFFFFFu && P1 == H) {   // one item longer than the window
                stuck = true;
                break;
            }
            P = P1;
            w0 = ci != 0xFFFFFFFFu ? ci : w0 + 2 * kFT;
            // slide once the window is cut or three quarters full (and there is
            // more to decode): its bytes out, the 64 KiB before P down as history
            if ((ci != 0xFFFFFFFFu || P - H >= kBWin - kBWin / 4) && w0 < nit && P < stop) {
                put_out(H, H, P);
                const uint32_t sh = P - H;
                u32x4 v[4];
    #pragma unroll
                for (uint32_t q = 0; q < 4; q++)
                    v[q] = lds16(ob0 + sh + 16 * (t + q * kFT));
                __syncthreads();
    #pragma unroll
                for (uint32_t q = 0; q < 4; q++)
                    *lp<u32x4>(ob0 + 16 * (t + q * kFT)) = v[q];
                for (uint32_t i = t; i < kBWin / 32 + 2; i += kFT)
                    done[i] = 0;
                __syncthreads();
                H = P;
                ZSK_BT(4)
                ZSK_BC(6)
            }
        }
        if (stuck)
            return false;
        put_out(H, H, min(hi_end, d.d_size));
#ifdef ZSK_TUNING
        __syncthreads();
        ZSK_BT(5)
#endif
        return true;
    };
    // the wave decoder's frame: a hand-off, or one no window can take (one
    // call site: the decoder inlined twice spilled)
    bool whole = __builtin_amdgcn_readfirstlane(status[f]) == ST_NOT_RUN;
    if (whole && !handoff)
        return;
    if (!whole)
        whole = !window_frame();
    if (whole) {
        if (wv == 0)
            lz4w::wave_frame<4096>(desc, f, comp, out, status, fail_at, ob);
    }
}

// ---- the one-frame route's big frames, block-parallel (round 6) ----
// A frame the block route accepted (64 KiB linked blocks, each block's items
// in its job's slots) is executed a block per 1,024-thread workgroup, all
// blocks at once.  A block's matches may read up to 64 KiB back, i.e. the
// previous block's output, which its own workgroup is still producing; so:
//   A. every workgroup executes its block at once with the previous block's
//      bytes unknown: the frame kernel's literal copies and match passes over
//      the block staged in LDS (block byte x at B + x).  A byte copied from
//      before the block, or from a byte so copied, is *tainted* (a bit per
//      byte): it holds not its value but its *origin*, the previous block's
//      byte it is a copy of, low byte at B + x and high byte at B - 64 KiB + x
//      (the LDS below B, free in this kernel).  A match reading no tainted
//      byte copies as usual; one that does carries values, origins and taint
//      bits -- in 16-byte pieces on its lane, or (offsets < 16, matches over
//      256 bytes) with the wave's 64 lanes a byte each (taint bits set before
//      the done bits, so a match that sees its source done sees its taint
//      too);
//   B. the block goes out at once, its untainted bytes final, and its taint
//      bits and origins go to the job's scratch (borg, btaint); then it
//      publishes (jres[j].pad, release at agent scope).  A block with tainted
//      bytes splits them evenly over its threads (binary searches over the
//      taint words' prefix counts), waits for every earlier block of its frame
//      to publish (acquire), and follows each tainted byte back block by block
//      -- an untainted byte at (block, position) is the value, a tainted one
//      names its origin one block further back -- then stores the values
//      over the origins.
// No block waits for another's final bytes: the wait is for phase A (all
// blocks finish it about together) and a chain of h hops costs h load round
// trips.  The waits are on lower-numbered workgroups, dispatched first, and
// bounded (~1 s), so a broken chain cannot hang the GPU.  The last frame
// stops at stop_last (later blocks skip).  A frame with a job at or past
// borg_cap (the scratch's jobs) is left to seq_exec_big_kernel.
#ifdef ZSK_TUNING
// tuning builds: seq_exec_blocks_kernel's timeline (ZSEEK_BLK_TIMERS), per
// job < 64: realtime at start, after phase A, after the untainted bytes went
// out, after the wait, after the gather, at the end; the tainted matches and
// bytes
__device__ unsigned long long g_ktime[64][10];
#define ZSK_KT(i)                                                             \
    if (t == 0 && j < 64)                                                     \
        g_ktime[j][i] = __builtin_amdgcn_s_memrealtime();
#else
#define ZSK_KT(i)
#endif

__global__ __launch_bounds__(kFT) void seq_exec_blocks_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp, uint8_t *__restrict__ out,
    const uint64_t *__restrict__ rec_base, const uint64_t *__restrict__ items,
    const uint32_t *__restrict__ bfirst, const BlockJob *__restrict__ jobs, BlockRes *__restrict__ jres,
    const uint32_t *__restrict__ njobs, uint32_t stop_last, uint16_t *__restrict__ borg,
    uint32_t *__restrict__ btaint, const uint32_t *__restrict__ bcount, uint32_t borg_cap)
{
    __shared__ __attribute__((aligned(16))) uint8_t ob[2 * kBWin + 80];   // origins' high bytes, then the block
    __shared__ uint32_t done[kBWin / 32 + 2];
    __shared__ uint32_t taint[kBWin / 32 + 2];
    __shared__ uint32_t wsum[kFT / 64];
    __shared__ uint32_t ntm, hi_end;
    const uint32_t j = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (j >= (uint32_t)__builtin_amdgcn_readfirstlane(*njobs))
        return;
    const BlockJob J = jobs[j];
    if (J.f == kNoJob || J.f >= n)
        return;
    const uint32_t f = J.f;
    const uint32_t j0 = __builtin_amdgcn_readfirstlane(bfirst[f]);
    if (j0 == kNoJob || j0 + (uint32_t)__builtin_amdgcn_readfirstlane(bcount[f]) > borg_cap)
        return;   // re-parsed, or jobs past the scratch: seq_exec_big_kernel's frame
    const FrameDesc d = desc[f];
    const uint32_t stop = f + 1 == n ? min(stop_last, d.d_size) : d.d_size;
    const uint32_t bop = J.bop;
    auto publish = [&]() {   // this block's phase A is out
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (t == 0)
            __hip_atomic_store(&jres[j].pad, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    };
    if (bop >= stop) {
        publish();
        return;
    }
    ZSK_KT(0)
    const uint32_t lim = min(stop - bop, kBWin);   // block bytes the request needs
    const uint32_t nit = jres[j].n;
    const uint64_t *it = items + rec_base[f] + J.slot_off;
    const Span lsp = make_span(comp + d.c_off, d.c_size);
    const uint32_t ob0 = (uint32_t)(uintptr_t)ob, B = ob0 + kBWin;   // block byte x at B + x
    for (uint32_t i = t; i < kBWin / 32 + 2; i += kFT)
        done[i] = taint[i] = 0;
    if (t == 0) {
        hi_end = 0;
        ntm = 0;
    }
    __syncthreads();

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
    auto bits_or = [&](uint32_t *w, uint32_t a, uint32_t len) {
        for (const uint32_t e = a + len; a < e;) {
            const uint32_t b0 = a & 31, nb = min(32 - b0, e - a);
            __hip_atomic_fetch_or(&w[a >> 5], nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1) << b0, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
            a += nb;
        }
    };
    auto all_set = [&](uint32_t *w, uint32_t a, uint32_t len) -> bool {
        bool all = true;
        for (const uint32_t e = a + len; a < e;) {
            const uint32_t b0 = a & 31, nb = min(32 - b0, e - a);
            const uint32_t m = nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1) << b0;
            all &= (__hip_atomic_load(&w[a >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & m) == m;
            a += nb;
        }
        return all;
    };
    auto any_set = [&](uint32_t *w, uint32_t a, uint32_t len) -> bool {
        bool any = false;
        for (const uint32_t e = a + len; a < e;) {
            const uint32_t b0 = a & 31, nb = min(32 - b0, e - a);
            const uint32_t m = nb == 32 ? 0xFFFFFFFFu : ((1u << nb) - 1) << b0;
            any |= (__hip_atomic_load(&w[a >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & m) != 0;
            a += nb;
        }
        return any;
    };
    auto mark = [&](uint32_t a, uint32_t len) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        bits_or(done, a, len);
    };
    // a match reading no tainted byte: a plain copy inside the staged block
    auto copy_match = [&](uint32_t mb, uint32_t ov, uint32_t m) {
        const uint32_t db = B + mb, sb = db - ov;
        if (ov >= m && m <= 128) {
            scopy(db, sb, min(m, 64u));
            if (m > 64)
                scopy(db + 64, sb + 64, m - 64);
        } else if (ov >= m || ov >= 16) {
            lcopy(db, sb, m, ov >= m ? 64u : min(64u, ov & ~15u));
        } else {
            const uint32_t e = ov * ((16 + ov - 1) / ov);
            const uint32_t h = min(e, m);
            for (uint32_t k = 0; k < h; k++) {
                *lp<uint8_t>(db + k) = *lp<uint8_t>(sb + k);
                wave_lds_sync();
            }
            for (uint32_t k = h; k < m; k += 16) {
                lds_put(db + k, lds16(db + k - e), min(16u, m - k));
                wave_lds_sync();
            }
        }
    };
    // one that does: the wave's 64 lanes a byte each, byte k's source
    // s = mb - ov + k mod ov (before the match, so the bytes are independent;
    // an overlapping match repeats its first ov source bytes), a byte before
    // the block becoming the origin s + 64 KiB, a tainted one passing its
    // origin on, an untainted one its value; the taint bits of 64 bytes at a
    // time from a ballot
    auto taint_wide = [&](uint32_t mb, uint32_t ov, uint32_t m) {
        const int32_t s0 = (int32_t)mb - (int32_t)ov;
        for (uint32_t k0 = 0; k0 < m; k0 += 64) {
            const uint32_t k = k0 + lane;
            const bool in = k < m;
            bool tb = false;
            if (in) {
                const int32_t s = s0 + (int32_t)(ov >= m ? k : k % ov);
                const uint32_t x = mb + k;
                if (s < 0) {
                    const uint32_t h = (uint32_t)(s + (int32_t)kBWin);
                    *lp<uint8_t>(B + x) = (uint8_t)h;
                    *lp<uint8_t>(ob0 + x) = (uint8_t)(h >> 8);
                    tb = true;
                } else {
                    const uint32_t sx = (uint32_t)s;
                    tb = (__hip_atomic_load(&taint[sx >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >>
                          (sx & 31)) & 1;
                    *lp<uint8_t>(B + x) = *lp<uint8_t>(B + sx);
                    if (tb)
                        *lp<uint8_t>(ob0 + x) = *lp<uint8_t>(ob0 + sx);
                }
            }
            const uint64_t bm = __ballot(tb);
            if (lane == 0 && bm) {
                const uint32_t x0 = mb + k0, w = x0 >> 5, sh = x0 & 31;
                const uint64_t lo = bm << sh;
                const uint32_t w2 = sh ? (uint32_t)(bm >> (64 - sh)) : 0u;
                if ((uint32_t)lo)
                    __hip_atomic_fetch_or(&taint[w], (uint32_t)lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if ((uint32_t)(lo >> 32))
                    __hip_atomic_fetch_or(&taint[w + 1], (uint32_t)(lo >> 32), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                if (w2)
                    __hip_atomic_fetch_or(&taint[w + 2], w2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    };
    // ... or, offset >= 16, by one lane in pieces of <= 16 bytes: a piece
    // from before the block its 16 origins built in registers, one from the
    // block its value and origin bytes and its 16 taint bits copied over
    auto taint_copy = [&](uint32_t mb, uint32_t ov, uint32_t m) {
        for (uint32_t k = 0; k < m;) {
            const uint32_t x = mb + k;
            const int32_t s = (int32_t)x - (int32_t)ov;
            uint32_t n = min(16u, m - k), bits;
            if (s < 0) {
                n = min(n, (uint32_t)-s);
                const uint32_t h0 = (uint32_t)(s + (int32_t)kBWin);
                uint32_t lo[4], hi[4];
#pragma unroll
                for (uint32_t i = 0; i < 4; i++) {
                    lo[i] = hi[i] = 0;
#pragma unroll
                    for (uint32_t b = 0; b < 4; b++) {
                        const uint32_t h = h0 + 4 * i + b;
                        lo[i] |= (h & 0xFF) << (8 * b);
                        hi[i] |= (h >> 8) << (8 * b);
                    }
                }
                lds_put(B + x, u32x4{lo[0], lo[1], lo[2], lo[3]}, n);
                lds_put(ob0 + x, u32x4{hi[0], hi[1], hi[2], hi[3]}, n);
                bits = (1u << n) - 1;
            } else {
                const uint32_t sx = (uint32_t)s;
                const uint64_t w = (uint64_t)__hip_atomic_load(&taint[sx >> 5], __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP) |
                                   (uint64_t)__hip_atomic_load(&taint[(sx >> 5) + 1], __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP) << 32;
                bits = (uint32_t)(w >> (sx & 31)) & ((1u << n) - 1);
                lds_put(B + x, lds16(B + sx), n);
                if (bits)
                    lds_put(ob0 + x, lds16(ob0 + sx), n);
            }
            if (bits) {
                const uint64_t sh = (uint64_t)bits << (x & 31);
                __hip_atomic_fetch_or(&taint[x >> 5], (uint32_t)sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if ((uint32_t)(sh >> 32))
                    __hip_atomic_fetch_or(&taint[(x >> 5) + 1], (uint32_t)(sh >> 32), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            k += n;
        }
    };
    // the readiness range of a match at mb: its source's first min(off, ml)
    // bytes, clipped to the block (bytes before it: always "ready")
    auto src_range = [&](uint32_t mb, uint32_t ov, uint32_t m, uint32_t &a, uint32_t &len) -> bool {
        const int32_t s0 = (int32_t)mb - (int32_t)ov, s1 = s0 + (int32_t)(ov >= m ? m : ov);
        a = s0 > 0 ? (uint32_t)s0 : 0u;
        len = s1 > (int32_t)a ? (uint32_t)s1 - a : 0u;
        return s0 < 0;   // reaches before the block
    };

    // ---- phase A: the block's items, batches of 2,048 ----
    {
        uint32_t P = 0;
        for (uint32_t w0 = 0; w0 < nit && P < lim; w0 += 2 * kFT) {
            uint32_t lit[2], ml[2], off[2], src[2], op[2], tot[2];
            for (int q = 0; q < 2; q++) {
                const uint32_t i = w0 + q * kFT + t;
                lit[q] = ml[q] = off[q] = src[q] = 0;
                if (i < nit) {
                    const uint64_t cur = it[i];
                    const uint32_t c0 = (uint32_t)cur, c1 = (uint32_t)(cur >> 32);
                    const bool second = i > 0 && ((uint32_t)it[i - 1] & kItemExt);
                    if (!second) {
                        src[q] = c0 & kItemPos;
                        if (c0 & kItemExt) {
                            const uint64_t nx = it[i + 1];
                            lit[q] = (uint32_t)nx;
                            ml[q] = (uint32_t)(nx >> 32);
                            off[q] = c1;
                        } else {
                            lit[q] = (c1 >> 16) & 0xFF;
                            const uint32_t mc = c1 >> 24;
                            ml[q] = mc ? mc + 3 : 0;
                            off[q] = c1 & 0xFFFF;
                        }
                    }
                }
            }
            const uint32_t x0 = scan(lit[0] + ml[0], tot[0]);
            const uint32_t x1 = scan(lit[1] + ml[1], tot[1]);
            op[0] = P + x0;
            op[1] = P + tot[0] + x1;
            bool pend[2];
            for (int q = 0; q < 2; q++) {
                const bool on = op[q] < lim && lit[q] + ml[q] != 0 && op[q] + lit[q] + ml[q] <= kBWin;
                const uint32_t L = on ? lit[q] : 0;
                const uint32_t dst = B + op[q];
                const bool coop = L > kFLong;
                for (uint64_t lm = __ballot(coop); lm; lm &= lm - 1) {
                    const int qq = (int)__builtin_ctzll(lm);
                    const uint32_t d0 = lane_val(dst, qq), sx = lane_val(src[q], qq), nq = lane_val(L, qq);
                    for (uint32_t k = 16 * lane; k < nq; k += 1024)
                        lds_put(d0 + k, load16u(lsp.r, lsp.s0 + sx + k), min(16u, nq - k));
                }
                if (!coop && L) {
                    for (uint32_t k = 0; k < L; k += 64) {
                        u32x4 v[4];
#pragma unroll
                        for (uint32_t qq = 0; qq < 4; qq++)
                            v[qq] = load16u(lsp.r, k + 16 * qq < L ? lsp.s0 + src[q] + k + 16 * qq : kBad);
#pragma unroll
                        for (uint32_t qq = 0; qq < 4; qq++)
                            if (k + 16 * qq < L)
                                lds_put(dst + k + 16 * qq, v[qq], min(16u, L - k - 16 * qq));
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                for (uint64_t lm = __ballot(coop); lm; lm &= lm - 1) {
                    const int qq = (int)__builtin_ctzll(lm);
                    const uint32_t a = lane_val(op[q], qq), e = a + lane_val(L, qq) - 1;
                    for (uint32_t g = (a >> 5) + lane; g <= e >> 5; g += 64) {
                        const uint32_t lo = g == a >> 5 ? a & 31 : 0, hi = g == e >> 5 ? e & 31 : 31;
                        const uint32_t m = hi - lo == 31 ? 0xFFFFFFFFu : ((1u << (hi - lo + 1)) - 1) << lo;
                        __hip_atomic_fetch_or(&done[g], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                if (!coop && L)
                    mark(op[q], L);
                pend[q] = on && ml[q] != 0;
            }
            {
                const bool on0 = op[0] < lim && lit[0] + ml[0] != 0, on1 = op[1] < lim && lit[1] + ml[1] != 0;
                const uint32_t e = max(on0 ? op[0] + lit[0] + ml[0] : 0u, on1 ? op[1] + lit[1] + ml[1] : 0u);
                const uint32_t we = wave_incl_max(e);
                if (lane == 63 && we)
                    atomicMax(&hi_end, we);
            }
            __syncthreads();
            for (uint32_t pass = 0;; pass++) {
                bool moved = false;
                for (int q = 0; q < 2; q++) {
                    const uint32_t mb = op[q] + lit[q], ov = off[q], m = ml[q];
                    bool rdy = false, tnt = false;
                    if (pend[q]) {
                        uint32_t a, len;
                        const bool before = src_range(mb, ov, m, a, len);
                        rdy = !len || all_set(done, a, len);
                        if (rdy) {
                            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                            tnt = before || (len && any_set(taint, a, len));
                        }
                    }
                    // tainted: short offsets and long matches with the
                    // wave's lanes a byte each, the others by their lane
                    const bool wide = rdy && tnt && (ov < 16 || m > 256);
                    for (uint64_t lm = __ballot(wide); lm; lm &= lm - 1) {
                        const int qq = (int)__builtin_ctzll(lm);
                        taint_wide(lane_val(mb, qq), lane_val(ov, qq), lane_val(m, qq));
                    }
                    if (rdy && tnt && !wide)
                        taint_copy(mb, ov, m);
                    if (rdy && !tnt)
                        copy_match(mb, ov, m);
                    if (rdy) {
                        if (tnt)
                            atomicAdd(&ntm, 1u);
                        mark(mb, m);
                        pend[q] = false;
                        moved = true;
                    }
                }
                if (!__any(pend[0] || pend[1]) || pass > (1u << 22))
                    break;
                if (!__any(moved))
                    __builtin_amdgcn_s_sleep(1);
            }
            __syncthreads();
            P += tot[0] + tot[1];
        }
    }
    __syncthreads();
    const uint32_t nt = ntm;
    ZSK_KT(1)

    // ---- phase B: the block's bytes [0, E) out at once (the tainted ones
    // holding origins yet): a byte head to 16-byte alignment, whole 16-byte
    // stores, a byte tail; its taint bits and (with tainted bytes) its
    // origins to the job's scratch; then published ----
    const uint32_t E = min(hi_end, lim);
    uint8_t *o = out + d.d_off + bop;
    const uint32_t head = min(E, (uint32_t)((16 - ((uintptr_t)o & 15)) & 15));
    const uint32_t nchunks = (E - head) / 16, tail0 = head + 16 * nchunks;
    if (t < head)
        o[t] = ob[kBWin + t];
    for (uint32_t c = t; c < nchunks; c += kFT)
        *reinterpret_cast<u32x4 *>(o + head + 16 * c) = lds16(B + head + 16 * c);
    if (tail0 + t < E)
        o[tail0 + t] = ob[kBWin + tail0 + t];
    for (uint32_t i = t; i < kBWin / 32; i += kFT)
        btaint[(size_t)j * (kBWin / 32) + i] = taint[i];
    if (nt) {
        // origin of byte x as one u16 (low byte from the block plane, high
        // from the plane below it), 16 bytes a thread a step
        u32x4 *og = reinterpret_cast<u32x4 *>(borg + (size_t)j * kBWin);
        for (uint32_t c = t; c < kBWin / 16; c += kFT) {
            if (!((taint[c >> 1] >> (16 * (c & 1))) & 0xFFFF))
                continue;   // (no tainted byte: no origin read)
            const u32x4 lo = lds16(B + 16 * c), hi = lds16(ob0 + 16 * c);
            const uint32_t l[4] = {lo.x, lo.y, lo.z, lo.w}, h[4] = {hi.x, hi.y, hi.z, hi.w};
            uint32_t w[8];
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                w[2 * i] = (l[i] & 0xFF) | (h[i] & 0xFF) << 8 | (l[i] & 0xFF00) << 8 | (h[i] & 0xFF00) << 16;
                w[2 * i + 1] = (l[i] >> 16 & 0xFF) | (h[i] >> 16 & 0xFF) << 8 | (l[i] >> 24) << 16 |
                               (h[i] >> 24) << 24;
            }
            og[2 * c] = u32x4{w[0], w[1], w[2], w[3]};
            og[2 * c + 1] = u32x4{w[4], w[5], w[6], w[7]};
        }
    }
    publish();
    ZSK_KT(2)
    if (nt) {
        // the tainted bytes split evenly: ranks [r0, r1) a thread, over the
        // taint words' prefix counts (in done[], dead now)
        const uint32_t c0 = __builtin_popcount(taint[2 * t]), c1 = __builtin_popcount(taint[2 * t + 1]);
        uint32_t T;
        const uint32_t pre = scan(c0 + c1, T);
        done[2 * t] = pre;
        done[2 * t + 1] = pre + c0;
        __syncthreads();
        const uint32_t r0 = (uint32_t)((uint64_t)T * t / kFT), r1 = (uint32_t)((uint64_t)T * (t + 1) / kFT);
        // the next kG ranks' bytes and origins: rank r's word the last w
        // with done[w] <= r (kG interleaved binary searches), its bit the
        // (r - done[w])-th set one (a select by halves)
        constexpr uint32_t kG = 8;
        uint32_t xs[kG], og[kG];
        auto collect = [&](uint32_t r) {
            uint32_t wk[kG];
#pragma unroll
            for (uint32_t k = 0; k < kG; k++)
                wk[k] = 0;
            for (uint32_t st = kBWin / 64; st; st >>= 1) {
#pragma unroll
                for (uint32_t k = 0; k < kG; k++)
                    if (r + k < r1 && done[wk[k] + st] <= r + k)
                        wk[k] += st;
            }
#pragma unroll
            for (uint32_t k = 0; k < kG; k++) {
                xs[k] = ~0u;
                og[k] = 0;
                if (r + k < r1) {
                    const uint32_t m = taint[wk[k]];
                    uint32_t nb = r + k - done[wk[k]], pos = 0;
                    for (uint32_t h = 16; h; h >>= 1) {
                        const uint32_t c = __builtin_popcount((m >> pos) & ((1u << h) - 1));
                        if (c <= nb) {
                            nb -= c;
                            pos += h;
                        }
                    }
                    const uint32_t x = 32 * wk[k] + pos;
                    xs[k] = x;
                    og[k] = *lp<uint8_t>(B + x) | (uint32_t)*lp<uint8_t>(ob0 + x) << 8;
                }
            }
        };
        collect(r0);
        // every earlier block of the frame published (they finish phase A
        // about together): a thread a block
        if (t < j - j0) {
            uint32_t k = 0;
            while (__hip_atomic_load(&jres[j0 + t].pad, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0 &&
                   k++ < (1u << 24))
                __builtin_amdgcn_s_sleep(2);
        }
        __syncthreads();
        ZSK_KT(3)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        // each tainted byte followed back block by block: at (block cb,
        // position p) an untainted byte is the value, a tainted one sends it
        // on to its origin in block cb - 1 (the taint word, the origin and the
        // byte loaded together: one round trip a hop)
        const uint8_t *fo = out + d.d_off;
        for (uint32_t r = r0; r < r1;) {
            uint32_t cb[kG], val[kG];
            bool pend[kG];
#pragma unroll
            for (uint32_t k = 0; k < kG; k++) {
                cb[k] = j - 1;
                val[k] = 0;
                pend[k] = xs[k] != ~0u;
            }
            for (uint32_t hop = 0; hop <= j - j0; hop++) {
                bool any = false;
                uint32_t tw[kG], o2[kG], v[kG];
#pragma unroll
                for (uint32_t k = 0; k < kG; k++) {
                    if (pend[k]) {
                        const uint32_t p = og[k], b = cb[k];
                        tw[k] = btaint[(size_t)b * (kBWin / 32) + (p >> 5)];
                        o2[k] = borg[(size_t)b * kBWin + p];
                        v[k] = fo[(size_t)bop - (size_t)(j - b) * kBWin + p];
                    }
                }
#pragma unroll
                for (uint32_t k = 0; k < kG; k++) {
                    if (pend[k]) {
                        if (!((tw[k] >> (og[k] & 31)) & 1)) {
                            val[k] = v[k];
                            pend[k] = false;
                        } else if (cb[k] == j0) {
                            pend[k] = false;   // (cannot happen: nothing reaches before a frame)
                        } else {
                            og[k] = o2[k];
                            cb[k]--;
                            any = true;
                        }
                    }
                }
                if (!any)
                    break;
            }
#pragma unroll
            for (uint32_t k = 0; k < kG; k++)
                if (xs[k] < E)
                    o[xs[k]] = (uint8_t)val[k];
            r += kG;
            if (r < r1)
                collect(r);
        }
        ZSK_KT(4)
    }
    ZSK_KT(5)
#ifdef ZSK_TUNING
    if (t == 0 && j < 64) {
        uint32_t pc = 0;
        for (uint32_t i = 0; i < kBWin / 32; i++)
            pc += __builtin_popcount(taint[i]);
        g_ktime[j][8] = nt;
        g_ktime[j][9] = pc;
    }
#endif
}

}   // namespace

#ifdef ZSK_TUNING
int launch_seq_exec_variant(int version, const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                            uint8_t *d_out, const uint64_t *rec_base, const uint64_t *items, const uint32_t *nitems,
                            const int32_t *d_status, hipStream_t stream, uint32_t stop_last, uint32_t min_dsize);
#endif

// version: 0 = the production kernel; tuning builds time the diagnostic
// variants of seq_exec_tune.hip through it (launch_seq_exec_variant).
int launch_seq_exec(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                    uint8_t *d_out, const uint64_t *rec_base, const uint64_t *items,
                    const uint32_t *nitems, const int32_t *d_status, hipStream_t stream,
                    int version, const SplitScratch *blk, uint32_t stop_last, uint32_t min_dsize)
{
    if (nframes == 0)
        return 0;
    if (blk)   // the block route (production kernel only)
        return launch_seq_exec_seg(d_desc, nframes, d_comp, d_out, rec_base, items, nitems, d_status, stream, blk);
#ifdef ZSK_TUNING
    if (version != 0)
        return launch_seq_exec_variant(version, d_desc, nframes, d_comp, d_out, rec_base, items, nitems, d_status,
                                       stream, stop_last, min_dsize);
#else
    (void)version;
#endif
    hipLaunchKernelGGL((seq_exec_kernel<kExecStage, false>), dim3((nframes + kXW - 1) / kXW), dim3(64 * kXW), 0,
                       stream, d_desc, nframes, d_comp, d_out, rec_base, items, nitems, d_status, nullptr, nullptr,
                       nullptr, nullptr, nullptr, stop_last, min_dsize);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_seq_exec_frames(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
                           const uint64_t *rec_base, const uint64_t *items, const uint32_t *nitems,
                           int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream, uint32_t stop_last,
                           bool handoff, const uint8_t *lit, const HostPost *post)
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
    // (post: one frame, host-checked; its hand-off decoded here)
    const HostPost hp = post && nframes == 1 && handoff && !lit ? *post : HostPost{};
    hipLaunchKernelGGL(seq_exec_frame_kernel, dim3(nframes), dim3(kFT), 0, stream, d_desc, nframes, d_comp, d_out,
                       rec_base, items, nitems, d_status, d_fail_at, stop_last, handoff && !lit ? 1u : 0u, lit, hp);
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

int launch_seq_exec_big(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
                        const uint64_t *rec_base, const uint64_t *items, const uint32_t *nitems,
                        int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream, uint32_t stop_last,
                        bool handoff, const SplitScratch *blk, uint32_t skip_jobs)
{
    if (nframes == 0)
        return 0;
    hipLaunchKernelGGL(seq_exec_big_kernel, dim3(nframes), dim3(kFT), 0, stream, d_desc, nframes, d_comp, d_out,
                       rec_base, items, nitems, d_status, d_fail_at, stop_last, handoff ? 1u : 0u,
                       blk ? blk->bfirst : nullptr, blk ? blk->bcount : nullptr, blk ? blk->jobs : nullptr,
                       blk ? blk->jres : nullptr, skip_jobs);
#ifdef ZSK_TUNING
    // ZSEEK_BIG_TIMERS: accumulate the phase cycles, print every 100 launches
    static const bool timers = getenv("ZSEEK_BIG_TIMERS") != nullptr;
    static int calls = 0;
    if (timers && ++calls % 100 == 0) {
        unsigned long long z[9] = {0};
        (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_btime), sizeof(z), 0, hipMemcpyDeviceToHost, stream);
        (void)hipStreamSynchronize(stream);
        const double fr = z[8] ? (double)z[8] : 1.0;
        fprintf(stderr,
                "big execute cycles per frame: init %.0f items+scan %.0f cut+literals %.0f matches %.0f slides %.0f "
                "output %.0f | slides %.2f batches %.2f (%llu frames)\n",
                z[0] / fr, z[1] / fr, z[2] / fr, z[3] / fr, z[4] / fr, z[5] / fr, z[6] / fr, z[7] / fr, z[8]);
    }
#endif
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_seq_exec_blocks(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
                           const uint64_t *rec_base, const uint64_t *items, hipStream_t stream, uint32_t stop_last,
                           const SplitScratch *blk, uint32_t jobs)
{
    if (nframes == 0 || jobs == 0)
        return 0;
    hipLaunchKernelGGL(seq_exec_blocks_kernel, dim3(jobs), dim3(kFT), 0, stream, d_desc, nframes, d_comp, d_out,
                       rec_base, items, blk->bfirst, blk->jobs, blk->jres, blk->njobs, stop_last, blk->borg,
                       blk->btaint, blk->bcount, blk->borg_cap);
#ifdef ZSK_TUNING
    // ZSEEK_BLK_TIMERS: every 100th launch, each job's timeline in µs from the
    // first job's start
    static const bool timers = getenv("ZSEEK_BLK_TIMERS") != nullptr;
    static int calls = 0;
    if (timers && ++calls % 100 == 0) {
        static unsigned long long z[64][10];
        (void)hipStreamSynchronize(stream);
        (void)hipMemcpyFromSymbol(z, HIP_SYMBOL(g_ktime), sizeof(z), 0, hipMemcpyDeviceToHost);
        const unsigned long long t0 = z[0][0];
        for (uint32_t k = 0; k < jobs && k < 64; k++)
            fprintf(stderr,
                    "blk %2u: start %6.2f A %6.2f published %6.2f wait %6.2f resolved %6.2f end %6.2f us | tainted matches "
                    "%llu bytes %llu\n",
                    k, (double)(long long)(z[k][0] - t0) / 100.0, (double)(long long)(z[k][1] - t0) / 100.0,
                    (double)(long long)(z[k][2] - t0) / 100.0, (double)(long long)(z[k][3] - t0) / 100.0,
                    (double)(long long)(z[k][4] - t0) / 100.0, (double)(long long)(z[k][5] - t0) / 100.0, z[k][8],
                    z[k][9]);
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
                           d_out, rec_base, items, nitems, d_status, nullptr, stop_last, 0u, lit, HostPost{});
        if (max_dsize <= kFMax)
            return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    hipLaunchKernelGGL((seq_exec_kernel<4096, false>), dim3((nframes + kXW - 1) / kXW), dim3(64 * kXW), 0,
                       stream, d_desc, nframes, nullptr, d_out, rec_base, items, nitems, d_status, lit, nullptr,
                       nullptr, nullptr, nullptr, stop_last, one ? kFMax + 1 : 0u);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk
