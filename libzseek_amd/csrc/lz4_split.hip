// lz4_split.hip — the two-phase LZ4-frame decoder's launcher (gfx950).
//
// Replaces the per-frame liblz4 call of the reference hot path
// (/root/reference/src/decompress.c:752-773, LZ4F_decompress in a loop) with
// one stream-ordered sequence of launches over every frame a zseek_pread
// range covers:
//
//   plan     lz4_plan_direct_kernel (lane per frame): each frame's slots in
//            the item scratch, straight from its compressed offset; frames out
//            of file order fall back to a scan by its last workgroup;
//   parse    ONE LANE PER FRAME for 64 KiB-class frames (lz4_lean.hip,
//            lz4_scan.hip for short frames) or ONE WAVE PER FRAME for big
//            frames and small batches (lz4_chunk.hip): the serial token chain
//            with liblz4 1.9.3's validation, one 8-byte item per sequence;
//   execute  ONE WAVE PER FRAME (seq_exec.hip): items in batches of 64, output
//            staged in LDS and written as whole aligned 16-byte chunks;
//   hand-off frames the parse declined (block / content checksums, zero
//            offsets, item overflow) go to the wave-per-frame decoder
//            (lz4_wave.hip), which checks XXH32 as it decodes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <map>
#include <mutex>
#include <utility>
#include <vector>
#include <vector>

#include "lz4_dev.h"
#include "pool.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4d;

// ---- block route plan ---------------------------------------------------------
// Lane per frame: a frame of > 64 KiB decoded and >= min_csize compressed
// bytes whose header passes every check lz4_lean_kernel's hdr_status makes
// (no checksum flags; content size, when present, equal to the seek table's
// dSize) and whose block headers chain to an end mark at exactly c_size, with
// at most kMaxBlockJobs blocks and a dSize those blocks can hold, gets one job
// per block (reserved with one atomic, written in block order).  Every other
// frame keeps kNoJob and the chunk parse decodes it as before; a reservation
// past the job slots marks the slots it got as no job.
__device__ __forceinline__ uint32_t xxh32_short(const uint8_t *c, uint32_t p, uint32_t n)
{
    uint32_t acc = 0x165667B1u + n, i = 0;
    for (; i + 4 <= n; i += 4) {
        const uint32_t w = c[p + i] | c[p + i + 1] << 8 | c[p + i + 2] << 16 | (uint32_t)c[p + i + 3] << 24;
        acc += w * 0xC2B2AE3Du;
        acc = ((acc << 17) | (acc >> 15)) * 0x27D4EB2Fu;
    }
    for (; i < n; i++) {
        acc += c[p + i] * 0x165667B1u;
        acc = ((acc << 11) | (acc >> 21)) * 0x9E3779B1u;
    }
    acc ^= acc >> 15;
    acc *= 0x85EBCA77u;
    acc ^= acc >> 13;
    acc *= 0xC2B2AE3Du;
    acc ^= acc >> 16;
    return acc;
}

struct BlockPlanArgs {
    const uint8_t *comp;
    uint32_t min_csize;
    uint32_t *bfirst, *bcount, *njobs;
    BlockJob *jobs;
    uint32_t jobs_cap, max_bsid;
};

__device__ void block_plan_frame(uint32_t f, const FrameDesc *__restrict__ desc, const BlockPlanArgs &A)
{
    const uint8_t *__restrict__ comp = A.comp;
    uint32_t *__restrict__ bfirst = A.bfirst, *__restrict__ bcount = A.bcount, *__restrict__ njobs = A.njobs;
    BlockJob *__restrict__ jobs = A.jobs;
    const uint32_t min_csize = A.min_csize, jobs_cap = A.jobs_cap, max_bsid = A.max_bsid;
    const FrameDesc d = desc[f];
    bfirst[f] = kNoJob;
    bcount[f] = 0;
    const uint32_t clen = d.c_size;
    if (d.d_size <= 65536 || clen < min_csize || clen < 15 || clen > 0x3FFFFFFFu)   // item positions: 30 bits
        return;
    const uint8_t *c = comp + d.c_off;
    auto r32 = [&](uint32_t p) -> uint32_t {
        return c[p] | c[p + 1] << 8 | c[p + 2] << 16 | (uint32_t)c[p + 3] << 24;
    };
    if (r32(0) != kLz4Magic)
        return;
    const uint32_t flg = c[4], bd = c[5];
    if ((flg & 0xC0) != 0x40 || (flg & 0x16) || (bd & 0x8F) || ((bd >> 4) & 7) < 4 || ((bd >> 4) & 7) > max_bsid)
        return;
    const uint32_t csz = (flg >> 3) & 1, dictid = flg & 1;
    const uint32_t hdr = 7 + 8 * csz + 4 * dictid;
    if (clen < hdr + 4 || ((xxh32_short(c, 4, hdr - 5) >> 8) & 0xFF) != c[hdr - 1])
        return;
    if (csz && (r32(6) != d.d_size || r32(10) != 0))
        return;
    const uint32_t bsid = (bd >> 4) & 7, max_block = 1u << (8 + 2 * bsid);
    uint32_t p = hdr, nb = 0;
    for (;;) {
        if (clen - p < 4)
            return;
        const uint32_t h = r32(p);
        if (h == 0) {
            if (clen - p != 4)
                return;
            break;
        }
        const uint32_t sz = h & 0x7FFFFFFFu;
        if (sz == 0 || sz > max_block || sz > clen - p - 8 || ++nb > kMaxBlockJobs)
            return;
        p += 4 + sz;
    }
    if ((uint64_t)(nb - 1) * max_block >= d.d_size || (uint64_t)nb * max_block < d.d_size)
        return;
    const uint32_t base = atomicAdd(njobs, nb);
    if (base >= jobs_cap || nb > jobs_cap - base) {
        for (uint32_t i = base; i < jobs_cap && i - base < nb; i++)
            jobs[i].f = kNoJob;
        return;
    }
    const uint32_t info = bsid | ((flg >> 5) & 1) << 8;
    p = hdr;
    for (uint32_t j = 0; j < nb; j++) {
        const uint32_t q = p + 4 + (r32(p) & 0x7FFFFFFFu);
        const uint32_t so = j ? (p >> 3) & ~3u : 0;
        const uint32_t se = j + 1 < nb ? (q >> 3) & ~3u : slots_of(clen);
        jobs[base + j] = BlockJob{f, p, q, so, se - so, info, j * max_block, 0};
        p = q;
    }
    bfirst[f] = base;
    bcount[f] = nb;
}

__global__ __launch_bounds__(256) void lz4_block_plan_kernel(const FrameDesc *__restrict__ desc, uint32_t n,
                                                              BlockPlanArgs A)
{
    const uint32_t f = blockIdx.x * 256 + threadIdx.x;
    if (f < n)
        block_plan_frame(f, desc, A);
}


// ---- plan: per-frame item slot offsets ------------------------------------
constexpr uint32_t kPlanGroups = 256;
// Slot offsets without a scan (the usual case): when the frames lie in order
// in the input (c_off[f+1] >= c_off[f] + c_size[f], as in every batch the
// reader builds), frame f's slots start at ceil4((c_off[f] - c_off[0]) / 8 +
// 40 f), and the gap to frame f+1 is >= c_size/8 + 37 > slots_of(c_size).  A
// frame out of order sets redo[0]; the workgroup that finishes last (redo[1]
// counts finished workgroups) then lays the slots out by a scan of
// slots_of(c_size) instead, and clears both words for the next launch on this
// scratch (zeroed at allocation).  Round 3 ran the scan as its own launch
// behind a flag memset: two launches that did nothing in the usual batch.
__global__ __launch_bounds__(256) void lz4_plan_direct_kernel(const FrameDesc *__restrict__ desc,
                                                               uint32_t n, uint64_t *__restrict__ rec_base,
                                                               uint64_t *__restrict__ total,
                                                               uint32_t *__restrict__ redo,
                                                               int32_t *__restrict__ status,
                                                               uint32_t *__restrict__ fail_at,
                                                               BlockPlanArgs bp)
{
    __shared__ uint64_t part[256];
    __shared__ uint32_t last;
    // the block plan's job count zeroed (bp.njobs): the block plan runs next,
    // or -- one workgroup and bp.bfirst set -- here, a lane per frame, behind
    // a barrier (one launch less: a small batch's block plan is one lane's
    // walk over a frame's block headers)
    if (bp.njobs && blockIdx.x == 0 && threadIdx.x == 0)
        *bp.njobs = 0;
    if (bp.bfirst && gridDim.x == 1) {
        __syncthreads();
        for (uint32_t f = threadIdx.x; f < n; f += 256)
            block_plan_frame(f, desc, bp);
    }
    // at most kPlanGroups workgroups (the finish counter is one atomic per
    // workgroup: 4,096 of them cost 0.11 ms at 1,048,576 frames), each thread
    // striding over its frames
    const uint64_t c0 = desc[0].c_off;
    for (uint32_t f = blockIdx.x * 256 + threadIdx.x; f < n; f += gridDim.x * 256) {
        // every frame starts as not run (a parse kernel then owns it), with no
        // failing block: the reader needs no fills of its own
        status[f] = ST_NOT_RUN;
        if (fail_at)
            fail_at[f] = 0;
        const FrameDesc d = desc[f];
        const uint64_t r = (((d.c_off - c0) >> 3) + 40ull * f + 3) & ~3ull;
        rec_base[f] = r;
        if (d.c_off < c0 || (f + 1 < n && desc[f + 1].c_off < d.c_off + d.c_size))
            atomicOr(&redo[0], 1u);
        if (f + 1 == n)
            *total = r + slots_of(d.c_size);
    }
    if (n == 1)   // one frame is always in order
        return;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(&redo[1], 1u) == gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (!last)
        return;
    __threadfence();
    if (atomicOr(&redo[0], 0u)) {
        const uint32_t t = threadIdx.x;
        const uint32_t chunk = (n + 255) / 256;
        const uint32_t i0 = t * chunk < n ? t * chunk : n;
        const uint32_t i1 = i0 + chunk < n ? i0 + chunk : n;
        uint64_t sum = 0;
        for (uint32_t i = i0; i < i1; i++)
            sum += slots_of(desc[i].c_size);
        part[t] = sum;
        __syncthreads();
        for (uint32_t k = 1; k < 256; k <<= 1) {
            const uint64_t v = t >= k ? part[t - k] : 0;
            __syncthreads();
            part[t] += v;
            __syncthreads();
        }
        uint64_t run = part[t] - sum;
        for (uint32_t i = i0; i < i1; i++) {
            rec_base[i] = run;
            run += slots_of(desc[i].c_size);
        }
        if (t == 255)
            *total = part[t];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        redo[0] = 0;
        redo[1] = 0;
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
    if (s->bfirst)
        (void)hipFree(s->bfirst);
    if (s->bcount)
        (void)hipFree(s->bcount);
    if (s->njobs)
        (void)hipFree(s->njobs);
    if (s->jobs)
        (void)hipFree(s->jobs);
    if (s->jres)
        (void)hipFree(s->jres);
    if (s->borg)
        (void)hipFree(s->borg);
    if (s->btaint)
        (void)hipFree(s->btaint);
    *s = SplitScratch();
}

namespace {
// block route scratch for (frames, jobs); stream-ordered like the rest
int block_scratch_reserve(SplitScratch *s, uint32_t frames, uint32_t jobs, hipStream_t stream)
{
    if (!s->njobs && hipMalloc((void **)&s->njobs, sizeof(uint32_t)) != hipSuccess)
        return -1;
    if (frames > s->bframes_cap) {
        const uint32_t cap = frames < 1024 ? 1024 : frames;
        (void)hipStreamSynchronize(stream);
        if (s->bfirst)
            (void)hipFree(s->bfirst);
        if (s->bcount)
            (void)hipFree(s->bcount);
        s->bfirst = s->bcount = nullptr;
        s->bframes_cap = 0;
        if (hipMalloc((void **)&s->bfirst, (size_t)cap * 4) != hipSuccess ||
            hipMalloc((void **)&s->bcount, (size_t)cap * 4) != hipSuccess)
            return -1;
        s->bframes_cap = cap;
    }
    if (jobs > s->jobs_cap) {
        (void)hipStreamSynchronize(stream);
        if (s->jobs)
            (void)hipFree(s->jobs);
        if (s->jres)
            (void)hipFree(s->jres);
        s->jobs = nullptr;
        s->jres = nullptr;
        s->jobs_cap = 0;
        if (hipMalloc((void **)&s->jobs, (size_t)jobs * sizeof(BlockJob)) != hipSuccess ||
            hipMalloc((void **)&s->jres, (size_t)jobs * sizeof(BlockRes)) != hipSuccess)
            return -1;
        s->jobs_cap = jobs;
    }
    return 0;
}

// the block-parallel execute's scratch for `jobs` jobs (136 KiB each)
constexpr uint32_t kOriginJobsMax = 1024;
int origin_scratch_reserve(SplitScratch *s, uint32_t jobs, hipStream_t stream)
{
    if (jobs <= s->borg_cap)
        return 0;
    (void)hipStreamSynchronize(stream);
    if (s->borg)
        (void)hipFree(s->borg);
    if (s->btaint)
        (void)hipFree(s->btaint);
    s->borg = nullptr;
    s->btaint = nullptr;
    s->borg_cap = 0;
    const uint32_t cap = jobs < 16 ? 16 : jobs;
    if (hipMalloc((void **)&s->borg, (size_t)cap * 65536 * sizeof(uint16_t)) != hipSuccess ||
        hipMalloc((void **)&s->btaint, (size_t)cap * 2048 * sizeof(uint32_t)) != hipSuccess)
        return -1;
    s->borg_cap = cap;
    return 0;
}

// The block route for a batch: on (AUTO) for >= 1024 frames and < 32768 --
// the batches whose big frames take the chunk parse (config 3: 4,096 frames
// of 1 MiB, 16 blocks each) -- with frames of >= chunk_min compressed bytes,
// used on the device only when >= 16,384 jobs were planned (fewer leave the
// lean parse's lanes idle and the chunk parse wins); ROUTE_BLOCK forces it
// for every frame and any job count.
struct BlockRoute {
    bool on;
    uint32_t min_csize, min_jobs;
};
// Env ZSEEK_BLOCK_ROUTE=0 turns the automatic choice off (A/B runs).
BlockRoute block_route(uint32_t nframes, int route, const ParseRoute &r)
{
    static const bool off = [] {
        const char *v = getenv("ZSEEK_BLOCK_ROUTE");
        return v && !strcmp(v, "0");
    }();
    if (route == ROUTE_BLOCK)
        return {true, 0, 1};
    if (off || route != ROUTE_AUTO || nframes < 1024 || nframes >= 32768 || r.chunk_min == 0xFFFFFFFFu)
        return {false, 0, 0};
    return {true, r.chunk_min, 16384};
}
constexpr uint32_t kJobsCapMax = 1u << 21;

// The one-frame route: batches of a few frames -- a cached
// reader's single-frame miss, a request's first batch -- where one frame's
// serial chain is the whole launch: each frame's chunk parse reads it staged
// in LDS, one frame per workgroup.  Env
// ZSEEK_ONE_ROUTE=0 turns the automatic choice off (A/B runs); ZSEEK_PARSE
// forcing a parse keeps it off too.
bool one_route(uint32_t nframes, int route)
{
    static const bool off = [] {
        const char *v = getenv("ZSEEK_ONE_ROUTE");
        return (v && !strcmp(v, "0")) || getenv("ZSEEK_PARSE") != nullptr;
    }();
    return route == ROUTE_ONE || (route == ROUTE_AUTO && !off && nframes <= kOneMaxFrames);
}
}   // namespace

int split_scratch_reserve(SplitScratch *s, uint32_t frames, uint64_t items, hipStream_t stream)
{
    if (!s->total) {
        if (hipHostMalloc((void **)&s->total, sizeof(uint64_t), hipHostMallocMapped) != hipSuccess)
            return -1;
        *s->total = 0;
    }
    if (!s->redo) {   // [out-of-order flag, plan workgroups done]: zero between launches
        if (hipMalloc((void **)&s->redo, 2 * sizeof(uint32_t)) != hipSuccess)
            return -1;
        if (hipMemsetAsync(s->redo, 0, 2 * sizeof(uint32_t), stream) != hipSuccess) {
            (void)hipFree(s->redo);
            s->redo = nullptr;
            return -1;
        }
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
        if (hipMalloc((void **)&s->items, cap * 8 + 64) != hipSuccess)
            return -1;
        s->items_cap = cap;
    }
    return 0;
}

// ---- per-stage launch timing (zsk_kernel_timing / zsk_kernel_times) ----------
// Events around the stages of each launch on its stream: [plan, parse,
// execute, hand-off]; zstd launches add spans around their per-chunk kernels
// on the streams those run on (kernel_span_begin / _end; summed per launch in
// slots kTimedStages..).  Read back on request as the MEDIAN over the launches
// recorded (a warm-up or a straggler does not move it).
namespace {
struct Span3 {
    int slot;
    hipEvent_t a, b;
};
struct Pend {
    std::array<hipEvent_t, kTimedStages + 1> ev;
    std::vector<Span3> spans;
};
struct StageTimer {
    std::mutex mu;
    bool on = false;
    std::vector<hipEvent_t> pool;
    std::vector<Pend> pend;
    std::vector<std::array<double, kTimedSlots>> rec;   // per launch
};
StageTimer g_timer;
thread_local Pend t_pend;
thread_local bool t_active = false;

hipEvent_t timer_event()   // (g_timer.mu held)
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

void timer_release(Pend &p)   // (g_timer.mu held)
{
    for (auto e : p.ev)
        g_timer.pool.push_back(e);
    for (auto &x : p.spans) {
        g_timer.pool.push_back(x.a);
        g_timer.pool.push_back(x.b);
    }
}

void timer_collect()   // (g_timer.mu held) pending launches -> records
{
    for (auto &p : g_timer.pend) {
        (void)hipEventSynchronize(p.ev[kTimedStages]);
        std::array<double, kTimedSlots> r{};
        for (int i = 0; i < kTimedStages; i++) {
            float t = 0;
            if (hipEventElapsedTime(&t, p.ev[i], p.ev[i + 1]) == hipSuccess)
                r[i] = t;
        }
        for (auto &x : p.spans) {
            float t = 0;
            (void)hipEventSynchronize(x.b);
            if (hipEventElapsedTime(&t, x.a, x.b) == hipSuccess)
                r[x.slot] += t;
        }
        g_timer.rec.push_back(r);
        timer_release(p);
    }
    g_timer.pend.clear();
}
}   // namespace

void stage_mark(int boundary, hipStream_t stream)
{
    if (boundary == 0) {
        std::lock_guard<std::mutex> g(g_timer.mu);
        t_active = g_timer.on;
        if (!t_active)
            return;
        for (auto &e : t_pend.ev)
            e = timer_event();
        t_pend.spans.clear();
    }
    if (!t_active)
        return;
    (void)hipEventRecord(t_pend.ev[boundary], stream);
    if (boundary == kTimedStages) {
        std::lock_guard<std::mutex> g(g_timer.mu);
        g_timer.pend.push_back(t_pend);
        t_pend.spans.clear();
        t_active = false;
    }
}

hipEvent_t kernel_span_begin(hipStream_t stream)
{
    if (!t_active)
        return nullptr;
    hipEvent_t e;
    {
        std::lock_guard<std::mutex> g(g_timer.mu);
        e = timer_event();
    }
    (void)hipEventRecord(e, stream);
    return e;
}

void kernel_span_end(int slot, hipEvent_t begin, hipStream_t stream)
{
    if (!t_active || !begin || slot < kTimedStages || slot >= kTimedSlots)
        return;
    hipEvent_t e;
    {
        std::lock_guard<std::mutex> g(g_timer.mu);
        e = timer_event();
    }
    (void)hipEventRecord(e, stream);
    t_pend.spans.push_back({slot, begin, e});
}

int kernel_timing(int on)
{
    std::lock_guard<std::mutex> g(g_timer.mu);
    for (auto &p : g_timer.pend) {
        (void)hipEventSynchronize(p.ev[kTimedStages]);
        for (auto &x : p.spans)
            (void)hipEventSynchronize(x.b);
        timer_release(p);
    }
    g_timer.pend.clear();
    g_timer.rec.clear();
    g_timer.on = on != 0;
    return 0;
}

int kernel_times(double *ms, int cap)
{
    std::lock_guard<std::mutex> g(g_timer.mu);
    timer_collect();
    const size_t n = g_timer.rec.size();
    for (int i = 0; i < cap && i < kTimedSlots; i++) {
        std::vector<double> v;
        for (auto &r : g_timer.rec)
            v.push_back(r[i]);
        std::sort(v.begin(), v.end());
        ms[i] = n == 0 ? 0.0 : (n & 1) ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
    }
    return (int)n;
}

ParseRoute parse_route(uint32_t nframes, int route)
{
    switch (route) {
    case ROUTE_LEAN: return {0xFFFFFFFFu, 0};
    case ROUTE_SCAN: return {0xFFFFFFFFu, 0xFFFFFFFFu};
    case ROUTE_CHUNK:
    case ROUTE_BLOCK:
    case ROUTE_ONE: return {0, 0};
    default: break;
    }
    const uint32_t cmin = chunk_parse_min(nframes);
    return {cmin, cmin < kLeanMinCsize ? cmin : kLeanMinCsize};
}

const char *parse_kernel_name(uint32_t nframes, uint32_t c_size, int route)
{
    if (lz4_pick_engine(nframes) == ENGINE_WAVE && route == ROUTE_AUTO)
        return "lz4_wave_kernel";
    if (one_route(nframes, route))
        return "lz4_chunk_kernel (one-frame route)";
    const ParseRoute r = parse_route(nframes, route);
    // (block route: frames of > 64 KiB decoded; named for the compressed
    // sizes those frames have)
    const BlockRoute br = block_route(nframes, route, r);
    if (br.on && c_size >= br.min_csize && c_size >= 65536)
        return "lz4_lean_kernel (block route)";
    if (c_size >= r.chunk_min)
        return "lz4_chunk_kernel";
    return c_size >= r.lean_min ? "lz4_lean_kernel" : "lz4_scan_kernel";
}

int launch_lz4_split(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                     uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at,
                     hipStream_t stream, SplitScratch *s, int route, int stages, int tune, uint32_t stop_last,
                     uint32_t max_dsize, const HostPost *post, bool *posted, bool in_order)
{
    if (posted)
        *posted = false;
    if (nframes == 0)
        return 0;
    if (s->frames_cap < nframes || !s->rec_base || !s->redo)
        return -1;
    (void)hipGetLastError();   // a stale error of an earlier call is not this launch's
    uint64_t *total_dev = nullptr;
    (void)hipHostGetDevicePointer((void **)&total_dev, s->total, 0);
    const bool one = one_route(nframes, route);
    const ParseRoute r = one ? ParseRoute{0, 0} : parse_route(nframes, route);
    BlockRoute br = one ? BlockRoute{false, 0, 0} : block_route(nframes, route, r);
    const uint64_t jw = (uint64_t)nframes * kMaxBlockJobs;
    const uint32_t jlanes = (uint32_t)(jw < kJobsCapMax ? jw : kJobsCapMax);
    // the one-frame route's frames of > 64 KiB: their blocks
    // of <= 64 KiB get block-plan jobs, parsed a workgroup each
    // (launch_lz4_job_parse), and the windowed execute takes them
    // (launch_seq_exec_big); env ZSEEK_ONE_BIG=0: as round 5
    static const bool big_off = [] {
        const char *v = getenv("ZSEEK_ONE_BIG");
        return v && !strcmp(v, "0");
    }();
    bool big = one && max_dsize > 65536 && !big_off && ((tune >> 8) & 0xFFF) == 0;
    if (big)
        br = BlockRoute{true, 0, 1};
    if (br.on && block_scratch_reserve(s, nframes, jlanes, stream) != 0)
        br.on = big = false;   // no room: the chunk parse takes the frames as before
    // the accepted big frames block-parallel (their jobs: at most
    // ceil(max_dsize / 64 KiB) a frame; the device API's unknown sizes: the
    // job lanes, at most kOriginJobsMax -- a frame with a job past the scratch
    // goes through the window), the others through the window; env
    // ZSEEK_ONE_BLOCKS=0 (or no room for the origins): all through the window
    static const bool blocks_off = [] {
        const char *v = getenv("ZSEEK_ONE_BLOCKS");
        return v && !strcmp(v, "0");
    }();
    bool blocks = big && !blocks_off;
    if (blocks) {
        const uint64_t need = std::min<uint64_t>((uint64_t)nframes * (((uint64_t)max_dsize + 65535) / 65536),
                                                 std::min<uint64_t>(jlanes, kOriginJobsMax));
        blocks = origin_scratch_reserve(s, (uint32_t)need, stream) == 0;
    }
    SplitScratch *blk = br.on ? s : nullptr;
    stage_mark(0, stream);
    // one frame on the one-frame route: the chunk kernel does the plan's work
    // (frames in order: a lone frame, or the caller says so -- the reader's
    // batches are file order)
    const bool solo = one && (nframes == 1 || in_order) && (stages & 3) == 3 && !big;
    if ((stages & 1) && !solo) {
        const uint32_t pgroups = std::min<uint32_t>((nframes + 255) / 256, kPlanGroups);
        BlockPlanArgs bp{d_comp, br.min_csize, nullptr, nullptr, nullptr, nullptr, jlanes, big ? 4u : 7u};
        if (blk) {
            bp.bfirst = s->bfirst;
            bp.bcount = s->bcount;
            bp.njobs = s->njobs;
            bp.jobs = s->jobs;
        }
        // (one plan workgroup: the block plan inside it)
        BlockPlanArgs pbp = bp;
        if (pgroups != 1)
            pbp.bfirst = nullptr;
        hipLaunchKernelGGL(lz4_plan_direct_kernel, dim3(pgroups), dim3(256), 0, stream, d_desc, nframes, s->rec_base,
                           total_dev, s->redo, d_status, d_fail_at, pbp);
        if (blk && pgroups != 1)
            hipLaunchKernelGGL(lz4_block_plan_kernel, dim3((nframes + 255) / 256), dim3(256), 0, stream, d_desc,
                               nframes, bp);
    }
    stage_mark(1, stream);
    // parse: each kernel takes the frames of its compressed-size range and
    // skips the others (launched only when the range is not empty); block
    // route jobs before the chunk parse, which accepts or re-parses their
    // frames
    if (stages & 2) {
        if (big)
            launch_lz4_job_parse(d_desc, d_comp, s->rec_base, (uint64_t)s->items_cap, s->items, s, jlanes, stream);
        else if (blk)
            launch_lz4_lean_blocks(d_desc, d_comp, s->rec_base, (uint64_t)s->items_cap, s->items, s, jlanes,
                                   br.min_jobs, stream);
        if (r.chunk_min > r.lean_min)
            launch_lz4_lean(d_desc, nframes, d_comp, s->rec_base, (uint64_t)s->items_cap, s->items,
                            s->nitems, d_status, d_fail_at, stream, r.chunk_min, tune & 0xFF, r.lean_min);
        if (r.lean_min != 0)
            launch_lz4_scan(d_desc, nframes, d_comp, s->rec_base, (uint64_t)s->items_cap, s->items,
                            s->nitems, d_status, d_fail_at, stream, r.lean_min < r.chunk_min ? r.lean_min : r.chunk_min);
        if (r.chunk_min != 0xFFFFFFFFu)
            launch_lz4_chunk(d_desc, nframes, d_comp, s->rec_base, (uint64_t)s->items_cap, s->items,
                             s->nitems, d_status, d_fail_at, stream, r.chunk_min, blk, br.min_jobs, one,
                             solo ? total_dev : nullptr);
    }
    stage_mark(2, stream);
    bool frame_handoff = false;
    if (stages & 4) {
        // the one-frame route executes a frame of <= 64 KiB per workgroup
        // (env ZSEEK_ONE_EXEC=wave: the wave kernel, as round 3)
        static const bool wave_exec = [] {
            const char *v = getenv("ZSEEK_ONE_EXEC");
            return v && !strcmp(v, "wave");
        }();
        if (one && !wave_exec && ((tune >> 8) & 0xFFF) == 0) {
            // hand-offs of <= 64 KiB frames decoded inside (when the batch has
            // no bigger frame and the hand-off stage is asked for: no
            // hand-off launch below)
            frame_handoff = (stages & 8) && (max_dsize <= 65536 || big);
            // a lone frame posts its results to the host itself (no download)
            const bool post_here = post && frame_handoff && nframes == 1 && !big;
            if (!(big && nframes == 1))   // (a lone big frame: nothing for it)
                launch_seq_exec_frames(d_desc, nframes, d_comp, d_out, s->rec_base, s->items, s->nitems, d_status,
                                       d_fail_at, stream, stop_last, frame_handoff, nullptr,
                                       post_here ? post : nullptr);
            if (post_here && posted)
                *posted = true;
            if (blocks)
                launch_seq_exec_blocks(d_desc, nframes, d_comp, d_out, s->rec_base, s->items, stream, stop_last, s,
                                       jlanes);
            if (big)
                launch_seq_exec_big(d_desc, nframes, d_comp, d_out, s->rec_base, s->items, s->nitems, d_status,
                                    d_fail_at, stream, stop_last, frame_handoff, s, blocks ? s->borg_cap : 0u);
            else if (max_dsize > 65536)
                launch_seq_exec(d_desc, nframes, d_comp, d_out, s->rec_base, s->items, s->nitems, d_status, stream,
                                0, nullptr, stop_last, 65537);
        } else {
            launch_seq_exec(d_desc, nframes, d_comp, d_out, s->rec_base, s->items, s->nitems, d_status, stream,
                            (tune >> 8) & 0xFFF, blk, stop_last);
        }
    }
    stage_mark(3, stream);
    if (hipGetLastError() != hipSuccess) {
        // a plan cut short may leave its finish counter or out-of-order flag
        // set: the next plan on this scratch must start from zero
        (void)hipMemsetAsync(s->redo, 0, 2 * sizeof(uint32_t), stream);
        (void)hipGetLastError();
        stage_mark(4, stream);
        return -1;
    }
    int rc = 0;
    if ((stages & 8) && !frame_handoff)
        rc = launch_lz4_wave_deferred(d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream);
    stage_mark(4, stream);
    return rc;
}

// Public device API (zsk_lz4_decode_frames): the host does not see the
// descriptors, so scratch comes from a per-device pool and is sized before
// the plan runs: from the compressed bytes d_comp's allocation can hold past
// d_comp (hipMemGetAddressRange) -- the plan lays frames out at
// (c_off - c_off[0]) / 8 + 40 f, so span / 8 + 44 n + 64 slots always fit
// frames stored in file order in that span, whatever their size -- capped at
// what n frames of up to 4 MiB compressed can use (a caller's span may sit in
// a multi-GiB arena: a few frames must not reserve GiBs), else for 64 KiB
// frames; and never below the item total the previous plan on that set
// reported.  Frames that still do not fit go to the wave kernel and the
// next call grows.  (Round 3 sized a first call for 64 KiB frames only, so
// a first call over 1 MiB frames handed every frame to the wave kernel.)
// `route` (ROUTE_*) forces one production decoder for every frame (tests).
int launch_lz4_frames(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                      uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream,
                      int route, int tune)
{
    if (nframes == 0)
        return 0;
    if (route == ROUTE_WAVE || (route == ROUTE_AUTO && lz4_pick_engine(nframes) == ENGINE_WAVE))
        return launch_lz4_wave(d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream);
    static ScratchPool<SplitScratch> pool;
    SplitScratch *s = pool.acquire(stream);
    if (!s)
        return -1;
    uint64_t want = (uint64_t)nframes * slots_of(65536 + 64);
    if (want > (512ull << 20))
        want = 512ull << 20;
    hipDeviceptr_t base = 0;
    size_t bytes = 0;
    if (hipMemGetAddressRange(&base, &bytes, (hipDeviceptr_t)d_comp) == hipSuccess && bytes &&
        (uintptr_t)d_comp >= (uintptr_t)base && (uintptr_t)d_comp < (uintptr_t)base + bytes) {
        const uint64_t span = (uintptr_t)base + bytes - (uintptr_t)d_comp;
        uint64_t by_span = span / 8 + 44ull * nframes + 64;
        const uint64_t by_frames = (uint64_t)nframes * slots_of((4u << 20) + 64) + 64;
        if (by_span > by_frames)
            by_span = by_frames;
        if (by_span <= (1ull << 30))   // up to 8 GiB of items
            want = by_span;
    }
    (void)hipGetLastError();   // (a failed range query is not this launch's error)
    if (s->total && *s->total > want)
        want = *s->total;
    int rc;
    if (split_scratch_reserve(s, nframes, want, stream) != 0) {
        (void)hipGetLastError();   // the failed allocation is not the wave launch's error
        rc = launch_lz4_wave(d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream);
    }
    else
        rc = launch_lz4_split(d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream, s, route, 15, tune);
    pool.release(s, stream);
    return rc;
}

// Automatic choice: the two-phase decoder for every batch
// (its parse per frame size and batch size, chunk_parse_min: a single 64 KiB
// frame takes the wave-parallel chunk parse); the wave-per-frame kernel
// decodes only the frames the parse hands off.  Env ZSEEK_HIP_KERNEL=wave
// forces the wave kernel for every frame.
int lz4_pick_engine(uint32_t nframes)
{
    (void)nframes;
    const int e = lz4_engine();
    return e == ENGINE_WAVE ? ENGINE_WAVE : ENGINE_SPLIT;
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
        if (!strcmp(v, "split"))
            return (int)ENGINE_SPLIT;
        if (!strcmp(v, "wave"))
            return (int)ENGINE_WAVE;
        return (int)ENGINE_AUTO;
    }();
    return e;
}

const char *lz4_kernel_name(uint32_t nframes)
{
    return lz4_pick_engine(nframes) == ENGINE_SPLIT ? "seq_exec_kernel" : "lz4_wave_kernel";
}

}   // namespace zsk
