// reader.cpp — the zseek_reader_* / zseek_pread C API on top of the GPU
// batch decoder.
//
// Reference: /root/reference/src/decompress.c.  Open/close/stats/error
// conventions follow it line for line in behaviour (cited per function);
// the pread hot path is redesigned:
//
//   reference (decompress.c:377-804)       this file (pread_frames)
//   -------------------------------------  -------------------------------------
//   1 frame per call                        every frame covered by
//                                           [offset, offset+count) per call
//   1 user pread per frame                  1 user pread per batch (contiguous
//                                           compressed span, pinned staging)
//   LZ4F_decompress / ZSTD_decompress*      HIP kernels over the batch (LZ4:
//   on the CPU                              lz4_*.hip + seq_exec.hip; zstd:
//                                           zstd_decode.hip + seq_exec.hip)
//   serial                                  a pipeline of kSlots batches per
//                                           device: the user pread of batch
//                                           k+1, the upload / decode / download
//                                           of batch k and the copy of batch
//                                           k-1 into the caller's buffer overlap
//   one decoder                             the range split over the reader's
//                                           devices (ZSEEK_HIP_DEVICES), one
//                                           pipeline ("lane") per device
//   cache every decoded frame               cache the last cache_size frames of
//                                           the request (same final LRU state
//                                           as the reference's call loop)
//
// A corrupt frame inside a range makes the call return the bytes before it
// (a short read); the next call, starting at that frame, returns -1 with the
// error string the reference would produce — the same observable sequence a
// caller looping on the reference sees.
#include <errno.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <thread>
#include <utility>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../include/zseek_hip.h"
#include "host.h"
#include "lane_plan.h"
#include "pool.h"

using namespace zsk;

namespace {
constexpr uint32_t kZstdMagic = 0xFD2FB528u;   // ref decompress.c:22
constexpr uint32_t kLz4Magic = 0x184D2204u;    // ref decompress.c:23
constexpr size_t kDefaultBatch = 64u << 20;    // decoded bytes per batch
constexpr size_t kFirstBatch = 4u << 20;       // the first batch of a request (latency)
constexpr size_t kLaneMin = 1u << 20;          // decoded bytes per lane, at least
}   // namespace

struct zseek_reader {
    zseek_read_file_t user_file;
    zseek_compression_type_t type;
    // the reference's rwlock (decompress.c:38): shared for cache hits
    // (:699-706), exclusive for misses, no-cache reads and GPU batches
    // (:714-720); lru_lock orders the MRU promotion of concurrent hits (the
    // reference promotes under its read lock, cache.c:125)
    std::shared_mutex lock;
    std::mutex lru_lock;
    // zseek_reader_stats' changing fields, published under the exclusive
    // lock after every change, read without the reader lock: a stats call
    // never waits behind a multi-GiB GPU read (the reference takes its read
    // lock, :850-875, and waits at most one frame decode)
    std::atomic<size_t> snap_cache_memory{0}, snap_cached_frames{0}, snap_buffered{0};
    std::mutex io_lock;   // one user pread callback at a time (lanes run in threads)
    SeekTable st;
    FrameCache *cache = nullptr;   // NULL when cache_size == 0 (ref :219-227)
    std::mutex cursor_lock;        // zseek_read: cursor read, pread, advance as one step
    size_t pos = 0;                // zseek_read cursor (ref :826-835)
    size_t batch_bytes = kDefaultBatch;
    int io_threads = 1;    // > 1: the caller allows concurrent pread callbacks
    bool verify = false;   // check seek-table frame checksums (the reference never does)
    std::vector<int> devices;                       // lane i decodes on devices[i]
    std::vector<std::unique_ptr<DeviceCtx>> lanes;  // created at first use
};

// ---------------------------------------------------------------------------
// default FILE* I/O (ref decompress.c:47-98): save position, seek, read,
// restore — the caller's FILE position is left untouched.
// ---------------------------------------------------------------------------
static ssize_t default_pread(void *data, size_t size, size_t offset, void *user_data,
                             void *call_data)
{
    (void)call_data;
    FILE *f = (FILE *)user_data;
    long prev = ftell(f);
    if (prev == -1)
        return -1;
    if (fseeko(f, (off_t)offset, SEEK_SET) == -1)
        return -1;
    size_t got = fread(data, 1, size, f);
    if (got != size && ferror(f))
        return -1;
    if (fseek(f, prev, SEEK_SET) == -1)
        return -1;
    return (ssize_t)got;
}

static ssize_t default_fsize(void *user_data, void *call_data)
{
    (void)call_data;
    int fd = fileno((FILE *)user_data);
    if (fd == -1)
        return -1;
    struct stat sb;
    if (fstat(fd, &sb) == -1)
        return -1;
    return sb.st_size;
}

// ---------------------------------------------------------------------------
// open / close (ref decompress.c:100-295, 297-375)
// ---------------------------------------------------------------------------
extern "C" ZSEEK_EXPORT zseek_reader_t *zseek_reader_open_full(zseek_read_file_t user_file,
                                                               size_t cache_size,
                                                               void *call_data, char *errbuf)
{
    uint8_t m[4];
    ssize_t got = user_file.pread(m, 4, 0, user_file.user_data, call_data);
    if (got != 4) {
        set_error(errbuf, got >= 0 ? "unexpected EOF" : "read file failed");
        return nullptr;
    }
    uint32_t magic = (uint32_t)m[0] | ((uint32_t)m[1] << 8) | ((uint32_t)m[2] << 16) |
                     ((uint32_t)m[3] << 24);
    zseek_compression_type_t type;
    if (magic == kZstdMagic) {
        type = ZSEEK_ZSTD;
    } else if (magic == kLz4Magic) {
        type = ZSEEK_LZ4;
    } else {
        set_error(errbuf, "unrecognized file format");
        return nullptr;
    }
    zseek_reader *r = new (std::nothrow) zseek_reader();
    if (!r) {
        set_error_errno(errbuf, "allocate reader", ENOMEM);
        return nullptr;
    }
    r->type = type;
    r->user_file = user_file;
    if (!read_seek_table(user_file, call_data, &r->st)) {
        set_error(errbuf, "read_seek_table failed");
        delete r;
        return nullptr;
    }
    if (cache_size > 0)
        r->cache = new (std::nothrow) FrameCache(cache_size);
    if (cache_size > 0 && !r->cache) {
        set_error(errbuf, "cache creation failed");
        delete r;
        return nullptr;
    }
    const char *vck = getenv("ZSEEK_VERIFY_CHECKSUMS");
    r->verify = vck && *vck && strcmp(vck, "0") != 0;
    const char *io = getenv("ZSEEK_IO_THREADS");
    if (io && *io && atoi(io) > 1)
        r->io_threads = atoi(io) > 64 ? 64 : atoi(io);
    const char *env = getenv("ZSEEK_HIP_BATCH_BYTES");
    if (env && *env) {
        size_t b = strtoull(env, nullptr, 0);
        if (b >= 4096)
            r->batch_bytes = b;
    }
    return r;
}

extern "C" ZSEEK_EXPORT zseek_reader_t *zseek_reader_open(FILE *cfile, size_t cache_size,
                                                          void *call_data, char *errbuf)
{
    zseek_read_file_t uf = {cfile, default_pread, default_fsize};
    return zseek_reader_open_full(uf, cache_size, call_data, errbuf);
}

extern "C" ZSEEK_EXPORT bool zseek_reader_close(zseek_reader_t *reader, void *call_data,
                                                char *errbuf)
{
    (void)call_data;
    (void)errbuf;
    if (!reader)
        return true;   // ref decompress.c:362-363
    delete reader->cache;
    delete reader;     // lanes: streams drained, scratch and buffers freed
    return true;
}

// ---------------------------------------------------------------------------
// error wording
// ---------------------------------------------------------------------------
namespace {

// LZ4F_decompress (liblz4 1.9.3) as the reference's no-cache read drives it
// (decompress.c:614-669): a block's data is decoded only once the request
// reaches into it, but the header after a block that ends exactly at the
// request's end is read and checked in the same call, and so is the end mark
// with what follows it.  Failures met at a header (block size, truncation,
// content size / checksum at the end) are therefore met by a request that ends
// at the failing position; failures inside a block's data (and our
// seek-table-size checks) only by one that goes past it.
bool header_level(int32_t st)
{
    switch (st & 0xFFFF) {
    case ST_MAXBLOCK:
    case ST_TRUNCATED:
    case ST_FRAME_SIZE:
    case ST_CONTENT_CHECKSUM:
        return true;
    default:
        return false;
    }
}

// Does a no-cache request ending `end_in_frame` bytes into a failed LZ4 frame
// succeed in the reference?  fail_at = output offset of the failing block (or
// of the end mark); the decoders leave every byte before it in place.
bool lz4_partial_ok(int32_t st, uint64_t fail_at, uint64_t end_in_frame)
{
    const int32_t code = st & 0xFFFF;
    if (code == ST_SEEK_CHECKSUM || code == ST_NOT_RUN)
        return false;
    return header_level(st) ? end_in_frame < fail_at : end_in_frame <= fail_at;
}

// The same for zstd: libzstd's streaming decoder (decompress.c:414-454)
// decodes a block as soon as the previous one is flushed, so a request ending
// exactly at the failing block's start meets the failure too (golden
// zstd1m_block4_*: (0, 524287) succeeds, (0, 524288) fails).
bool zstd_partial_ok(int32_t st, uint64_t fail_at, uint64_t end_in_frame)
{
    if (st == ST_SEEK_CHECKSUM || st == ST_NOT_RUN)
        return false;
    return end_in_frame < fail_at;
}

// Error text for a failed frame, worded as the reference words the same
// failure.  Cached reads decode the whole frame ("decompress frame: ...",
// decompress.c:766-768); no-cache reads first decode-and-discard the
// offset_in_frame prefix, then decode into the caller's buffer
// (:635-660).  For a failure inside an LZ4 block liblz4 says ERROR_GENERIC
// when the block was decoded straight into the destination (room >= max
// block size) and ERROR_decompressionFailed when it went through its
// temporary buffer; the room depends on which buffer the block landed in.
void frame_error(zseek_reader *r, int32_t st, uint32_t fail_at, size_t frame, size_t offset_in_frame,
                 size_t count, char *errbuf)
{
    const uint64_t dsize = r->st.dsize(frame);
    const uint64_t at = fail_at;
    const char *prefix;
    uint64_t room;
    if (r->cache) {
        prefix = "decompress frame";
        room = dsize - at;
    } else if (offset_in_frame > 0 &&
               (header_level(st) ? at <= offset_in_frame : at < offset_in_frame)) {
        // the discard pass (decode-and-drop of the in-frame prefix) met it
        prefix = "decompress discard data";
        room = offset_in_frame - at;
    } else {
        prefix = "decompress user data";
        uint64_t want = count < dsize - offset_in_frame ? count : dsize - offset_in_frame;
        uint64_t used = at - offset_in_frame;
        room = want > used ? want - used : 0;
    }
    if (r->type == ZSEEK_ZSTD) {
        // libzstd: ZSTD_decompressDCtx (cached) or ZSTD_decompressStream
        // (discard the in-frame prefix, then the caller's bytes,
        // decompress.c:434-451); the discard pass meets a failure whose block
        // starts at or before the prefix's end (a block is decoded as soon
        // as the previous one is flushed)
        if (!r->cache)
            prefix = offset_in_frame > 0 && at <= offset_in_frame ? "decompress discard data"
                                                                   : "decompress user data";
        set_error(errbuf, "%s: %s", prefix, status_name(st));
        return;
    }
    const char *name = status_name(st);
    if (st & ST_BLOCK_FAIL_FLAG)
        name = status_name(room >= status_max_block(st) ? ST_GENERIC : ST_DECOMPRESS_FAILED);
    set_error(errbuf, "%s: %s", prefix, name);
}

// ---------------------------------------------------------------------------
// the batch pipeline of one lane (device)
// ---------------------------------------------------------------------------
struct CacheItem {
    size_t frame;
    uint8_t *data;   // malloc'd, owned until inserted
    size_t len;
};

// One lane's share of a request: frames [fa, fb); bytes [offset, end) of the
// decoded range go to buf at (x - offset).
struct LaneJob {
    zseek_reader *r = nullptr;
    DeviceCtx *g = nullptr;
    size_t fa = 0, fb = 0;
    uint64_t offset = 0, end = 0;
    uint8_t *buf = nullptr;
    bool device_dst = false;
    int dst_dev = -1;
    void *call_data = nullptr;
    size_t cache_cap = 0;   // keep the last cache_cap good frames' bytes
    // results
    bool io_failed = false;   // pread / HIP failure (err holds the text)
    char err[ZSEEK_ERRBUF_SIZE] = {0};
    size_t first_bad = SIZE_MAX;   // first failed frame, if any
    int32_t status = ST_OK;
    uint32_t fail_at = 0;
    uint64_t good_end = 0;   // the lane's bytes before good_end are in buf
    std::deque<CacheItem> cached;
};

void free_items(std::deque<CacheItem> &q)
{
    for (CacheItem &c : q)
        free(c.data);
    q.clear();
}

size_t batch_end(const SeekTable &st, size_t f, size_t fb, size_t limit)
{
    size_t g = f + 1;
    while (g < fb && st.d_off[g + 1] - st.d_off[f] <= limit)
        g++;
    return g;
}

// Concurrent pread callbacks a batch may use: the reader's io_threads, at most
// half the copy pool (the other half keeps the previous batch's host copies
// moving: both run on the pool)
int io_parts(const zseek_reader *r)
{
    const int half = copy_pool_threads() / 2;
    return std::max(1, std::min(r->io_threads, half));
}

// The batch's compressed span through the user's pread callback: one call
// at a time (the reference's contract: it calls pread under the reader's
// lock), or, where the caller allowed it (zsk_reader_set_io_threads), up to
// io_threads concurrent calls on disjoint pieces of >= 4 MiB.
bool read_span(LaneJob &J, uint8_t *dst, uint64_t len, uint64_t off)
{
    zseek_reader *r = J.r;
    const uint64_t kPiece = 4u << 20;
    const int parts = (int)std::min<uint64_t>((uint64_t)io_parts(r), len / kPiece);
    if (parts <= 1) {
        std::lock_guard<std::mutex> io(r->io_lock);
        ssize_t got = r->user_file.pread(dst, len, off, r->user_file.user_data, J.call_data);
        if (got != (ssize_t)len) {
            // ref decompress.c:735-741
            set_error(J.err, got >= 0 ? "unexpected EOF" : "read file failed");
            return false;
        }
        return true;
    }
    std::vector<ssize_t> got(parts, 0);
    CopyTicket t;
    const uint64_t per = (len / parts + 4095) & ~4095ull;
    for (int i = 0; i < parts; i++) {
        const uint64_t a = std::min<uint64_t>(len, per * i), b = std::min<uint64_t>(len, per * (i + 1));
        pool_run([&, i, a, b] {
            got[i] = b > a ? r->user_file.pread(dst + a, b - a, off + a, r->user_file.user_data, J.call_data)
                           : 0;
            if (got[i] == (ssize_t)(b - a))
                got[i] = 0;   // complete
            else if (got[i] >= 0)
                got[i] = 1;   // short: EOF
        }, &t);
    }
    pool_wait(&t);
    for (int i = 0; i < parts; i++)
        if (got[i] != 0) {
            set_error(J.err, got[i] > 0 ? "unexpected EOF" : "read file failed");
            return false;
        }
    return true;
}

#ifdef ZSK_TUNING
// tuning builds, ZSEEK_HOST_TIMERS: a batch's host steps (ns, summed):
// [0] submit to after the read, [1] read to queued, [2] finish's wait, [3]
// finish after the wait, [4] batches; [5] queued to the wait's start
std::atomic<uint64_t> g_ht[6];
uint64_t ht_now()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}
void ht_report()
{
    static const bool on = getenv("ZSEEK_HOST_TIMERS") != nullptr;
    const uint64_t b = g_ht[4].load();
    // (the first 20 batches -- allocations, first launches -- left out)
    if (b == 20)
        for (int i : {0, 1, 2, 3, 5})
            g_ht[i] = 0;
    if (!on || b <= 20 || b % 200)
        return;
    fprintf(stderr, "host per batch (us): read %.1f enqueue %.1f to-wait %.1f wait %.1f after %.1f (%llu batches)\n",
            g_ht[0] / 1e3 / (b - 20), g_ht[1] / 1e3 / (b - 20), g_ht[5] / 1e3 / (b - 20), g_ht[2] / 1e3 / (b - 20),
            g_ht[3] / 1e3 / (b - 20), (unsigned long long)(b - 20));
}
thread_local uint64_t t_queued = 0;
#define HT_T(v) const uint64_t v = ht_now();
#define HT_ADD(i, v) g_ht[i] += ht_now() - v;
#else
#define HT_T(v)
#define HT_ADD(i, v)
#endif

// Read, upload, decode and queue the download of frames [f0, f1) on slot s.
bool submit(LaneJob &J, Slot &s, size_t f0, size_t f1)
{
    HT_T(ht0)
    zseek_reader *r = J.r;
    DeviceCtx &g = *J.g;
    const SeekTable &st = r->st;
    const size_t n = f1 - f0;
    const uint64_t c0 = st.c_off[f0], csz = st.c_off[f1] - c0;
    const uint64_t d0 = st.d_off[f0], dsz = st.d_off[f1] - d0;
    // where the batch's bytes go (lane_plan.h): the request's part (host
    // bounce, same-device or peer copy), and the bytes the host downloads --
    // the request's part for a host destination plus the frames the cache
    // may keep (its last cache_cap frames)
    const BatchRoute br = route_batch(J.device_dst, J.dst_dev, g.device, J.offset, J.end, st.d_off.data(), f0, f1,
                                      J.cache_cap);
    const bool ck = r->verify && st.checksum_flag;
    // no cache and no checksum pass: the batch's last frame is executed only
    // as far as the request reaches into it (the reference's no-cache read
    // also stops there, decompress.c:646-663)
    uint32_t stop_last = 0xFFFFFFFFu;
    if (!J.cache_cap && !ck && J.end < st.d_off[f1])
        stop_last = (uint32_t)(J.end - st.d_off[f1 - 1]);
    (void)hipSetDevice(g.device);
    // the host copies of this slot's previous batch read its pinned bounce
    // h_out: wait for them only when reserve() will reallocate it (waiting
    // always serialized each batch's host copy with the next batch's read
    // and upload: end to end 50.6 -> 33 GB/s); the download into h_out below
    // waits for them anyway
    if (br.h_len > s.h_out_cap)
        pool_wait(&s.copies);
    // the descriptors ride behind the compressed span (past its 256-byte
    // read slack) in the same pinned buffer and the same upload
    const uint64_t doff = (csz + 256 + 255) & ~255ull;
    // (zstd, a request's few frames: the host plan rides behind them too)
    const bool zplan = r->type == ZSEEK_ZSTD && n <= kOneMaxFrames;
    const uint64_t poff = doff + n * sizeof(FrameDesc), up = poff + (zplan ? 16 * (n + 1) : 0);
    if (!s.reserve(up, dsz, br.h_len, n, ck, J.err)) {
        J.io_failed = true;
        return false;
    }
    if (csz && !read_span(J, s.h_comp, csz, c0)) {
        J.io_failed = true;
        return false;
    }
    HT_ADD(0, ht0)
    HT_T(ht1)
    FrameDesc *const h_desc = reinterpret_cast<FrameDesc *>(s.h_comp + doff);
    const FrameDesc *const d_desc = reinterpret_cast<const FrameDesc *>(s.d_comp + doff);
    uint32_t max_dsize = 0;
    for (size_t i = 0; i < n; i++) {
        FrameDesc &d = h_desc[i];
        d.c_off = st.c_off[f0 + i] - c0;
        d.d_off = st.d_off[f0 + i] - d0;
        d.c_size = (uint32_t)st.csize(f0 + i);
        d.d_size = (uint32_t)st.dsize(f0 + i);
        max_dsize = std::max(max_dsize, d.d_size);
    }
    s.f0 = f0;
    s.f1 = f1;
    // per-frame status then fail_at, back to back (one download for both)
    uint32_t *d_fail = reinterpret_cast<uint32_t *>(s.d_status + n);
    s.h_from = br.h_from;
    s.h_len = br.h_len;
    ZstdHostPlan zp{};
    if (zplan)
        zstd_host_plan(h_desc, s.h_comp, (uint32_t)n, reinterpret_cast<uint64_t *>(s.h_comp + poff), &zp);
    hipError_t e = hipSuccess;
    // (a small upload as a kernel on the stream: no DMA hand-off before the
    // decode's first kernel, host_io.hip; env ZSEEK_HOST_DMA=1: always DMA,
    // the download too)
    static const bool host_dma = getenv("ZSEEK_HOST_DMA") != nullptr;
    // env ZSEEK_DONE_FLAG=0: a batch's completion by the stream's event only
    // (no pinned completion word, no results posted by the execute)
    static const bool no_flag = [] {
        const char *v = getenv("ZSEEK_DONE_FLAG");
        return v && !strcmp(v, "0");
    }();
    s.flagged = false;
    // (the LZ4 two-phase decoder's plan kernel initializes both itself, the
    // zstd sequence kernel writes both for every frame)
    const bool lz4_split = r->type == ZSEEK_LZ4 && lz4_pick_engine((uint32_t)n) != ENGINE_WAVE;
    if (host_dma)
        e = hipMemcpyAsync(s.d_comp, s.h_comp, up, hipMemcpyHostToDevice, s.stream);
    else if (upload_small(s.d_comp, s.h_comp, s.h_comp_dev, up, s.stream) != 0)
        e = hipErrorLaunchFailure;
    const bool preset = r->type == ZSEEK_LZ4 && !lz4_split;
    if (e == hipSuccess && preset)
        e = hipMemsetD32Async((hipDeviceptr_t)s.d_status, ST_NOT_RUN, n, s.stream);
    if (e == hipSuccess && preset)
        e = hipMemsetD32Async((hipDeviceptr_t)d_fail, 0, n, s.stream);
    // (zstd: a request's few frames are planned on the host from the pinned
    // span -- no plan launch, no synchronization between plan and decode)
    if (e == hipSuccess && r->type == ZSEEK_ZSTD &&
        (zplan ? zstd_decode_frames_planned(zp, reinterpret_cast<const uint64_t *>(s.d_comp + poff), d_desc,
                                            (uint32_t)n, s.d_comp, s.d_out, s.d_status, &s.zs, s.stream, d_fail,
                                            stop_last)
                            : zstd_decode_frames(d_desc, (uint32_t)n, s.d_comp, s.d_out, s.d_status, &s.zs,
                                                 s.stream, d_fail, stop_last)) != 0)
        e = hipErrorLaunchFailure;
    if (e == hipSuccess && r->type == ZSEEK_LZ4) {
        if (lz4_pick_engine((uint32_t)n) == ENGINE_WAVE) {
            if (launch_lz4_wave(d_desc, (uint32_t)n, s.d_comp, s.d_out, s.d_status, d_fail, s.stream) != 0)
                e = hipErrorLaunchFailure;
        } else if (split_scratch_reserve(&s.split, (uint32_t)n, split_items_needed(h_desc, (uint32_t)n),
                                         s.stream) != 0) {
            e = hipErrorOutOfMemory;
        } else {
            // a lone frame with a host destination (or none): its execute
            // writes the status words, the bytes and the completion word
            // itself when it takes the one-frame route (no download kernel)
            HostPost post;
            const bool want_post = n == 1 && !host_dma && !no_flag && !ck && br.route != COPY_DEVICE &&
                                   br.route != COPY_PEER && s.h_status_dev &&
                                   (!s.h_len || (s.h_out_dev && !(reinterpret_cast<uintptr_t>(s.h_out_dev) & 15)));
            if (want_post) {
                if (s.h_len)
                    pool_wait(&s.copies);   // (the execute writes h_out)
                s.h_flag = reinterpret_cast<volatile uint32_t *>(s.h_status + 2 * n);
                *s.h_flag = 0;
                s.seq = s.seq + 1 ? s.seq + 1 : 1;
                post.h_status = reinterpret_cast<uint32_t *>(s.h_status_dev);
                post.h_out = static_cast<uint8_t *>(s.h_out_dev);
                post.h_from = (uint32_t)s.h_from;
                post.h_len = (uint32_t)s.h_len;
                post.h_flag = reinterpret_cast<uint32_t *>(s.h_status_dev) + 2 * n;
                post.seq = s.seq;
            }
            bool posted = false;
            if (launch_lz4_split(d_desc, (uint32_t)n, s.d_comp, s.d_out, s.d_status, d_fail, s.stream, &s.split,
                                 ROUTE_AUTO, 15, 0, stop_last, max_dsize, want_post ? &post : nullptr,
                                 &posted, true) != 0)
                e = hipErrorLaunchFailure;
            s.flagged = posted;
        }
    }
    // seek-table checksums (descriptor bit 7) when asked for: XXH64 low 32
    // bits of every decoded frame, on the GPU (frame_check.hip)
    if (e == hipSuccess && ck) {
        memcpy(s.h_ck, st.checksum.data() + f0, n * sizeof(uint32_t));
        e = hipMemcpyAsync(s.d_ck, s.h_ck, n * sizeof(uint32_t), hipMemcpyHostToDevice, s.stream);
        if (e == hipSuccess &&
            launch_frame_checksums(d_desc, (uint32_t)n, s.d_out, s.d_ck, s.d_status, s.stream) != 0)
            e = hipErrorLaunchFailure;
    }
    // decoded bytes out: straight into a device destination (a peer copy from
    // another lane's device), or into the slot's pinned bounce once the host
    // copies of its previous batch are done; the status words and the bounce
    // part in one small-download kernel (host_io.hip) when they are small
    if (e == hipSuccess && br.route == COPY_DEVICE)
        e = hipMemcpyAsync(J.buf + br.dst_off, s.d_out + br.src_off, br.len, hipMemcpyDeviceToDevice, s.stream);
    else if (e == hipSuccess && br.route == COPY_PEER)
        e = hipMemcpyPeerAsync(J.buf + br.dst_off, J.dst_dev, s.d_out + br.src_off, g.device, br.len, s.stream);
    if (e == hipSuccess && s.h_len)
        pool_wait(&s.copies);
    if (e == hipSuccess && s.flagged) {
        // (posted by the execute: nothing to download)
    } else if (e == hipSuccess && host_dma) {
        e = hipMemcpyAsync(s.h_status, s.d_status, 2 * n * sizeof(int32_t), hipMemcpyDeviceToHost, s.stream);
        if (e == hipSuccess && s.h_len)
            e = hipMemcpyAsync(s.h_out, s.d_out + s.h_from, s.h_len, hipMemcpyDeviceToHost, s.stream);
    } else if (e == hipSuccess) {
        // a small batch posts its completion to a pinned word the host spins
        // on (finish)
        int rc = 1;
        if (!no_flag && s.h_status_dev) {
            // the word past the 2n status words: in h_status's 256-byte slack
            // (cleared first: the word may hold an older batch's fail_at)
            s.h_flag = reinterpret_cast<volatile uint32_t *>(s.h_status + 2 * n);
            *s.h_flag = 0;
            s.seq = s.seq + 1 ? s.seq + 1 : 1;
            rc = download_flagged(reinterpret_cast<uint32_t *>(s.h_status), s.h_status_dev,
                                  reinterpret_cast<const uint32_t *>(s.d_status), (uint32_t)(2 * n), s.h_out,
                                  s.h_out_dev, s.d_out + s.h_from, s.h_len,
                                  reinterpret_cast<uint32_t *>(s.h_status_dev) + 2 * n, s.seq, s.stream);
            s.flagged = rc == 0;
        }
        if (rc == 1)
            rc = download_small(reinterpret_cast<uint32_t *>(s.h_status), s.h_status_dev,
                                reinterpret_cast<const uint32_t *>(s.d_status), (uint32_t)(2 * n), s.h_out,
                                s.h_out_dev, s.d_out + s.h_from, s.h_len, s.stream);
        if (rc != 0)
            e = hipErrorLaunchFailure;
    }
    if (e == hipSuccess)
        e = hipEventRecord(s.done, s.stream);
    if (e != hipSuccess) {
        set_error(J.err, "GPU decode failed: %s", hipGetErrorString(e));
        J.io_failed = true;
        (void)hipStreamSynchronize(s.stream);
        return false;
    }
    g.batches++;
    g.frames_decoded += n;
    g.bytes_decoded += dsz;
    g.bytes_uploaded += csz;
    HT_ADD(1, ht1)
#ifdef ZSK_TUNING
    t_queued = ht_now();
#endif
    return true;
}

// Wait for slot s's batch; hand its bytes to the caller (host: pool copies
// from the bounce) and its last good frames to the cache candidates.  false
// when a frame of the batch failed (the lane stops there).
bool finish(LaneJob &J, Slot &s)
{
    zseek_reader *r = J.r;
    const SeekTable &st = r->st;
#ifdef ZSK_TUNING
    if (t_queued)
        g_ht[5] += ht_now() - t_queued;
    const uint64_t ht2 = ht_now();
#endif
    // (hipEventSynchronize: polling hipEventQuery instead for a small batch
    // measured no better, LZ4 4 KiB p50 85.6-86.2 against 83.5-84.4 us.)
    // A flagged batch: spin on its pinned completion word -- posted once its
    // download is in host memory -- asking the event every 256 spins, so a
    // batch that fails before the download (no flag ever) still ends
    hipError_t e = hipErrorNotReady;
    if (s.flagged) {
        for (uint32_t k = 0;; k++) {
            if (__atomic_load_n(s.h_flag, __ATOMIC_ACQUIRE) == s.seq) {
                e = hipSuccess;
                break;
            }
            if ((k & 255) == 255 && hipEventQuery(s.done) != hipErrorNotReady)
                break;
            __builtin_ia32_pause();
        }
    }
    if (e != hipSuccess)
        e = hipEventSynchronize(s.done);
#ifdef ZSK_TUNING
    g_ht[2] += ht_now() - ht2;
    struct HtAfter {
        uint64_t t = ht_now();
        ~HtAfter()
        {
            g_ht[3] += ht_now() - t;
            g_ht[4]++;
            ht_report();
        }
    } ht_after;
#endif
    if (e != hipSuccess) {
        set_error(J.err, "GPU decode failed: %s", hipGetErrorString(e));
        J.io_failed = true;
        return false;
    }
    const size_t f0 = s.f0, f1 = s.f1, n = f1 - f0;
    const uint64_t d0 = st.d_off[f0];
    size_t bad = f1;
    for (size_t i = 0; i < n; i++)
        if (s.h_status[i] != ST_OK) {
            bad = f0 + i;
            break;
        }
    uint64_t good_end = st.d_off[bad];
    if (bad < f1) {
        J.first_bad = bad;
        J.status = s.h_status[bad - f0];
        J.fail_at = reinterpret_cast<const uint32_t *>(s.h_status + n)[bad - f0];
        // Without a cache the reference decodes a frame only as far as the
        // request reaches (lz4_partial_ok, zstd_partial_ok).
        const uint64_t end_in = J.end - st.d_off[bad];
        if (!r->cache && (r->type == ZSEEK_LZ4 ? lz4_partial_ok(J.status, J.fail_at, end_in)
                                               : zstd_partial_ok(J.status, J.fail_at, end_in)))
            good_end = J.end;
    }
    const uint64_t lo = std::max<uint64_t>(J.offset, d0);
    const uint64_t hi = std::min<uint64_t>(J.end, good_end);
    if (!J.device_dst && hi > lo)
        pool_copy(J.buf + (lo - J.offset), s.h_out + (lo - d0 - s.h_from), hi - lo, &s.copies);
    J.good_end = std::max<uint64_t>(J.good_end, std::min<uint64_t>(J.end, good_end));
    if (J.cache_cap) {
        // the last cache_cap good frames of the batch, in frame order
        const size_t a = bad - std::min(bad - f0, J.cache_cap);
        for (size_t i = a; i < bad; i++) {
            const size_t len = st.dsize(i);
            uint8_t *p = (uint8_t *)malloc(len ? len : 1);
            if (!p) {
                set_error_errno(J.err, "allocate decompressed buffer", errno);
                J.io_failed = true;
                return false;
            }
            const uint64_t x = st.d_off[i] - d0;
            if (x >= s.h_from && x + len <= s.h_from + s.h_len) {
                memcpy(p, s.h_out + (x - s.h_from), len);
            } else if (len && hipMemcpy(p, s.d_out + x, len, hipMemcpyDeviceToHost) != hipSuccess) {
                free(p);
                set_error(J.err, "copy decoded data failed");
                J.io_failed = true;
                return false;
            }
            J.cached.push_back({i, p, len});
            if (J.cached.size() > J.cache_cap) {
                free(J.cached.front().data);
                J.cached.pop_front();
            }
        }
    }
    return bad == f1;
}

// The batch loop of one lane: up to kSlots batches in flight, finished in
// order; the first batch is small so a request's first bytes come early.
void run_lane(LaneJob &J)
{
    DeviceGuard keep;
    DeviceCtx &g = *J.g;
    (void)hipSetDevice(g.device);
    J.good_end = std::max<uint64_t>(J.offset, J.r->st.d_off[J.fa]);
    std::deque<int> inflight;
    size_t f = J.fa;
    int next = 0;
    bool stop = false;
    size_t limit = std::min(kFirstBatch, J.r->batch_bytes);
    for (;;) {
        if (!stop && f < J.fb && (int)inflight.size() < kSlots) {
            const size_t gend = batch_end(J.r->st, f, J.fb, limit);
            limit = J.r->batch_bytes;
            if (!submit(J, g.slot[next], f, gend)) {
                stop = true;
                continue;
            }
            inflight.push_back(next);
            next = (next + 1) % kSlots;
            f = gend;
            continue;
        }
        if (inflight.empty())
            break;
        Slot &s = g.slot[inflight.front()];
        inflight.pop_front();
        if (stop) {   // a failure before this batch: drain it, keep nothing
            (void)hipEventSynchronize(s.done);
            continue;
        }
        if (!finish(J, s))
            stop = true;
    }
    for (Slot &s : g.slot)
        pool_wait(&s.copies);
}

bool ensure_lanes(zseek_reader *r, char *errbuf)
{
    if (r->devices.empty())
        r->devices = default_devices();
    if (r->devices.empty()) {
        set_error(errbuf, "no HIP device available");
        return false;
    }
    while (r->lanes.size() < r->devices.size())
        r->lanes.emplace_back(new DeviceCtx());
    for (size_t i = 0; i < r->devices.size(); i++)
        if (!r->lanes[i]->init(r->devices[i], errbuf))
            return false;
    return true;
}

// The reader's stats fields that change (cache, staging) -> the lock-free
// snapshot zseek_reader_stats reads; called under the exclusive lock.
void publish_stats(zseek_reader *r)
{
    r->snap_cache_memory.store(r->cache ? r->cache->memory_usage() : 0, std::memory_order_relaxed);
    r->snap_cached_frames.store(r->cache ? r->cache->entries() : 0, std::memory_order_relaxed);
    size_t buffered = 0;
    for (auto &l : r->lanes)
        buffered += l->host_bytes();
    r->snap_buffered.store(buffered, std::memory_order_relaxed);
}

// bytes [rel, rel + count) of a cached frame (len bytes) -> the caller's
// buffer (ref decompress.c:786-790)
ssize_t copy_slice(void *buf, const uint8_t *data, size_t len, size_t rel, size_t count, bool device_dst,
                   char *errbuf)
{
    size_t n = count < len - rel ? count : len - rel;
    if (device_dst) {
        if (n && hipMemcpy(buf, data + rel, n, hipMemcpyHostToDevice) != hipSuccess) {
            set_error(errbuf, "copy decoded data failed");
            return -1;
        }
    } else {
        memcpy(buf, data + rel, n);
    }
    return (ssize_t)n;
}

// Range read: [offset, offset+count) into buf (host or device memory), both
// codecs (ref decompress.c:685-804 LZ4, :377-574 zstd).
ssize_t pread_frames(zseek_reader *r, void *buf, size_t count, size_t offset, void *call_data,
                     char *errbuf, bool device_dst)
{
    const SeekTable &st = r->st;
    int64_t fi = st.frame_of(offset);
    if (fi < 0)
        return 0;   // EOF (ref decompress.c:695-697)
    DeviceGuard keep_device;   // the caller's current device is restored on return
    const size_t f_first = (size_t)fi;
    const uint64_t end = offset + count < st.decompressed_size() ? offset + count
                                                                 : st.decompressed_size();
    const bool one_cached = r->cache && (count == 0 || (size_t)st.frame_of(end - 1) == f_first);
    // a cache hit under the shared lock (decompress.c:699-706): concurrent
    // hits copy at once; a frame is only evicted under the exclusive lock
    if (one_cached) {
        std::shared_lock<std::shared_mutex> shared(r->lock);
        size_t len = 0;
        const uint8_t *data;
        {
            std::lock_guard<std::mutex> g(r->lru_lock);
            data = r->cache->find(f_first, &len);
        }
        if (data)
            return copy_slice(buf, data, len, offset - st.d_off[f_first], count, device_dst, errbuf);
    }
    std::unique_lock<std::shared_mutex> guard(r->lock);
    struct Publish {   // the stats snapshot once this request is done
        zseek_reader *r;
        ~Publish() { publish_stats(r); }
    } publish{r};
    // single-frame request with a cache: the reference's cached path
    // (decompress.c:699-796), GPU-decoded on a miss (one batch of one frame,
    // one synchronisation)
    if (one_cached) {
        size_t len = 0;
        const uint8_t *data = r->cache->find(f_first, &len);   // (another thread's miss may have filled it)
        if (!data) {
            if (!ensure_lanes(r, errbuf))
                return -1;
            LaneJob J;
            J.r = r;
            J.g = r->lanes[0].get();
            J.fa = f_first;
            J.fb = f_first + 1;
            J.offset = J.end = st.d_off[f_first + 1];   // nothing to copy: the cache serves it
            J.device_dst = true;
            J.call_data = call_data;
            J.cache_cap = 1;
            run_lane(J);
            if (J.io_failed) {
                set_error(errbuf, "%s", J.err);
                free_items(J.cached);
                return -1;
            }
            if (J.first_bad != SIZE_MAX || J.cached.empty()) {
                frame_error(r, J.status, J.fail_at, f_first, offset - st.d_off[f_first], count, errbuf);
                free_items(J.cached);
                return -1;
            }
            CacheItem c = J.cached.back();
            J.cached.pop_back();
            if (!r->cache->insert(c.frame, c.data, c.len)) {
                free(c.data);
                set_error(errbuf, "frame caching failed");
                return -1;
            }
            data = r->cache->find(f_first, &len);
        }
        return copy_slice(buf, data, len, offset - st.d_off[f_first], count, device_dst, errbuf);
    }
    if (count == 0)
        return 0;
    if (!ensure_lanes(r, errbuf))
        return -1;

    // multi-frame (or no-cache) request: lanes of whole frames, split by
    // decoded bytes over the reader's devices
    const size_t f_last = (size_t)st.frame_of(end - 1);
    size_t L = r->lanes.size();
    // a lane gets at least one full batch (and 1 MiB)
    const size_t per_lane = std::max<size_t>(r->batch_bytes, kLaneMin);
    int dst_dev = -1;
    if (device_dst) {
        hipPointerAttribute_t pa;
        dst_dev = hipPointerGetAttributes(&pa, buf) == hipSuccess ? pa.device : r->lanes[0]->device;
    }
    const std::vector<LaneShare> share =
        plan_lanes(L, offset, end, f_first, f_last, per_lane, [&](uint64_t x) { return st.frame_of(x); });
    L = share.size();
    std::vector<LaneJob> jobs(L);
    for (size_t i = 0; i < L; i++) {
        LaneJob &J = jobs[i];
        J.r = r;
        J.g = r->lanes[i].get();
        J.fa = share[i].fa;
        J.fb = share[i].fb;
        J.offset = offset;
        J.end = end;
        J.buf = (uint8_t *)buf;
        J.device_dst = device_dst;
        J.dst_dev = dst_dev;
        J.call_data = call_data;
        J.cache_cap = r->cache ? r->cache->capacity() : 0;
    }
    std::vector<std::thread> th;
    for (size_t i = 1; i < L; i++)
        th.emplace_back(run_lane, std::ref(jobs[i]));
    run_lane(jobs[0]);
    for (auto &t : th)
        t.join();

    // the contiguous prefix the lanes delivered, up to the first failure
    ssize_t done = 0;
    size_t stop_lane = L;
    for (size_t i = 0; i < L; i++) {
        LaneJob &J = jobs[i];
        done = (ssize_t)(J.good_end - offset);
        if (J.io_failed || J.first_bad != SIZE_MAX) {
            stop_lane = i;
            break;
        }
    }
    // the cache ends as a reference caller's looping frame by frame over the
    // delivered range would leave it: its last `capacity` good frames, MRU last
    if (r->cache) {
        std::deque<CacheItem> keep;
        for (size_t i = 0; i < L; i++) {
            if (i <= stop_lane || stop_lane == L) {
                for (CacheItem &c : jobs[i].cached)
                    keep.push_back(c);
                jobs[i].cached.clear();
            } else {
                free_items(jobs[i].cached);
            }
        }
        while (keep.size() > r->cache->capacity()) {
            free(keep.front().data);
            keep.pop_front();
        }
        for (CacheItem &c : keep)
            if (!r->cache->insert(c.frame, c.data, c.len))
                free(c.data);
    }
    if (stop_lane < L && done == 0) {
        LaneJob &J = jobs[stop_lane];
        if (J.io_failed)
            set_error(errbuf, "%s", J.err);
        else
            frame_error(r, J.status, J.fail_at, J.first_bad,
                        offset > st.d_off[J.first_bad] ? offset - st.d_off[J.first_bad] : 0, count,
                        errbuf);
        return -1;
    }
    return done;
}

}   // namespace

// ---------------------------------------------------------------------------
// pread / read / stats (ref decompress.c:806-891)
// ---------------------------------------------------------------------------
extern "C" ZSEEK_EXPORT ssize_t zseek_pread(zseek_reader_t *reader, void *buf, size_t count,
                                            size_t offset, void *call_data, char *errbuf)
{
    if (!reader) {
        set_error(errbuf, "invalid reader");
        return 0;   // ref decompress.c:809-812 returns false (0)
    }
    return pread_frames(reader, buf, count, offset, call_data, errbuf, false);
}

extern "C" ZSEEK_EXPORT ssize_t zseek_read(zseek_reader_t *reader, void *buf, size_t count,
                                           void *call_data, char *errbuf)
{
    if (!reader) {
        set_error(errbuf, "invalid reader");
        return 0;
    }
    // the reference reads and advances pos outside its lock
    // (decompress.c:831-832) although zseek.h:404 documents the call as safe
    // to call concurrently; here concurrent zseek_read calls take disjoint
    // consecutive ranges
    std::lock_guard<std::mutex> guard(reader->cursor_lock);
    ssize_t ret = zseek_pread(reader, buf, count, reader->pos, call_data, errbuf);
    if (ret > 0)
        reader->pos += (size_t)ret;
    return ret;
}

extern "C" ZSEEK_EXPORT bool zseek_reader_stats(zseek_reader_t *reader,
                                                zseek_reader_stats_t *stats, char *errbuf)
{
    if (!reader) {
        set_error(errbuf, "invalid reader");
        return false;
    }
    if (!stats) {
        set_error(errbuf, "invalid stats pointer");
        return false;
    }
    // the seek table is immutable after open; the rest is the snapshot the
    // last request published (no reader lock: see publish_stats)
    stats->seek_table_memory = reader->st.memory_usage();
    stats->frames = reader->st.frames();
    stats->decompressed_size = reader->st.decompressed_size();
    stats->cache_memory = reader->snap_cache_memory.load(std::memory_order_relaxed);
    stats->cached_frames = reader->snap_cached_frames.load(std::memory_order_relaxed);
    stats->buffer_size = reader->snap_buffered.load(std::memory_order_relaxed);
    return true;
}

// ---------------------------------------------------------------------------
// GPU extensions (include/zseek_hip.h)
// ---------------------------------------------------------------------------
extern "C" ZSEEK_EXPORT int zsk_lz4_decode_frames(const zsk_frame_desc_t *d_desc,
                                                  uint32_t nframes, const void *d_comp,
                                                  void *d_out, int32_t *d_status, void *stream)
{
    static_assert(sizeof(zsk_frame_desc_t) == sizeof(FrameDesc), "descriptor ABI");
    return launch_lz4_frames(reinterpret_cast<const FrameDesc *>(d_desc), nframes,
                             static_cast<const uint8_t *>(d_comp), static_cast<uint8_t *>(d_out),
                             d_status, nullptr, static_cast<hipStream_t>(stream));
}

extern "C" ZSEEK_EXPORT int zsk_lz4_decode_frames_ex(const zsk_frame_desc_t *d_desc, uint32_t nframes,
                                                     const void *d_comp, void *d_out, int32_t *d_status,
                                                     void *stream, int decoder)
{
    if (decoder < ZSK_DECODER_AUTO || decoder > ZSK_DECODER_ONE)
        return -1;
    return launch_lz4_frames(reinterpret_cast<const FrameDesc *>(d_desc), nframes,
                             static_cast<const uint8_t *>(d_comp), static_cast<uint8_t *>(d_out),
                             d_status, nullptr, static_cast<hipStream_t>(stream), decoder);
}

extern "C" ZSEEK_EXPORT const char *zsk_lz4_kernel_name(uint32_t nframes)
{
    return zsk::lz4_kernel_name(nframes);
}

extern "C" ZSEEK_EXPORT const char *zsk_lz4_parse_kernel_name(uint32_t nframes, uint32_t c_size)
{
    return zsk::parse_kernel_name(nframes, c_size);
}

#ifdef ZSK_TUNING
// Kernel tuning hook (libzseek_tune.so only): decode with an explicit launch
// variant, see launch_lz4_frames_variant (tuning.hip).
extern "C" ZSEEK_EXPORT int zsk_dev_lz4_decode_variant(int variant, const zsk_frame_desc_t *d_desc,
                                                       uint32_t nframes, const void *d_comp,
                                                       void *d_out, int32_t *d_status,
                                                       void *stream)
{
    return launch_lz4_frames_variant(variant, reinterpret_cast<const FrameDesc *>(d_desc),
                                     nframes, static_cast<const uint8_t *>(d_comp),
                                     static_cast<uint8_t *>(d_out), d_status,
                                     static_cast<hipStream_t>(stream));
}
#endif

// The device API's zstd scratch: a bounded stream-ordered pool (pool.h).
extern "C" ZSEEK_EXPORT int zsk_zstd_decode_frames(const zsk_frame_desc_t *d_desc,
                                                   uint32_t nframes, const void *d_comp,
                                                   void *d_out, int32_t *d_status, void *stream)
{
    static ScratchPool<ZstdScratch> pool;
    hipStream_t hs = static_cast<hipStream_t>(stream);
    ZstdScratch *s = pool.acquire(hs);
    if (!s)
        return -1;
    const int rc = zsk::zstd_decode_frames(reinterpret_cast<const FrameDesc *>(d_desc), nframes,
                                           static_cast<const uint8_t *>(d_comp),
                                           static_cast<uint8_t *>(d_out), d_status, s, hs);
    pool.release(s, hs);
    return rc;
}

extern "C" ZSEEK_EXPORT int zsk_kernel_timing(int on)
{
    return zsk::kernel_timing(on);
}

extern "C" ZSEEK_EXPORT int zsk_kernel_times(double *ms, int cap)
{
    return zsk::kernel_times(ms, cap);
}

extern "C" ZSEEK_EXPORT const char *zsk_status_string(int32_t status)
{
    return status_name(status);
}

extern "C" ZSEEK_EXPORT ssize_t zsk_reader_frames(zseek_reader_t *reader, uint64_t *c_off,
                                                  uint64_t *d_off)
{
    if (!reader)
        return -1;
    size_t n = reader->st.frames();
    if (c_off)
        memcpy(c_off, reader->st.c_off.data(), (n + 1) * sizeof(uint64_t));
    if (d_off)
        memcpy(d_off, reader->st.d_off.data(), (n + 1) * sizeof(uint64_t));
    return (ssize_t)n;
}

extern "C" ZSEEK_EXPORT int zsk_reader_type(zseek_reader_t *reader)
{
    return reader ? (int)reader->type : -1;
}

extern "C" ZSEEK_EXPORT ssize_t zsk_pread_device(zseek_reader_t *reader, void *d_buf,
                                                 size_t count, size_t offset, void *call_data,
                                                 char *errbuf)
{
    if (!reader) {
        set_error(errbuf, "invalid reader");
        return 0;
    }
    return pread_frames(reader, d_buf, count, offset, call_data, errbuf, true);
}

// Writes the first `size` bytes of the counters (at most sizeof): a caller
// built against an older, shorter zsk_gpu_stats_t gets exactly its fields.
extern "C" ZSEEK_EXPORT bool zsk_reader_gpu_stats_ex(zseek_reader_t *reader, zsk_gpu_stats_t *out, size_t size)
{
    if (!reader || !out || size == 0)
        return false;
    zsk_gpu_stats_t s;
    memset(&s, 0, sizeof(s));
    {
        std::unique_lock<std::shared_mutex> guard(reader->lock);
        s.device = reader->lanes.empty() ? -1 : reader->lanes[0]->device;
        s.copy_threads = copy_pool_threads();
        s.io_parts = io_parts(reader);
        for (auto &l : reader->lanes) {
            s.batches += l->batches;
            s.frames_decoded += l->frames_decoded;
            s.bytes_decoded += l->bytes_decoded;
            s.bytes_uploaded += l->bytes_uploaded;
            s.device_memory += l->device_bytes();
        }
    }
    memcpy(out, &s, size < sizeof(s) ? size : sizeof(s));
    return true;
}

// The round-4 layout (through `device`): what callers of this entry point
// were built with before copy_threads / io_parts were added;
// zsk_reader_gpu_stats_ex returns the whole struct.
extern "C" ZSEEK_EXPORT bool zsk_reader_gpu_stats(zseek_reader_t *reader, zsk_gpu_stats_t *s)
{
    return zsk_reader_gpu_stats_ex(reader, s, offsetof(zsk_gpu_stats_t, copy_threads));
}

extern "C" ZSEEK_EXPORT bool zsk_reader_set_batch_bytes(zseek_reader_t *reader, size_t bytes)
{
    if (!reader || bytes < 4096)
        return false;
    std::unique_lock<std::shared_mutex> guard(reader->lock);
    reader->batch_bytes = bytes;
    return true;
}

// Concurrent pread callbacks (zseek_hip.h): an opt-in beyond the reference's
// contract, for callbacks that are safe to call from several threads.
extern "C" ZSEEK_EXPORT bool zsk_reader_set_io_threads(zseek_reader_t *reader, int n)
{
    if (!reader || n < 1 || n > 64)
        return false;
    std::unique_lock<std::shared_mutex> guard(reader->lock);
    reader->io_threads = n;
    return true;
}

// Seek-table checksum verification switch (zseek_hip.h).
extern "C" ZSEEK_EXPORT bool zsk_reader_set_verify_checksums(zseek_reader_t *reader, bool on)
{
    if (!reader)
        return false;
    std::unique_lock<std::shared_mutex> guard(reader->lock);
    reader->verify = on;
    return true;
}

// Devices a reader decodes on (zseek_hip.h): one lane per entry, a device may
// repeat (several pipelines on one GPU).  Takes effect at the next read.
extern "C" ZSEEK_EXPORT bool zsk_reader_set_devices(zseek_reader_t *reader, const int *devices,
                                                    int n)
{
    if (!reader || n < 0 || (n > 0 && !devices))
        return false;
    int count = 0;
    if (n > 0 && hipGetDeviceCount(&count) != hipSuccess)
        return false;
    for (int i = 0; i < n; i++)
        if (devices[i] < 0 || devices[i] >= count)
            return false;
    std::unique_lock<std::shared_mutex> guard(reader->lock);
    reader->lanes.clear();   // drains and frees the old lanes
    reader->devices.assign(devices, devices + n);
    publish_stats(reader);
    return true;
}

// The devices a reader decodes on: up to cap entries into devices (NULL:
// count only); returns the count (0 before the first read picks the default).
extern "C" ZSEEK_EXPORT int zsk_reader_devices(zseek_reader_t *reader, int *devices, int cap)
{
    if (!reader)
        return -1;
    std::unique_lock<std::shared_mutex> guard(reader->lock);
    const int n = (int)reader->devices.size();
    for (int i = 0; devices && i < n && i < cap; i++)
        devices[i] = reader->devices[i];
    return n;
}
