// writer.cpp — zseek_writer_* (sequential writer of seekable LZ4 / zstd files).
//
// Out of the GPU hot path: kept so the library stays a
// drop-in for the reference's full C API and so tests/bench can produce
// inputs.  Frames are compressed on the host with the same liblz4 / libzstd
// calls and parameters as the reference (/root/reference/src/compress.c), so
// the files are byte-identical to the reference writer's for the same write
// sequence.  One reference defect is not reproduced: a short buffered write
// followed by a write >= min_frame_size (compress.c:791-795 checks frame_cm,
// which LZ4 never sets) logs a frame with a stale dSize and corrupts the file;
// here buffered bytes always end their frame first.
//
// GPU mode (zsk_writer_set_gpu_compress, env ZSEEK_GPU_COMPRESS; LZ4 frames
// of <= 4 MiB, levels < 3): lz4_frame queues the frame instead of
// compressing it, and a batch of queued frames is compressed by
// zsk_lz4_compress_frames (csrc/lz4_compress.hip, byte-identical to
// LZ4F_compressFrame) and then written and logged in queue order, each with
// the call_data of the zseek_write that produced it.  Frames the GPU path
// does not take flush the queue first, so the file is the same byte for byte.
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include <hip/hip_runtime.h>
#include <lz4frame.h>
#include <zstd.h>

#include "../../include/zseek.h"
#include "../../include/zseek_hip.h"
#include "host.h"

using namespace zsk;

namespace {
constexpr uint32_t kMaxFrames = 0x8000000u;   // ZSTD_SEEKABLE_MAXFRAMES (ref seek_table.c:17)

struct FrameLogEntry {
    uint32_t c_size, d_size;
};

constexpr size_t kGpuDefaultBatch = 1u << 30;   // 16,384 frames of 64 KiB: ~20 GB/s per launch (bench launch_by_frames)
constexpr size_t kGpuMaxFrame = ZSK_LZ4_COMPRESS_MAX_FRAME;   // the GPU compressor's limit
constexpr size_t kGpuMinBatch = 65536;   // smallest batch: one 64 KiB frame
constexpr size_t kGpuMaxBatchFrames = 65536;
constexpr size_t kGpuTableBytes = 65536;      // compressor scratch per queued frame
constexpr size_t kGpuFirstStaging = 64u << 20;   // staging starts here, grows x2 to the batch

// Queued LZ4 frames of a writer in GPU mode and the buffers they go through.
struct GpuLz4 {
    size_t batch_bytes = 0;   // 0: off
    size_t max_frames = 0;    // frames per flush: table scratch <= batch_bytes
    bool failed = false;      // a flush failed: later writes and close fail too
    int device = -1;
    hipStream_t stream = nullptr;
    uint8_t *h_in = nullptr, *h_out = nullptr;   // pinned staging
    size_t in_cap = 0, out_cap = 0, in_used = 0, out_used = 0;
    uint8_t *d_in = nullptr, *d_out = nullptr, *d_scratch = nullptr;
    zsk_compress_desc_t *d_desc = nullptr;
    uint32_t *d_csize = nullptr;
    size_t d_frames = 0, d_scratch_cap = 0;
    std::vector<zsk_compress_desc_t> desc;
    std::vector<uint32_t> csize;
    std::vector<void *> call_data;

    void release()
    {
        if (device < 0)
            return;
        DeviceGuard keep;
        (void)hipSetDevice(device);
        if (stream)
            (void)hipStreamSynchronize(stream);
        for (void *p : {(void *)d_in, (void *)d_out, (void *)d_scratch, (void *)d_desc, (void *)d_csize})
            if (p)
                (void)hipFree(p);
        for (void *p : {(void *)h_in, (void *)h_out})
            if (p)
                (void)hipHostFree(p);
        if (stream)
            hip_stream_put(stream);
        *this = GpuLz4();
    }

    // pinned + device staging for in_need input bytes (a flush happened
    // first: nothing is queued)
    bool reserve(size_t in_need)
    {
        // (the first staging is allocated even for an empty frame: its output
        // slot needs room although it has no input bytes)
        if (in_need <= in_cap && out_cap)
            return true;
        size_t cap = in_cap ? in_cap : kGpuFirstStaging;
        while (cap < in_need)
            cap *= 2;
        cap = std::min(cap, batch_bytes + kGpuMaxFrame);
        if (cap < in_need)
            return false;
        for (void *p : {(void *)d_in, (void *)d_out})
            if (p)
                (void)hipFree(p);
        for (void *p : {(void *)h_in, (void *)h_out})
            if (p)
                (void)hipHostFree(p);
        d_in = d_out = h_in = h_out = nullptr;
        in_cap = out_cap = 0;
        // a slot per frame: ZSK_LZ4_COMPRESS_BOUND(n) <= n + n / 16384 + 39 bytes
        const size_t ocap = cap + cap / 16384 + 40 * std::min(max_frames, cap / 16 + 1);
        if (hipHostMalloc((void **)&h_in, cap, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&h_out, ocap, hipHostMallocDefault) != hipSuccess ||
            hipMalloc((void **)&d_in, cap) != hipSuccess || hipMalloc((void **)&d_out, ocap) != hipSuccess)
            return false;
        in_cap = cap;
        out_cap = ocap;
        return true;
    }
};
}   // namespace

struct zseek_writer {
    zseek_write_file_t user_file;
    zseek_compression_type_t type;
    ZSTD_CCtx *cctx = nullptr;
    bool mt = false;
    LZ4F_preferences_t prefs;
    size_t frame_uc = 0;   // current frame, uncompressed bytes
    size_t frame_cm = 0;   // current frame, compressed bytes already written
    size_t min_frame_size = 0;
    size_t total_cm = 0;
    std::vector<FrameLogEntry> log;
    std::vector<uint8_t> ubuf, cbuf;
    GpuLz4 gpu;
};

static bool default_write(const void *data, size_t size, void *user_data, void *call_data)
{
    (void)call_data;
    return fwrite(data, 1, size, (FILE *)user_data) == size;
}

static bool log_frame(zseek_writer *w, char *errbuf)
{
    if (w->log.size() == kMaxFrames) {
        set_error(errbuf, "log frame: Frame index is too large");
        return false;
    }
    w->log.push_back(FrameLogEntry{(uint32_t)w->frame_cm, (uint32_t)w->frame_uc});
    w->total_cm += w->frame_cm;
    w->frame_uc = 0;
    w->frame_cm = 0;
    return true;
}

static bool emit(zseek_writer *w, const void *p, size_t n, void *call_data, char *errbuf)
{
    if (!w->user_file.write(p, n, w->user_file.user_data, call_data)) {
        set_error(errbuf, "write to file failed");
        return false;
    }
    return true;
}

// Compress the queued frames on the GPU, then write and log them in order.
static bool gpu_flush(zseek_writer *w, char *errbuf)
{
    GpuLz4 &g = w->gpu;
    if (g.failed) {
        set_error(errbuf, "%s: %s", "compress frame", "GPU compression failed");
        return false;
    }
    const size_t n = g.desc.size();
    if (n == 0)
        return true;
    DeviceGuard keep;
    bool ok = hipSetDevice(g.device) == hipSuccess;
    if (ok && g.d_frames < n) {
        if (g.d_desc)
            (void)hipFree(g.d_desc);
        if (g.d_csize)
            (void)hipFree(g.d_csize);
        g.d_desc = nullptr;
        g.d_csize = nullptr;
        g.d_frames = 0;
        ok = hipMalloc(&g.d_desc, n * sizeof(zsk_compress_desc_t)) == hipSuccess &&
             hipMalloc(&g.d_csize, n * sizeof(uint32_t)) == hipSuccess;
        if (ok)
            g.d_frames = n;
    }
    const size_t scratch = zsk_lz4_compress_scratch_size((uint32_t)n);
    if (ok && g.d_scratch_cap < scratch) {
        if (g.d_scratch)
            (void)hipFree(g.d_scratch);
        g.d_scratch = nullptr;
        g.d_scratch_cap = 0;
        ok = hipMalloc(&g.d_scratch, scratch) == hipSuccess;
        if (ok)
            g.d_scratch_cap = scratch;
    }
    g.csize.resize(n);
    ok = ok && hipMemcpyAsync(g.d_in, g.h_in, g.in_used, hipMemcpyHostToDevice, g.stream) == hipSuccess &&
         hipMemcpyAsync(g.d_desc, g.desc.data(), n * sizeof(zsk_compress_desc_t), hipMemcpyHostToDevice,
                        g.stream) == hipSuccess &&
         zsk_lz4_compress_frames(g.d_desc, (uint32_t)n, g.d_in, g.d_out, g.d_csize, w->prefs.compressionLevel,
                                 g.d_scratch, g.stream) == 0 &&
         hipMemcpyAsync(g.csize.data(), g.d_csize, n * sizeof(uint32_t), hipMemcpyDeviceToHost, g.stream) ==
             hipSuccess &&
         hipMemcpyAsync(g.h_out, g.d_out, g.out_used, hipMemcpyDeviceToHost, g.stream) == hipSuccess &&
         hipStreamSynchronize(g.stream) == hipSuccess;
    std::vector<zsk_compress_desc_t> desc;
    std::vector<void *> cds;
    desc.swap(g.desc);
    cds.swap(g.call_data);
    if (!ok) {
        // copies already queued may still read the staging: drain the stream
        // before anything reuses it; the queued frames are lost, so the
        // writer stays failed (later writes and close return false)
        (void)hipStreamSynchronize(g.stream);
        g.in_used = g.out_used = 0;
        g.failed = true;
        set_error(errbuf, "%s: %s", "compress frame", "GPU compression failed");
        return false;
    }
    g.in_used = g.out_used = 0;
    // the frame being buffered (ubuf) keeps its counters across the flush
    const size_t uc = w->frame_uc, cm = w->frame_cm;
    for (size_t f = 0; f < n && ok; f++) {
        if (g.csize[f] == 0) {
            set_error(errbuf, "%s: %s", "compress frame", "GPU compression failed");
            ok = false;
            break;
        }
        w->frame_uc = desc[f].src_size;
        w->frame_cm = g.csize[f];
        ok = emit(w, g.h_out + desc[f].dst_off, g.csize[f], cds[f], errbuf) && log_frame(w, errbuf);
    }
    w->frame_uc = uc;
    w->frame_cm = cm;
    if (!ok)   // frames after the failing one are not in the file
        g.failed = true;
    return ok;
}

// Queue one frame for the GPU (the frame's bytes are copied: the caller may
// reuse its buffer when zseek_write returns).
static bool gpu_queue(zseek_writer *w, const void *src, size_t n, bool with_size, void *call_data,
                      char *errbuf)
{
    GpuLz4 &g = w->gpu;
    const size_t slot = ZSK_LZ4_COMPRESS_BOUND(n);
    if (g.failed)
        return gpu_flush(w, errbuf);   // (sets the error)
    if (g.in_used + n > g.in_cap || g.out_used + slot > g.out_cap || g.desc.size() == g.max_frames) {
        // a full staging of linked frames (> 64 KiB) below the batch size
        // doubles after the flush: a flush of them costs about one frame's
        // chain (~0.1 s for 1 MiB frames) whatever the batch holds, so the
        // batch should reach batch_bytes.  Frames of <= 64 KiB keep the first
        // staging (64 MiB: 1,024 frames; growing it cost more in pinned
        // reallocations than the wider launch gained, 2.02 -> 1.18 GB/s for
        // 1 GiB written)
        const bool full = n > 65536 && g.in_used > 0 && g.in_used + n > g.in_cap && g.in_cap < g.batch_bytes;
        if (!gpu_flush(w, errbuf))
            return false;
        if (full) {
            DeviceGuard keep;
            if (hipSetDevice(g.device) != hipSuccess || !g.reserve(g.in_cap + 1)) {
                g.failed = true;
                set_error(errbuf, "%s: %s", "compress frame", "GPU staging allocation failed");
                return false;
            }
        }
    }
    if (g.in_used + n > g.in_cap || g.out_used + slot > g.out_cap) {   // nothing queued: grow
        DeviceGuard keep;
        if (hipSetDevice(g.device) != hipSuccess || !g.reserve(g.in_used + n) || g.out_used + slot > g.out_cap) {
            g.failed = true;
            set_error(errbuf, "%s: %s", "compress frame", "GPU staging allocation failed");
            return false;
        }
    }
    if (n)
        memcpy(g.h_in + g.in_used, src, n);
    zsk_compress_desc_t d;
    d.src_off = g.in_used;
    d.dst_off = g.out_used;
    d.src_size = (uint32_t)n;
    d.flags = with_size ? ZSK_COMPRESS_CONTENT_SIZE : 0;
    g.desc.push_back(d);
    g.call_data.push_back(call_data);
    g.in_used += n;
    g.out_used += slot;
    w->frame_uc = 0;   // accounted when the batch is written (gpu_flush)
    w->frame_cm = 0;
    return g.in_used < g.batch_bytes || gpu_flush(w, errbuf);
}

// One LZ4 frame of src (ref compress.c:463-518 buffered, :737-786 direct).
// content_size = 0 omits the content-size field, as the reference's direct
// path does.
static bool lz4_frame(zseek_writer *w, const void *src, size_t n, size_t content_size,
                      void *call_data, char *errbuf)
{
    if (w->gpu.batch_bytes) {
        if (n <= kGpuMaxFrame)
            return gpu_queue(w, src, n, content_size != 0, call_data, errbuf);
        if (!gpu_flush(w, errbuf))   // frames stay in order
            return false;
    }
    w->prefs.frameInfo.contentSize = content_size;
    size_t bound = LZ4F_compressFrameBound(n, &w->prefs);
    w->cbuf.resize(bound);
    size_t c = LZ4F_compressFrame(w->cbuf.data(), bound, src, n, &w->prefs);
    if (LZ4F_isError(c)) {
        set_error(errbuf, "%s: %s", "compress frame", LZ4F_getErrorName(c));
        return false;
    }
    w->frame_uc += n;
    w->frame_cm += c;
    return emit(w, w->cbuf.data(), c, call_data, errbuf) && log_frame(w, errbuf);
}

static bool zstd_frame(zseek_writer *w, const void *src, size_t n, void *call_data,
                       char *errbuf)
{
    size_t bound = ZSTD_compressBound(n);
    w->cbuf.resize(bound);
    size_t c = ZSTD_compress2(w->cctx, w->cbuf.data(), bound, src, n);
    if (ZSTD_isError(c)) {
        set_error(errbuf, "%s: %s", "compress frame", ZSTD_getErrorName(c));
        return false;
    }
    w->frame_uc += n;
    w->frame_cm += c;
    return emit(w, w->cbuf.data(), c, call_data, errbuf) && log_frame(w, errbuf);
}

// End the buffered frame (ref end_frame_lz4 :463-518, end_frame_zstd :338-394,
// end_frame_zstd_mt :281-333).
static bool end_frame(zseek_writer *w, void *call_data, char *errbuf)
{
    if (w->type == ZSEEK_LZ4) {
        size_t n = w->ubuf.size();
        w->frame_uc = 0;
        bool ok = lz4_frame(w, w->ubuf.data(), n, n, call_data, errbuf);
        w->ubuf.clear();
        return ok;
    }
    if (!w->mt) {
        size_t n = w->ubuf.size();
        w->frame_uc = 0;
        bool ok = zstd_frame(w, w->ubuf.data(), n, call_data, errbuf);
        w->ubuf.clear();
        return ok;
    }
    size_t out_len = ZSTD_CStreamOutSize();
    w->cbuf.resize(out_len);
    ZSTD_inBuffer in = {nullptr, 0, 0};
    size_t rem;
    do {
        ZSTD_outBuffer out = {w->cbuf.data(), out_len, 0};
        rem = ZSTD_compressStream2(w->cctx, &out, &in, ZSTD_e_end);
        if (ZSTD_isError(rem)) {
            set_error(errbuf, "%s: %s", "compress", ZSTD_getErrorName(rem));
            return false;
        }
        w->frame_cm += out.pos;
        if (!emit(w, w->cbuf.data(), out.pos, call_data, errbuf))
            return false;
    } while (rem > 0);
    return log_frame(w, errbuf);
}

extern "C" ZSEEK_EXPORT bool zsk_writer_set_gpu_compress(zseek_writer_t *w, size_t batch_bytes)
{
    if (!w || w->type != ZSEEK_LZ4 || w->prefs.compressionLevel >= 3)
        return false;
    char err[ZSEEK_ERRBUF_SIZE];
    if (!gpu_flush(w, err))
        return false;
    w->gpu.release();
    if (batch_bytes == (size_t)-1)   // off
        return true;
    if (batch_bytes == 0)
        batch_bytes = kGpuDefaultBatch;
    batch_bytes = batch_bytes < kGpuMinBatch ? kGpuMinBatch : batch_bytes;
    GpuLz4 &g = w->gpu;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || hipGetDevice(&g.device) != hipSuccess) {
        g = GpuLz4();
        return false;
    }
    // staging is allocated at the first queued frame and grows with what is
    // queued (up to the batch); frames per flush are capped so the table
    // scratch (64 KiB per frame) stays within batch_bytes, whatever the
    // frame size
    g.batch_bytes = batch_bytes;
    g.max_frames = std::min(kGpuMaxBatchFrames, std::max<size_t>(16, batch_bytes / kGpuTableBytes));
    if (hip_stream_get(&g.stream, false) != hipSuccess) {
        g.release();
        return false;
    }
    return true;
}

extern "C" ZSEEK_EXPORT zseek_writer_t *zseek_writer_open_full(zseek_write_file_t user_file,
                                                               zseek_compression_param_t *zsp,
                                                               size_t min_frame_size,
                                                               void *call_data, char *errbuf)
{
    (void)call_data;
    zseek_compression_type_t type = zsp ? zsp->type : ZSEEK_ZSTD;   // ref :252-255
    if (type != ZSEEK_ZSTD && type != ZSEEK_LZ4) {
        set_error(errbuf, "wrong compression type (%d)", (int)type);
        return nullptr;
    }
    zseek_writer *w = new (std::nothrow) zseek_writer();
    if (!w) {
        set_error_errno(errbuf, "allocate writer", ENOMEM);
        return nullptr;
    }
    w->user_file = user_file;
    w->type = type;
    w->min_frame_size = min_frame_size;
    memset(&w->prefs, 0, sizeof(w->prefs));
    if (type == ZSEEK_LZ4) {
        // ref compress.c:203-207
        w->prefs.compressionLevel = zsp ? zsp->params.lz4_params.compression_level : 0;
        w->prefs.autoFlush = 1;
        w->prefs.frameInfo.blockSizeID = LZ4F_max64KB;
        w->ubuf.reserve(min_frame_size);
        if (const char *e = getenv("ZSEEK_GPU_COMPRESS")) {
            const unsigned long long v = strtoull(e, nullptr, 10);
            if (v)
                (void)zsk_writer_set_gpu_compress(w, v == 1 ? 0 : (size_t)v);
        }
        return w;
    }
    int level = zsp ? zsp->params.zstd_params.compression_level : ZSTD_CLEVEL_DEFAULT;
    int strategy = zsp ? zsp->params.zstd_params.strategy : (int)ZSTD_fast;
    w->cctx = ZSTD_createCCtx();
    if (!w->cctx) {
        set_error(errbuf, "context creation failed");
        delete w;
        return nullptr;
    }
    size_t r = ZSTD_CCtx_setParameter(w->cctx, ZSTD_c_compressionLevel, level);
    if (ZSTD_isError(r)) {
        set_error(errbuf, "%s: %s", "set compression level", ZSTD_getErrorName(r));
        goto fail;
    }
    r = ZSTD_CCtx_setParameter(w->cctx, ZSTD_c_strategy, strategy);
    if (ZSTD_isError(r)) {
        set_error(errbuf, "%s: %s", "set strategy", ZSTD_getErrorName(r));
        goto fail;
    }
    if (zsp && zsp->params.zstd_params.nb_workers > 1) {
        r = ZSTD_CCtx_setParameter(w->cctx, ZSTD_c_nbWorkers, zsp->params.zstd_params.nb_workers);
        if (ZSTD_isError(r)) {
            set_error(errbuf, "%s: %s", "set nb of workers", ZSTD_getErrorName(r));
            goto fail;
        }
        if (zsp->params.zstd_params.cpuset) {
            // create the worker pool while pinned to the caller's cpuset
            // (ref compress.c:105-139)
            pthread_t self = pthread_self();
            cpu_set_t prev;
            int pr = pthread_getaffinity_np(self, sizeof(prev), &prev);
            if (pr) {
                set_error_errno(errbuf, "get thread affinity", pr);
                goto fail;
            }
            pthread_setaffinity_np(self, zsp->params.zstd_params.cpusetsize,
                                   zsp->params.zstd_params.cpuset);
            ZSTD_inBuffer in = {nullptr, 0, 0};
            ZSTD_outBuffer out = {nullptr, 0, 0};
            r = ZSTD_compressStream2(w->cctx, &out, &in, ZSTD_e_continue);
            pthread_setaffinity_np(self, sizeof(prev), &prev);
            if (ZSTD_isError(r)) {
                set_error(errbuf, "%s: %s", "create threads", ZSTD_getErrorName(r));
                goto fail;
            }
        }
        w->mt = true;
    }
    w->ubuf.reserve(min_frame_size);
    return w;
fail:
    ZSTD_freeCCtx(w->cctx);
    delete w;
    return nullptr;
}

extern "C" ZSEEK_EXPORT zseek_writer_t *zseek_writer_open(FILE *cfile,
                                                          zseek_compression_param_t *zsp,
                                                          size_t min_frame_size, void *call_data,
                                                          char *errbuf)
{
    zseek_write_file_t uf = {cfile, default_write};
    return zseek_writer_open_full(uf, zsp, min_frame_size, call_data, errbuf);
}

static bool write_mt(zseek_writer *w, const void *buf, size_t len, void *call_data,
                     char *errbuf)
{
    // ref compress.c:599-648: end the previous frame lazily, then stream
    if (w->frame_uc >= w->min_frame_size && !end_frame(w, call_data, errbuf)) {
        set_error(errbuf, "end_frame_zstd failed");
        return false;
    }
    size_t out_len = ZSTD_compressBound(len);
    w->cbuf.resize(out_len);
    ZSTD_inBuffer in = {buf, len, 0};
    do {
        ZSTD_outBuffer out = {w->cbuf.data(), out_len, 0};
        size_t rem = ZSTD_compressStream2(w->cctx, &out, &in, ZSTD_e_continue);
        if (ZSTD_isError(rem)) {
            set_error(errbuf, "%s: %s", "compress", ZSTD_getErrorName(rem));
            return false;
        }
        w->frame_cm += out.pos;
        if (!emit(w, w->cbuf.data(), out.pos, call_data, errbuf))
            return false;
    } while (in.pos < in.size);
    w->frame_uc += len;
    return true;
}

extern "C" ZSEEK_EXPORT bool zseek_write(zseek_writer_t *w, const void *buf, size_t len,
                                         void *call_data, char *errbuf)
{
    if (!w) {
        set_error(errbuf, "invalid writer");
        return false;
    }
    if (w->type == ZSEEK_ZSTD && w->mt)
        return write_mt(w, buf, len, call_data, errbuf);
    if (w->ubuf.empty() && len >= w->min_frame_size) {
        // compress straight from the caller's buffer (ref :710-714, :791-795)
        return w->type == ZSEEK_LZ4 ? lz4_frame(w, buf, len, 0, call_data, errbuf)
                                    : zstd_frame(w, buf, len, call_data, errbuf);
    }
    if (len)
        w->ubuf.insert(w->ubuf.end(), (const uint8_t *)buf, (const uint8_t *)buf + len);
    w->frame_uc += len;
    if (w->frame_uc >= w->min_frame_size && !end_frame(w, call_data, errbuf)) {
        set_error(errbuf, w->type == ZSEEK_LZ4 ? "end_frame_lz4 failed" : "end_frame_zstd failed");
        return false;
    }
    return true;
}

static size_t seek_table_size(size_t frames)
{
    return 8 + 8 * frames + 9;
}

extern "C" ZSEEK_EXPORT bool zseek_writer_close(zseek_writer_t *w, void *call_data, char *errbuf)
{
    if (!w)
        return true;
    bool ok = true;
    if (w->frame_uc > 0 && !end_frame(w, call_data, errbuf)) {
        set_error(errbuf, w->type == ZSEEK_LZ4 ? "end_frame_lz4 failed" : "end_frame_zstd failed");
        ok = false;
    }
    if (ok && !gpu_flush(w, errbuf)) {
        set_error(errbuf, "end_frame_lz4 failed");
        ok = false;
    }
    w->gpu.release();
    // seekable-format seek table (ref seek_table.c:365-419): skippable
    // header, n x {cSize, dSize}, n, descriptor 0 (no checksums), magic
    std::vector<uint8_t> t(seek_table_size(w->log.size()));
    auto put32 = [&](size_t at, uint32_t v) {
        t[at] = (uint8_t)v;
        t[at + 1] = (uint8_t)(v >> 8);
        t[at + 2] = (uint8_t)(v >> 16);
        t[at + 3] = (uint8_t)(v >> 24);
    };
    put32(0, 0x184D2A5Eu);
    put32(4, (uint32_t)(t.size() - 8));
    size_t at = 8;
    for (const FrameLogEntry &e : w->log) {
        put32(at, e.c_size);
        put32(at + 4, e.d_size);
        at += 8;
    }
    put32(at, (uint32_t)w->log.size());
    t[at + 4] = 0;
    put32(at + 5, 0x8F92EAB1u);
    if (!w->user_file.write(t.data(), t.size(), w->user_file.user_data, call_data) && ok) {
        set_error(errbuf, "write to file failed");
        ok = false;
    }
    ZSTD_freeCCtx(w->cctx);
    delete w;
    return ok;
}

extern "C" ZSEEK_EXPORT bool zseek_writer_stats(zseek_writer_t *w, zseek_writer_stats_t *stats,
                                                char *errbuf)
{
    if (!w) {
        set_error(errbuf, "invalid writer");
        return false;
    }
    if (!stats) {
        set_error(errbuf, "invalid stats pointer");
        return false;
    }
    // queued GPU frames are written first, so the counts below include them
    if (!gpu_flush(w, errbuf))
        return false;
    // ref compress.c:835-881
    size_t frames = w->log.size() + (w->frame_uc > 0 ? 1 : 0);
    stats->seek_table_size = seek_table_size(w->log.size()) + (w->frame_uc > 0 ? 8 : 0);
    stats->seek_table_memory = sizeof(w->log) + w->log.capacity() * sizeof(FrameLogEntry);
    stats->frames = frames;
    stats->compressed_size = w->total_cm + w->frame_cm + stats->seek_table_size;
    size_t buffered = w->ubuf.capacity() + w->cbuf.capacity();
    if (w->type == ZSEEK_ZSTD)
        buffered += ZSTD_sizeof_CCtx(w->cctx);
    stats->buffer_size = buffered;
    return true;
}
