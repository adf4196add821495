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
//   cache every decoded frame               cache the last cache_size frames of
//                                           the request (same final LRU state
//                                           as the reference's call loop)
//
// A corrupt frame inside a range makes the call return the bytes before it
// (a short read); the next call, starting at that frame, returns -1 with the
// error string the reference would produce — the same observable sequence a
// caller looping on the reference sees.
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <mutex>
#include <map>
#include <new>
#include <utility>

#include <hip/hip_runtime_api.h>

#include "../../include/zseek_hip.h"
#include "host.h"

using namespace zsk;

namespace {
constexpr uint32_t kZstdMagic = 0xFD2FB528u;   // ref decompress.c:22
constexpr uint32_t kLz4Magic = 0x184D2204u;    // ref decompress.c:23
constexpr size_t kDefaultBatch = 256u << 20;
}   // namespace

struct zseek_reader {
    zseek_read_file_t user_file;
    zseek_compression_type_t type;
    std::mutex lock;   // serialises decode + cache (ref uses a rwlock, :38)
    SeekTable st;
    FrameCache *cache = nullptr;   // NULL when cache_size == 0 (ref :219-227)
    std::mutex cursor_lock;        // zseek_read: cursor read, pread, advance as one step
    size_t pos = 0;                // zseek_read cursor (ref :826-835)
    size_t batch_bytes = kDefaultBatch;
    bool verify = false;   // check seek-table frame checksums (the reference never does)
    DeviceCtx gpu;
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
    delete reader;
    return true;
}

// ---------------------------------------------------------------------------
// GPU batch decode: frames [f0, f1) -> gpu.d_out (frame i at d_off[i]-d_off[f0])
// ---------------------------------------------------------------------------
namespace {

struct BatchResult {
    size_t first_bad;   // == f1 when every frame decoded
    int32_t status;
    uint32_t fail_at;   // output offset (within the frame) of the failure
};

bool read_span(zseek_reader *r, void *dst, size_t len, uint64_t off, void *call_data,
               char *errbuf)
{
    ssize_t got = r->user_file.pread(dst, len, off, r->user_file.user_data, call_data);
    if (got != (ssize_t)len) {
        // ref decompress.c:735-741
        set_error(errbuf, got >= 0 ? "unexpected EOF" : "read file failed");
        return false;
    }
    return true;
}

bool gpu_decode(zseek_reader *r, size_t f0, size_t f1, void *call_data, char *errbuf,
                BatchResult *res)
{
    DeviceCtx &g = r->gpu;
    if (!g.init(errbuf))
        return false;
    const SeekTable &st = r->st;
    const size_t n = f1 - f0;
    const uint64_t c0 = st.c_off[f0], csz = st.c_off[f1] - c0;
    const uint64_t d0 = st.d_off[f0], dsz = st.d_off[f1] - d0;
    if (!g.reserve(csz, dsz, n, errbuf))
        return false;
    if (csz && !read_span(r, g.h_comp, csz, c0, call_data, errbuf))
        return false;
    for (size_t i = 0; i < n; i++) {
        FrameDesc &d = g.h_desc[i];
        d.c_off = st.c_off[f0 + i] - c0;
        d.d_off = st.d_off[f0 + i] - d0;
        d.c_size = (uint32_t)st.csize(f0 + i);
        d.d_size = (uint32_t)st.dsize(f0 + i);
    }
    (void)hipSetDevice(g.device);
    hipError_t e = hipSuccess;
    if (csz)
        e = hipMemcpyAsync(g.d_comp, g.h_comp, csz, hipMemcpyHostToDevice, g.stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(g.d_desc, g.h_desc, n * sizeof(FrameDesc), hipMemcpyHostToDevice,
                           g.stream);
    if (e == hipSuccess)
        e = hipMemsetD32Async((hipDeviceptr_t)g.d_status, ST_NOT_RUN, n, g.stream);
    if (r->type == ZSEEK_ZSTD) {
        // zstd: plan + decode (zstd_decode.hip); a failure's output offset is
        // its block's start (the frame's end for the end-of-frame checks)
        if (e == hipSuccess)
            e = hipMemsetD32Async((hipDeviceptr_t)g.d_fail, 0, n, g.stream);
        if (e == hipSuccess && zstd_decode_frames(g.d_desc, (uint32_t)n, g.d_comp, g.d_out,
                                                  g.d_status, &g.zs, g.stream, g.d_fail) != 0)
            e = hipErrorLaunchFailure;
    }
    const int engine = r->type == ZSEEK_ZSTD ? -1 : lz4_pick_engine((uint32_t)n);
    if (e == hipSuccess && engine == ENGINE_WAVE &&
        launch_lz4_wave(g.d_desc, (uint32_t)n, g.d_comp, g.d_out, g.d_status, g.d_fail, g.stream) != 0)
        e = hipErrorLaunchFailure;
    if (e == hipSuccess && engine == ENGINE_SPLIT &&
        split_scratch_reserve(&g.split, (uint32_t)n, split_items_needed(g.h_desc, (uint32_t)n),
                              g.stream) != 0)
        e = hipErrorOutOfMemory;
    if (e == hipSuccess && engine == ENGINE_SPLIT &&
        launch_lz4_split(g.d_desc, (uint32_t)n, g.d_comp, g.d_out, g.d_status, g.d_fail,
                         g.stream, &g.split) != 0)
        e = hipErrorLaunchFailure;
    // seek-table checksums (descriptor bit 7) when asked for: XXH64 low 32
    // bits of every decoded frame, on the GPU (frame_check.hip)
    if (e == hipSuccess && r->verify && st.checksum_flag) {
        e = hipMemcpyAsync(g.d_ck, st.checksum.data() + f0, n * sizeof(uint32_t),
                           hipMemcpyHostToDevice, g.stream);
        if (e == hipSuccess &&
            launch_frame_checksums(g.d_desc, (uint32_t)n, g.d_out, g.d_ck, g.d_status, g.stream) != 0)
            e = hipErrorLaunchFailure;
    }
    if (e == hipSuccess)
        e = hipMemcpyAsync(g.h_status, g.d_status, n * sizeof(int32_t), hipMemcpyDeviceToHost,
                           g.stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(g.h_fail, g.d_fail, n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           g.stream);
    if (e == hipSuccess)
        e = hipStreamSynchronize(g.stream);
    if (e != hipSuccess) {
        set_error(errbuf, "GPU decode failed: %s", hipGetErrorString(e));
        return false;
    }
    g.batches++;
    g.frames_decoded += n;
    g.bytes_decoded += dsz;
    g.bytes_uploaded += csz;
    res->first_bad = f1;
    res->status = ST_OK;
    res->fail_at = 0;
    for (size_t i = 0; i < n; i++) {
        if (g.h_status[i] != ST_OK) {
            res->first_bad = f0 + i;
            res->status = g.h_status[i];
            res->fail_at = g.h_fail[i];
            break;
        }
    }
    return true;
}

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
void frame_error(zseek_reader *r, const BatchResult &br, size_t frame, size_t offset_in_frame,
                 size_t count, char *errbuf)
{
    const int32_t st = br.status;
    const uint64_t dsize = r->st.dsize(frame);
    const uint64_t at = br.fail_at;
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

bool copy_out(DeviceCtx &g, void *dst, uint64_t src_off, size_t len, bool device_dst,
              char *errbuf)
{
    if (!len)
        return true;
    hipError_t e = hipMemcpyAsync(dst, g.d_out + src_off, len,
                                  device_dst ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                  g.stream);
    if (e == hipSuccess)
        e = hipStreamSynchronize(g.stream);
    if (e != hipSuccess) {
        set_error(errbuf, "copy decoded data failed: %s", hipGetErrorString(e));
        return false;
    }
    return true;
}

// Insert frames [a, b) of the current batch (batch starts at frame f0) into
// the cache, MRU last.
bool cache_frames(zseek_reader *r, size_t f0, size_t a, size_t b, char *errbuf)
{
    const SeekTable &st = r->st;
    for (size_t i = a; i < b; i++) {
        size_t len = st.dsize(i);
        uint8_t *p = (uint8_t *)malloc(len ? len : 1);
        if (!p) {
            set_error_errno(errbuf, "allocate decompressed buffer", errno);
            return false;
        }
        if (!copy_out(r->gpu, p, st.d_off[i] - st.d_off[f0], len, false, errbuf)) {
            free(p);
            return false;
        }
        if (!r->cache->insert(i, p, len)) {
            free(p);
            set_error(errbuf, "frame caching failed");
            return false;
        }
    }
    return true;
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
    std::lock_guard<std::mutex> guard(r->lock);
    DeviceGuard keep_device;   // the caller's current device is restored on return
    const size_t f_first = (size_t)fi;
    const uint64_t end = offset + count < st.decompressed_size() ? offset + count
                                                                 : st.decompressed_size();

    // single-frame request with a cache: the reference's cached path
    // (decompress.c:699-796), GPU-decoded on a miss
    if (r->cache && (count == 0 || (size_t)st.frame_of(end - 1) == f_first)) {
        size_t len = 0;
        const uint8_t *data = r->cache->find(f_first, &len);
        if (!data) {
            BatchResult br;
            if (!gpu_decode(r, f_first, f_first + 1, call_data, errbuf, &br))
                return -1;
            if (br.first_bad != f_first + 1) {
                frame_error(r, br, f_first, offset - st.d_off[f_first], count, errbuf);
                return -1;
            }
            if (!cache_frames(r, f_first, f_first, f_first + 1, errbuf))
                return -1;
            data = r->cache->find(f_first, &len);
        }
        size_t rel = offset - st.d_off[f_first];
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
    if (count == 0)
        return 0;

    // multi-frame (or no-cache) request: batches of whole frames, one grid each
    const size_t f_last = (size_t)st.frame_of(end - 1);
    size_t done = 0;
    size_t f = f_first;
    while (f <= f_last) {
        // grow the batch up to batch_bytes of decoded data (at least 1 frame)
        size_t g_end = f + 1;
        while (g_end <= f_last && st.d_off[g_end + 1] - st.d_off[f] <= r->batch_bytes)
            g_end++;
        BatchResult br;
        if (!gpu_decode(r, f, g_end, call_data, errbuf, &br))
            return done ? (ssize_t)done : -1;
        const uint64_t lo = offset > st.d_off[f] ? offset : st.d_off[f];
        uint64_t good_end = br.first_bad < g_end ? st.d_off[br.first_bad] : st.d_off[g_end];
        // Without a cache the reference decodes a frame only as far as the
        // request reaches (lz4_partial_ok, zstd_partial_ok).
        if (br.first_bad < g_end && !r->cache &&
            (r->type == ZSEEK_LZ4 ? lz4_partial_ok(br.status, br.fail_at, end - st.d_off[br.first_bad])
                                  : zstd_partial_ok(br.status, br.fail_at, end - st.d_off[br.first_bad])))
            good_end = end;
        const uint64_t hi = end < good_end ? end : good_end;
        if (hi > lo) {
            if (!copy_out(r->gpu, (uint8_t *)buf + (lo - offset), lo - st.d_off[f], hi - lo,
                          device_dst, errbuf))
                return done ? (ssize_t)done : -1;
            done += hi - lo;
        }
        if (br.first_bad < g_end && good_end < end) {
            if (done)
                return (ssize_t)done;   // short read up to the corrupt frame
            frame_error(r, br, br.first_bad, offset - st.d_off[br.first_bad], count, errbuf);
            return -1;
        }
        // the cache ends as a reference caller's looping frame by frame over
        // the range would leave it: the range's last `capacity` frames, MRU
        // last, inserted batch by batch before the batch buffer is reused
        if (r->cache) {
            const size_t cap = r->cache->capacity();
            const size_t keep_from = f_last + 1 > cap ? f_last + 1 - cap : 0;
            const size_t a = keep_from > f ? keep_from : f;
            if (a < g_end && !cache_frames(r, f, a, g_end, errbuf))
                return (ssize_t)done;
        }
        f = g_end;
    }
    return (ssize_t)done;
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
    std::lock_guard<std::mutex> guard(reader->lock);
    stats->seek_table_memory = reader->st.memory_usage();
    stats->frames = reader->st.frames();
    stats->decompressed_size = reader->st.decompressed_size();
    stats->cache_memory = reader->cache ? reader->cache->memory_usage() : 0;
    stats->cached_frames = reader->cache ? reader->cache->entries() : 0;
    size_t buffered = reader->gpu.host_bytes();
    stats->buffer_size = buffered;
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
    if (decoder < ZSK_DECODER_AUTO || decoder > ZSK_DECODER_CHUNK)
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

extern "C" ZSEEK_EXPORT int zsk_zstd_decode_frames(const zsk_frame_desc_t *d_desc,
                                                   uint32_t nframes, const void *d_comp,
                                                   void *d_out, int32_t *d_status, void *stream)
{
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, ZstdScratch> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    ZstdScratch &s = cache[{dev, static_cast<hipStream_t>(stream)}];
    return zsk::zstd_decode_frames(reinterpret_cast<const FrameDesc *>(d_desc), nframes,
                                   static_cast<const uint8_t *>(d_comp),
                                   static_cast<uint8_t *>(d_out), d_status, &s,
                                   static_cast<hipStream_t>(stream));
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

extern "C" ZSEEK_EXPORT bool zsk_reader_gpu_stats(zseek_reader_t *reader, zsk_gpu_stats_t *s)
{
    if (!reader || !s)
        return false;
    std::lock_guard<std::mutex> guard(reader->lock);
    const DeviceCtx &g = reader->gpu;
    s->batches = g.batches;
    s->frames_decoded = g.frames_decoded;
    s->bytes_decoded = g.bytes_decoded;
    s->bytes_uploaded = g.bytes_uploaded;
    s->device_memory = g.device_bytes();
    s->device = g.device;
    return true;
}

extern "C" ZSEEK_EXPORT bool zsk_reader_set_batch_bytes(zseek_reader_t *reader, size_t bytes)
{
    if (!reader || bytes < 4096)
        return false;
    std::lock_guard<std::mutex> guard(reader->lock);
    reader->batch_bytes = bytes;
    return true;
}

// Seek-table checksum verification switch (zseek_hip.h).
extern "C" ZSEEK_EXPORT bool zsk_reader_set_verify_checksums(zseek_reader_t *reader, bool on)
{
    if (!reader)
        return false;
    std::lock_guard<std::mutex> guard(reader->lock);
    reader->verify = on;
    return true;
}
