// host_support.cpp — error buffers, seek table, decoded-frame LRU, GPU
// context.  Host C++ behind the C ABI of include/zseek.h.
#include <errno.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>

#include <hip/hip_runtime_api.h>

#include "host.h"

namespace zsk {

// ---------------------------------------------------------------------------
// errors (ref src/common.c:29-54)
// ---------------------------------------------------------------------------
void set_error(char *errbuf, const char *fmt, ...)
{
    if (!errbuf)
        return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(errbuf, ZSEEK_ERRBUF_SIZE, fmt, ap);
    va_end(ap);
}

void set_error_errno(char *errbuf, const char *msg, int errnum)
{
    char tmp[1024];
    const char *s = strerror_r(errnum, tmp, sizeof(tmp));   // GNU variant
    if (!msg || !*msg)
        set_error(errbuf, "%s", s);
    else
        set_error(errbuf, "%s: %s", msg, s);
}

// ---------------------------------------------------------------------------
// seek table (ref src/seek_table.c:15-23 constants, :62-176 parse)
// ---------------------------------------------------------------------------
namespace {
constexpr uint32_t kFooter = 9;
constexpr uint32_t kSeekMagic = 0x8F92EAB1u;
constexpr uint32_t kSkippableMagic = 0x184D2A5Eu;   // ZSTD_MAGIC_SKIPPABLE_START | 0xE
constexpr uint32_t kSkippableHdr = 8;
constexpr uint64_t kChunk = 1u << 20;   // entries read per callback (1 MiB)

inline uint32_t le32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
           ((uint32_t)p[3] << 24);
}
}   // namespace

size_t SeekTable::memory_usage() const
{
    return sizeof(*this) + c_off.capacity() * sizeof(uint64_t) +
           d_off.capacity() * sizeof(uint64_t) + checksum.capacity() * sizeof(uint32_t);
}

int64_t SeekTable::frame_of(uint64_t offset) const
{
    size_t n = frames();
    if (n == 0 || offset >= d_off[n])
        return -1;
    // last frame whose start is <= offset (same answer as the reference's
    // lo/hi bisection, including zero-size frames)
    size_t lo = 0, hi = n;
    while (lo + 1 < hi) {
        size_t mid = lo + (hi - lo) / 2;
        if (d_off[mid] <= offset)
            lo = mid;
        else
            hi = mid;
    }
    return (int64_t)lo;
}

bool read_seek_table(const zseek_read_file_t &uf, void *call_data, SeekTable *st)
{
    ssize_t fsize = uf.fsize(uf.user_data, call_data);
    if (fsize < (ssize_t)kFooter)
        return false;
    uint8_t footer[kFooter];
    if (uf.pread(footer, kFooter, (size_t)fsize - kFooter, uf.user_data, call_data) !=
        (ssize_t)kFooter)
        return false;
    if (le32(footer + 5) != kSeekMagic)
        return false;
    uint8_t desc = footer[4];
    if (desc & 0x7c)   // reserved descriptor bits
        return false;
    const bool ck = (desc & 0x80) != 0;
    const uint64_t n = le32(footer);
    const uint64_t esize = 8 + (ck ? 4 : 0);
    const uint64_t frame_size = kSkippableHdr + n * esize + kFooter;
    if (frame_size > (uint64_t)fsize)
        return false;
    const uint64_t table_at = (uint64_t)fsize - frame_size;
    uint8_t hdr[kSkippableHdr];
    if (uf.pread(hdr, kSkippableHdr, table_at, uf.user_data, call_data) !=
        (ssize_t)kSkippableHdr)
        return false;
    if (le32(hdr) != kSkippableMagic || le32(hdr + 4) != frame_size - kSkippableHdr)
        return false;

    st->checksum_flag = ck;
    st->c_off.assign(n + 1, 0);
    st->d_off.assign(n + 1, 0);
    st->checksum.assign(ck ? n : 0, 0);
    std::vector<uint8_t> buf;
    uint64_t c = 0, d = 0, pos = table_at + kSkippableHdr;
    for (uint64_t e = 0; e < n;) {
        uint64_t m = n - e < kChunk ? n - e : kChunk;
        buf.resize(m * esize);
        if (uf.pread(buf.data(), buf.size(), pos, uf.user_data, call_data) !=
            (ssize_t)buf.size())
            return false;
        pos += buf.size();
        const uint8_t *p = buf.data();
        for (uint64_t k = 0; k < m; k++, e++, p += esize) {
            st->c_off[e] = c;
            st->d_off[e] = d;
            c += le32(p);
            d += le32(p + 4);
            if (ck)
                st->checksum[e] = le32(p + 8);
        }
    }
    st->c_off[n] = c;
    st->d_off[n] = d;
    return true;
}

// ---------------------------------------------------------------------------
// decoded-frame LRU (ref src/cache.c:52-176)
// ---------------------------------------------------------------------------
FrameCache::~FrameCache()
{
    for (auto &e : lru_)
        free(e.data);
}

const uint8_t *FrameCache::find(size_t idx, size_t *len)
{
    auto it = map_.find(idx);
    if (it == map_.end())
        return nullptr;
    lru_.splice(lru_.end(), lru_, it->second);   // promote to MRU
    *len = it->second->len;
    return it->second->data;
}

bool FrameCache::insert(size_t idx, uint8_t *data, size_t len)
{
    if (capacity_ == 0)
        return false;
    auto it = map_.find(idx);
    if (it != map_.end()) {   // refresh an existing entry
        bytes_ -= it->second->len;
        free(it->second->data);
        it->second->data = data;
        it->second->len = len;
        bytes_ += len;
        lru_.splice(lru_.end(), lru_, it->second);
        return true;
    }
    if (lru_.size() == capacity_) {
        Entry &old = lru_.front();
        bytes_ -= old.len;
        free(old.data);
        map_.erase(old.idx);
        lru_.pop_front();
    }
    lru_.push_back(Entry{idx, data, len});
    map_[idx] = std::prev(lru_.end());
    bytes_ += len;
    return true;
}

size_t FrameCache::memory_usage() const
{
    // object + one list node and one hash node per entry + frame bytes
    return sizeof(*this) + lru_.size() * (sizeof(Entry) + 2 * sizeof(void *)) +
           map_.size() * (sizeof(size_t) + 3 * sizeof(void *)) + bytes_;
}

// ---------------------------------------------------------------------------
// CPUs this process may use: its affinity mask, capped by a cgroup CPU quota
// (v2 cpu.max, else v1 cfs_quota_us / cfs_period_us), rounded down, >= 1
int usable_cpus()
{
    static const int n = [] {
        cpu_set_t set;
        int aff = 0;
        if (sched_getaffinity(0, sizeof(set), &set) == 0)
            aff = CPU_COUNT(&set);
        if (aff <= 0)
            aff = (int)std::thread::hardware_concurrency();
        double quota = 0;
        if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {0};
            long long per = 0;
            if (fscanf(f, "%31s %lld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0)
                quota = atof(q) / (double)per;
            fclose(f);
        } else if (FILE *f1 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
            long long q = -1, per = 0;
            if (fscanf(f1, "%lld", &q) != 1)
                q = -1;
            fclose(f1);
            if (FILE *f2 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
                if (fscanf(f2, "%lld", &per) != 1)
                    per = 0;
                fclose(f2);
            }
            if (q > 0 && per > 0)
                quota = (double)q / (double)per;
        }
        int u = aff;
        if (quota > 0 && (int)quota < u)
            u = (int)quota;
        return u < 1 ? 1 : u;
    }();
    return n;
}

// copy pool: host memcpy on worker threads (process lifetime, never joined)
// ---------------------------------------------------------------------------
namespace {
constexpr size_t kCopyPiece = 4u << 20;    // bytes per task
constexpr size_t kCopyInline = 1u << 20;   // smaller copies run on the caller's thread

struct CopyTask {
    void *dst;
    const void *src;
    size_t n;
    CopyTicket *t;
    std::function<void()> fn;   // a task to run instead of the copy
};

class CopyPool {
  public:
    // one thread per usable CPU past two (the caller's thread and the HIP
    // runtime's), 2..16: the pool runs both the host copies out of the pinned
    // bounces and the concurrent pread callbacks (io_threads), so on a
    // 16-CPU cgroup quota it must not oversubscribe (round 4 sized it from
    // the 256 visible CPUs: 8 copy + 8 pread threads, and io8 ran slower than
    // io1 on a loaded box)
    CopyPool()
    {
        int n = usable_cpus() - 2;
        n = n < 2 ? 2 : n > 16 ? 16 : n;
        const char *env = getenv("ZSEEK_COPY_THREADS");
        if (env && *env && atoi(env) > 0)
            n = atoi(env);
        threads_ = n;
        for (int i = 0; i < n; i++)
            std::thread([this] { work(); }).detach();
    }
    int threads() const { return threads_; }
    void put(const CopyTask &t)
    {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(t);
        }
        cv_.notify_one();
    }
    void wait(CopyTicket *t)
    {
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [t] { return t->left.load() == 0; });
    }

  private:
    void work()
    {
        for (;;) {
            CopyTask t;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [this] { return !q_.empty(); });
                t = q_.front();
                q_.pop_front();
            }
            if (t.fn)
                t.fn();
            else
                memcpy(t.dst, t.src, t.n);
            if (t.t->left.fetch_sub(1) == 1) {
                std::lock_guard<std::mutex> g(mu_);
                done_.notify_all();
            }
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::deque<CopyTask> q_;
    int threads_ = 0;
};

CopyPool &copy_pool()
{
    static CopyPool *p = new CopyPool();   // never destroyed: its threads outlive exit
    return *p;
}
}   // namespace

int copy_pool_threads() { return copy_pool().threads(); }

void pool_copy(void *dst, const void *src, size_t n, CopyTicket *t)
{
    if (n <= kCopyInline) {
        memcpy(dst, src, n);
        return;
    }
    CopyPool &p = copy_pool();
    const size_t pieces = (n + kCopyPiece - 1) / kCopyPiece;
    t->left.fetch_add((int)pieces);
    for (size_t i = 0; i < pieces; i++) {
        const size_t o = i * kCopyPiece;
        p.put({(uint8_t *)dst + o, (const uint8_t *)src + o, n - o < kCopyPiece ? n - o : kCopyPiece, t, {}});
    }
}

void pool_run(std::function<void()> fn, CopyTicket *t)
{
    t->left.fetch_add(1);
    copy_pool().put({nullptr, nullptr, 0, t, std::move(fn)});
}

void pool_wait(CopyTicket *t)
{
    if (t->left.load() != 0)
        copy_pool().wait(t);
}

// ---------------------------------------------------------------------------
// HIP stream / event recycling (process lifetime; see zsk_internal.h)
// ---------------------------------------------------------------------------
namespace {
struct HandlePool {
    std::mutex mu;
    // free handles per (device, kind); kind 0 = stream, 1 = low-priority
    // stream, 2 = event; owner[] remembers each handle's key
    std::unordered_map<uint64_t, std::vector<void *>> free_;
    std::unordered_map<void *, uint64_t> owner;
};
HandlePool &handle_pool()
{
    static HandlePool *p = new HandlePool();   // never destroyed, like the handles
    return *p;
}
uint64_t handle_key(int kind)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    return (uint64_t)(uint32_t)dev << 8 | (uint32_t)kind;
}
void *handle_take(uint64_t key)
{
    HandlePool &p = handle_pool();
    std::lock_guard<std::mutex> g(p.mu);
    auto it = p.free_.find(key);
    if (it == p.free_.end() || it->second.empty())
        return nullptr;
    void *h = it->second.back();
    it->second.pop_back();
    return h;
}
void handle_note(void *h, uint64_t key)
{
    HandlePool &p = handle_pool();
    std::lock_guard<std::mutex> g(p.mu);
    p.owner[h] = key;
}
void handle_give(void *h)
{
    HandlePool &p = handle_pool();
    std::lock_guard<std::mutex> g(p.mu);
    auto it = p.owner.find(h);
    if (it != p.owner.end())
        p.free_[it->second].push_back(h);
}
}   // namespace

hipError_t hip_stream_get(hipStream_t *s, bool low)
{
    const uint64_t key = handle_key(low ? 1 : 0);
    if ((*s = (hipStream_t)handle_take(key)) != nullptr)
        return hipSuccess;
    hipError_t e;
    if (low) {
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        e = hipStreamCreateWithPriority(s, hipStreamNonBlocking, lo);
    } else {
        e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    }
    if (e == hipSuccess)
        handle_note(*s, key);
    return e;
}

// Streams and events are destroyed when released.  Env ZSEEK_HIP_POOL=1
// keeps them in the process-wide pool instead (round 3's workaround, kept as
// the control arm of scripts/hang_probe.py; see DESIGN.md §7 "Teardown").
static bool hip_destroy_handles()
{
    static const bool on = [] {
        const char *v = getenv("ZSEEK_HIP_POOL");
        return !(v && !strcmp(v, "1"));
    }();
    return on;
}

void hip_stream_put(hipStream_t s)
{
    if (s && hip_destroy_handles())
        (void)hipStreamDestroy(s);
    else if (s)
        handle_give(s);
}

hipError_t hip_event_get(hipEvent_t *ev)
{
    const uint64_t key = handle_key(2);
    if ((*ev = (hipEvent_t)handle_take(key)) != nullptr)
        return hipSuccess;
    const hipError_t e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (e == hipSuccess)
        handle_note(*ev, key);
    return e;
}

void hip_event_put(hipEvent_t e)
{
    if (e && hip_destroy_handles())
        (void)hipEventDestroy(e);
    else if (e)
        handle_give(e);
}

// ---------------------------------------------------------------------------
// GPU context: a lane of kSlots batch slots on one device
// ---------------------------------------------------------------------------
namespace {
template <typename T>
bool grow_dev(T **p, size_t *cap, size_t want_elems)
{
    if (want_elems <= *cap)
        return true;
    size_t n = *cap * 2 > want_elems ? *cap * 2 : want_elems;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    // +256 B: readable tail for the 4-byte-granular input window
    if (hipMalloc((void **)p, n * sizeof(T) + 256) != hipSuccess)
        return false;
    *cap = n;
    return true;
}

template <typename T>
bool grow_host(T **p, size_t *cap, size_t want_elems)
{
    if (want_elems <= *cap)
        return true;
    size_t n = *cap * 2 > want_elems ? *cap * 2 : want_elems;
    (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipHostMalloc((void **)p, n * sizeof(T) + 256, hipHostMallocDefault) != hipSuccess)
        return false;
    *cap = n;
    return true;
}
}   // namespace

bool Slot::reserve(size_t comp, size_t out, size_t host_out, size_t nframes, bool ck, char *errbuf)
{
    if (!grow_dev(&d_comp, &d_comp_cap, comp) || !grow_dev(&d_out, &d_out_cap, out) ||
        !grow_dev(&d_status, &d_status_cap, 2 * nframes) ||
        (ck && !grow_dev(&d_ck, &d_ck_cap, nframes))) {
        set_error(errbuf, "allocate GPU decode buffers failed");
        return false;
    }
    const void *const c0 = h_comp, *const s0 = h_status, *const o0 = h_out;
    if (!grow_host(&h_comp, &h_comp_cap, comp) ||
        !grow_host(&h_status, &h_status_cap, 2 * nframes) ||
        (ck && !grow_host(&h_ck, &h_ck_cap, nframes)) ||
        (host_out && !grow_host(&h_out, &h_out_cap, host_out))) {
        set_error(errbuf, "allocate pinned staging failed");
        return false;
    }
    // (re)allocated: their device mappings (none: the copies go by DMA)
    auto map = [](void *h, void **dev) {
        *dev = nullptr;
        if (h && hipHostGetDevicePointer(dev, h, 0) != hipSuccess)
            *dev = nullptr;
    };
    if (h_comp != c0 || (h_comp && !h_comp_dev))
        map(h_comp, &h_comp_dev);
    if (h_status != s0 || (h_status && !h_status_dev))
        map(h_status, &h_status_dev);
    if (h_out != o0 || (h_out && !h_out_dev))
        map(h_out, &h_out_dev);
    return true;
}

// Teardown order: every stream drained (the slot's, its host copies, the
// zstd scratch's side streams); then all memory, while every stream that used
// it still exists; then the streams and the events recorded on them go back
// go (hip_stream_put / hip_event_put destroy them).  Rounds 2-3 saw the host
// heap corrupted under reader churn; the cause was the compiled reference's
// libzstd 1.4.9 sharing one link namespace with the system libzstd in test
// processes, not HIP object lifetimes (DESIGN.md §7 "Teardown").
void Slot::destroy()
{
    if (!stream)
        return;
    (void)hipStreamSynchronize(stream);
    pool_wait(&copies);
    zstd_scratch_release_memory(&zs);
    split_scratch_free(&split);
    for (void *p : {(void *)d_comp, (void *)d_out, (void *)d_status, (void *)d_ck})
        if (p)
            (void)hipFree(p);
    for (void *p : {(void *)h_comp, (void *)h_status, (void *)h_ck, (void *)h_out})
        if (p)
            (void)hipHostFree(p);
    zstd_scratch_drop_streams(&zs);
    hip_stream_put(stream);
    hip_event_put(done);
    zstd_scratch_free(&zs);   // its events (its memory and streams are gone)
    stream = nullptr;
    done = nullptr;
    h_comp = h_out = nullptr;
    h_status = nullptr;
    h_ck = nullptr;
    h_comp_dev = h_status_dev = h_out_dev = nullptr;
    d_comp = d_out = nullptr;
    d_status = nullptr;
    d_ck = nullptr;
    h_comp_cap = h_status_cap = h_ck_cap = h_out_cap = 0;
    d_comp_cap = d_out_cap = d_status_cap = d_ck_cap = 0;
}

size_t Slot::device_bytes() const
{
    return d_comp_cap + d_out_cap + (d_status_cap + d_ck_cap) * 4 +
           split.frames_cap * 12 + split.items_cap * 8 + zs.frames_cap * 24 + zs.lit_cap + zs.items_cap * 8;
}

size_t Slot::host_bytes() const
{
    return h_comp_cap + h_out_cap + (h_status_cap + h_ck_cap) * 4;
}

DeviceCtx::~DeviceCtx()
{
    if (device < 0)
        return;
    DeviceGuard keep;
    (void)hipSetDevice(device);
    for (Slot &s : slot)
        s.destroy();
}

bool DeviceCtx::init(int dev, char *errbuf)
{
    if (device >= 0)
        return true;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        set_error(errbuf, "no HIP device available");
        return false;
    }
    if (dev < 0 || dev >= count || hipSetDevice(dev) != hipSuccess) {
        set_error(errbuf, "invalid HIP device %d", dev);
        return false;
    }
    for (Slot &s : slot) {
        if (hip_stream_get(&s.stream, false) != hipSuccess || hip_event_get(&s.done) != hipSuccess) {
            set_error(errbuf, "create HIP stream failed");
            for (Slot &t : slot)
                t.destroy();
            return false;
        }
    }
    device = dev;
    return true;
}

size_t DeviceCtx::device_bytes() const
{
    size_t n = 0;
    for (const Slot &s : slot)
        n += s.device_bytes();
    return n;
}

size_t DeviceCtx::host_bytes() const
{
    size_t n = 0;
    for (const Slot &s : slot)
        n += s.host_bytes();
    return n;
}

std::vector<int> default_devices()
{
    std::vector<int> out;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return out;
    const char *list = getenv("ZSEEK_HIP_DEVICES");
    if (list && *list) {
        const char *p = list;
        while (*p) {
            char *e = nullptr;
            long v = strtol(p, &e, 10);
            if (e == p)
                break;
            out.push_back((int)v);
            p = *e == ',' ? e + 1 : e;
            if (*e != ',' )
                break;
        }
        if (!out.empty())
            return out;
    }
    int dev = 0;
    const char *one = getenv("ZSEEK_HIP_DEVICE");
    if (one && *one)
        dev = atoi(one);
    else if (hipGetDevice(&dev) != hipSuccess)
        dev = 0;
    out.push_back(dev);
    return out;
}

// ---------------------------------------------------------------------------
// status names (LZ4F_getErrorName strings of liblz4 1.9.3 for 1..19)
// ---------------------------------------------------------------------------
// ZSTD_getErrorName strings of libzstd 1.4.9 (zstd_errors.h codes)
static const char *zstd_name(int32_t code)
{
    switch (code) {
    case 1: return "Error (generic)";
    case 10: return "Unknown frame descriptor";
    case 12: return "Version not supported";
    case 14: return "Unsupported frame parameter";
    case 16: return "Frame requires too much memory for decoding";
    case 20: return "Corrupted block detected";
    case 22: return "Restored data doesn't match checksum";
    case 30: return "Dictionary is corrupted";
    case 32: return "Dictionary mismatch";
    case 44: return "tableLog requires too much memory : unsupported";
    case 46: return "Unsupported max Symbol Value : too large";
    case 48: return "Specified maxSymbolValue is too small";
    case 70: return "Destination buffer is too small";
    case 72: return "Src size is incorrect";
    default: return "Unspecified error code";
    }
}

const char *status_name(int32_t st)
{
    if (st & ST_ZSTD_FLAG)
        return zstd_name(st & 0xFFFF);
    static const char *const names[] = {
        "OK_NoError", "ERROR_GENERIC", "ERROR_maxBlockSize_invalid",
        "ERROR_blockMode_invalid", "ERROR_contentChecksumFlag_invalid",
        "ERROR_compressionLevel_invalid", "ERROR_headerVersion_wrong",
        "ERROR_blockChecksum_invalid", "ERROR_reservedFlag_set",
        "ERROR_allocation_failed", "ERROR_srcSize_tooLarge",
        "ERROR_dstMaxSize_tooSmall", "ERROR_frameHeader_incomplete",
        "ERROR_frameType_unknown", "ERROR_frameSize_wrong", "ERROR_srcPtr_wrong",
        "ERROR_decompressionFailed", "ERROR_headerChecksum_invalid",
        "ERROR_contentChecksum_invalid", "ERROR_frameDecoding_alreadyStarted",
    };
    int32_t code = st & 0xFFFF;
    if (code >= 0 && code < (int32_t)(sizeof(names) / sizeof(names[0])))
        return names[code];
    switch (code) {
    case ST_DST_OVERFLOW:
        return "decoded data exceeds frame size";
    case ST_SHORT_FRAME:
        return "decoded data shorter than frame size";
    case ST_TRUNCATED:
        return "truncated frame";
    case ST_UNSUPPORTED:
        return "unsupported frame";
    case ST_SEEK_CHECKSUM:
        return "frame checksum mismatch";
    case ST_NOT_RUN:
        return "decoder did not run";
    default:
        return "Unspecified error code";
    }
}

}   // namespace zsk
