// host.h — host-side building blocks of the reader (internal).
#ifndef ZSK_HOST_H
#define ZSK_HOST_H

#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>
#include <functional>
#include <list>
#include <unordered_map>
#include <vector>

#include "../../include/zseek.h"
#include "zsk_internal.h"

namespace zsk {

// Error formatting (ref src/common.c:29-54): vsnprintf into an 80-byte
// caller buffer, no-op for NULL.
void set_error(char *errbuf, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void set_error_errno(char *errbuf, const char *msg, int errnum);

// In-memory seek table as prefix sums (ref src/seek_table.c:36-47, 62-110).
// SoA so a batch's descriptors are built with two subtractions per frame.
struct SeekTable {
    std::vector<uint64_t> c_off;   // n+1 entries, c_off[n] = total compressed
    std::vector<uint64_t> d_off;   // n+1 entries, d_off[n] = total decoded
    std::vector<uint32_t> checksum;   // n entries when the descriptor says so
    bool checksum_flag = false;

    size_t frames() const { return c_off.empty() ? 0 : c_off.size() - 1; }
    uint64_t decompressed_size() const { return d_off.empty() ? 0 : d_off.back(); }
    size_t memory_usage() const;
    // Frame holding decompressed offset, -1 past the end (ref :187-202).
    int64_t frame_of(uint64_t offset) const;
    uint64_t csize(size_t i) const { return c_off[i + 1] - c_off[i]; }
    uint64_t dsize(size_t i) const { return d_off[i + 1] - d_off[i]; }
};

// Parse the seekable-format footer/table through the user's callbacks with
// the reference's validation (ref src/seek_table.c:112-176).  false on any
// failure (the caller reports "read_seek_table failed").
bool read_seek_table(const zseek_read_file_t &uf, void *call_data, SeekTable *st);

// LRU of decoded frames keyed by frame index (ref src/cache.c): capacity in
// frames, find() promotes to MRU, insert() evicts the LRU when full and takes
// ownership of the frame bytes.
class FrameCache {
  public:
    explicit FrameCache(size_t capacity) : capacity_(capacity) {}
    ~FrameCache();
    // nullptr when absent; on hit *len = frame size.
    const uint8_t *find(size_t idx, size_t *len);
    bool contains(size_t idx) const { return map_.count(idx) != 0; }
    bool insert(size_t idx, uint8_t *data, size_t len);   // takes ownership
    size_t entries() const { return lru_.size(); }
    size_t memory_usage() const;
    size_t capacity() const { return capacity_; }

  private:
    struct Entry {
        size_t idx;
        uint8_t *data;
        size_t len;
    };
    size_t capacity_;
    size_t bytes_ = 0;
    std::list<Entry> lru_;   // front = LRU, back = MRU
    std::unordered_map<size_t, std::list<Entry>::iterator> map_;
};

// Keeps the calling thread's current HIP device across a library call: the
// reader switches to its own device (DeviceCtx::device) and this puts the
// caller's back on every return path.
struct DeviceGuard {
    int prev = -1;
    DeviceGuard()
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev)
            (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

// Host copies on a small process-wide worker pool (bounce buffer -> the
// caller's memory while the next batches read, upload and decode).  A ticket
// counts a batch's outstanding pieces.
struct CopyTicket {
    std::atomic<int> left{0};
};
int usable_cpus();          // affinity, capped by the cgroup CPU quota
int copy_pool_threads();    // the pool below: max(2, min(16, usable_cpus() - 2)), env ZSEEK_COPY_THREADS
void pool_copy(void *dst, const void *src, size_t n, CopyTicket *t);
void pool_run(std::function<void()> fn, CopyTicket *t);   // any task, same ticket rules
void pool_wait(CopyTicket *t);

// One batch of frames in flight: its own stream, pinned staging and device
// buffers (grown geometrically, kept across calls), decoder scratch.
struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;   // recorded after the batch's last command
    uint8_t *h_comp = nullptr;   // pinned: the batch's compressed span (user pread target), then its descriptors
    size_t h_comp_cap = 0;
    // pinned, per batch of n frames: n statuses, then n fail_at words (the
    // output offset of a failure), downloaded together
    int32_t *h_status = nullptr;
    size_t h_status_cap = 0;
    uint32_t *h_ck = nullptr;      // pinned: the batch's seek-table checksums
    size_t h_ck_cap = 0;
    uint8_t *h_out = nullptr;      // pinned bounce of decoded bytes (host destinations)
    size_t h_out_cap = 0;
    // the device mappings of h_comp, h_status, h_out (hipHostGetDevicePointer,
    // taken when they are allocated): small uploads and downloads as kernels
    void *h_comp_dev = nullptr, *h_status_dev = nullptr, *h_out_dev = nullptr;
    uint8_t *d_comp = nullptr;
    size_t d_comp_cap = 0;
    uint8_t *d_out = nullptr;
    size_t d_out_cap = 0;
    int32_t *d_status = nullptr;   // n statuses, then n fail_at words
    size_t d_status_cap = 0;
    uint32_t *d_ck = nullptr;
    size_t d_ck_cap = 0;
    SplitScratch split;   // two-phase LZ4 decoder scratch (lz4_split.hip)
    ZstdScratch zs;       // zstd decoder scratch (zstd_decode.hip)
    // the batch in flight
    size_t f0 = 0, f1 = 0;
    uint64_t h_from = 0, h_len = 0;   // batch-span bytes copied into h_out
    CopyTicket copies;                // h_out -> caller, still running
    // completion flag (download_flagged): the pinned word past the status
    // words (h_status's slack) that the batch's download sets to `seq`;
    // flagged: this batch posts it
    uint32_t seq = 0;
    bool flagged = false;
    volatile uint32_t *h_flag = nullptr;

    bool reserve(size_t comp, size_t out, size_t host_out, size_t nframes, bool ck, char *errbuf);
    void destroy();
    size_t device_bytes() const;
    size_t host_bytes() const;
};

// A reader's context on one device (a "lane"): kSlots batches in flight,
// created lazily at the first decode on that device.
constexpr int kSlots = 3;
struct DeviceCtx {
    int device = -1;
    Slot slot[kSlots];
    uint64_t batches = 0, frames_decoded = 0, bytes_decoded = 0, bytes_uploaded = 0;

    DeviceCtx() = default;
    DeviceCtx(const DeviceCtx &) = delete;
    DeviceCtx &operator=(const DeviceCtx &) = delete;
    ~DeviceCtx();
    bool init(int dev, char *errbuf);
    size_t device_bytes() const;
    size_t host_bytes() const;
};

// The devices a reader decodes on: env ZSEEK_HIP_DEVICES ("0,1,2,3"; a
// device may repeat), else ZSEEK_HIP_DEVICE, else the caller's current
// device.  Empty when no HIP device exists.
std::vector<int> default_devices();

}   // namespace zsk

#endif
