// pool.h — bounded, stream-ordered pools of decoder scratch for the device
// API (zsk_lz4_decode_frames / zsk_zstd_decode_frames), which has no reader
// to own scratch.  Internal.
//
// A set is reused in stream order: after a call's launches its event is
// recorded on the caller's stream; the next call (any stream) takes a set
// whose event has completed, or one last released on the same stream (stream
// order covers it), or a new set while the device has fewer than kPoolSets,
// or else the least recently released set after making its stream wait on
// that event.  Nothing is keyed by stream, so streams a caller destroys leave
// no entries behind, and a device never holds more than kPoolSets sets.
#ifndef ZSK_POOL_H
#define ZSK_POOL_H

#include <stdint.h>

#include <map>
#include <mutex>
#include <vector>

#include <hip/hip_runtime_api.h>

namespace zsk {

constexpr int kPoolSets = 4;

template <typename S>
class ScratchPool {
  public:
    // A free set for `stream` on the current device, nullptr when every set
    // is in use by a concurrent call (or on a HIP error).
    S *acquire(hipStream_t stream)
    {
        Dev *d = dev();
        std::lock_guard<std::mutex> g(d->mu);
        Set *pick = nullptr;
        for (Set *x : d->sets)   // same stream: ordered without a wait
            if (!x->busy && x->stream == stream) {
                pick = x;
                break;
            }
        for (size_t i = 0; !pick && i < d->sets.size(); i++)
            if (!d->sets[i]->busy && hipEventQuery(d->sets[i]->done) == hipSuccess)
                pick = d->sets[i];
        // hipEventQuery's hipErrorNotReady stays the thread's last error,
        // which the launchers' hipGetLastError checks would take for a
        // launch failure
        (void)hipGetLastError();
        if (!pick && (int)d->sets.size() < kPoolSets) {
            pick = new Set();
            if (hipEventCreateWithFlags(&pick->done, hipEventDisableTiming) != hipSuccess) {
                delete pick;
                return nullptr;
            }
            d->sets.push_back(pick);
        }
        if (!pick) {
            for (Set *x : d->sets)
                if (!x->busy && (!pick || x->last < pick->last))
                    pick = x;
            if (!pick || hipStreamWaitEvent(stream, pick->done, 0) != hipSuccess)
                return nullptr;
        }
        pick->busy = true;
        return &pick->s;
    }

    // The call's launches are queued on `stream`: the set is free once the
    // stream passes this point.
    void release(S *s, hipStream_t stream)
    {
        Dev *d = dev();
        std::lock_guard<std::mutex> g(d->mu);
        for (Set *x : d->sets)
            if (&x->s == s) {
                (void)hipEventRecord(x->done, stream);
                x->stream = stream;
                x->last = ++d->uses;
                x->busy = false;
                return;
            }
    }

  private:
    struct Set {
        S s;
        hipEvent_t done = nullptr;
        hipStream_t stream = nullptr;   // the stream of the last release
        uint64_t last = 0;
        bool busy = false;
    };
    struct Dev {
        std::mutex mu;
        std::vector<Set *> sets;
        uint64_t uses = 0;
    };
    Dev *dev()
    {
        int d = 0;
        (void)hipGetDevice(&d);
        std::lock_guard<std::mutex> g(mu_);
        Dev *&p = devs_[d];
        if (!p)
            p = new Dev();
        return p;
    }
    std::mutex mu_;
    std::map<int, Dev *> devs_;   // process lifetime, bounded per device
};

}   // namespace zsk

#endif
