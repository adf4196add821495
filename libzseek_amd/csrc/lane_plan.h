// Pure routing of a multi-frame zseek_pread over device lanes:
// which frames each lane decodes, and where a batch's decoded bytes go.  No
// HIP and no reader state, so tests/native/lane_plan_shim.cpp unit-tests every
// branch on the CPU; reader.cpp's run / submit use exactly these.
//
// Replaces the reference's serialised loop over a request's frames
// (decompress.c:714-718, one frame at a time into the caller's buffer).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace zsk {

// ---- lanes: a request [offset, end) over frames [f_first, f_last] ----------
// Contiguous frame shards split by decoded bytes, one per lane, each of at
// least per_lane bytes (and one frame); the last lane ends at f_last.
struct LaneShare {
    size_t fa, fb;   // frames [fa, fb)
};

template <class FrameOf>
std::vector<LaneShare> plan_lanes(size_t lanes, uint64_t offset, uint64_t end, size_t f_first, size_t f_last,
                                  uint64_t per_lane, FrameOf frame_of)
{
    const size_t nfr = f_last + 1 - f_first;
    size_t L = std::min<size_t>(lanes, std::max<uint64_t>(1, (end - offset) / std::max<uint64_t>(per_lane, 1)));
    L = std::max<size_t>(1, std::min(L, nfr));
    std::vector<LaneShare> out(L);
    size_t f = f_first;
    for (size_t i = 0; i < L; i++) {
        out[i].fa = f;
        if (i + 1 == L) {
            out[i].fb = f_last + 1;
        } else {
            const uint64_t cut = offset + (end - offset) * (i + 1) / L;
            out[i].fb = std::min(std::max((size_t)frame_of(cut), f + 1), f_last + 1 - (L - 1 - i));
        }
        f = out[i].fb;
    }
    return out;
}

// ---- one batch's decoded bytes ----------------------------------------------
enum CopyRoute : int {
    COPY_NONE = 0,      // the request needs none of the batch's bytes
    COPY_HOST = 1,      // host destination: download into the pinned bounce, pool copies to the caller
    COPY_DEVICE = 2,    // device destination on the lane's own device: one device-to-device copy
    COPY_PEER = 3,      // device destination on another device: one peer copy
};

struct BatchRoute {
    int route;           // CopyRoute of the request's bytes
    uint64_t dst_off;    // into the caller's buffer
    uint64_t src_off;    // from the batch's first decoded byte
    uint64_t len;        // the request's bytes in this batch
    uint64_t h_from;     // the pinned download: [h_from, h_from + h_len) of the batch
    uint64_t h_len;      //   (the request's bytes for a host destination, plus the
                         //   last cache_cap frames the cache may keep)
};

// Batch of frames [f0, f1) (decoded extents d_off[f0] .. d_off[f1]) of a
// request [offset, end); dst_dev / lane_dev for a device destination.
inline BatchRoute route_batch(bool device_dst, int dst_dev, int lane_dev, uint64_t offset, uint64_t end,
                              const uint64_t *d_off, size_t f0, size_t f1, size_t cache_cap)
{
    BatchRoute b{};
    const uint64_t d0 = d_off[f0];
    const uint64_t lo = std::max<uint64_t>(offset, d0), hi = std::min<uint64_t>(end, d_off[f1]);
    if (hi > lo) {
        b.route = !device_dst ? COPY_HOST : dst_dev == lane_dev ? COPY_DEVICE : COPY_PEER;
        b.dst_off = lo - offset;
        b.src_off = lo - d0;
        b.len = hi - lo;
    }
    uint64_t h_lo = UINT64_MAX, h_hi = 0;
    if (b.route == COPY_HOST) {
        h_lo = lo;
        h_hi = hi;
    }
    if (cache_cap) {
        const size_t cf = f1 - std::min(f1 - f0, cache_cap);
        h_lo = std::min<uint64_t>(h_lo, d_off[cf]);
        h_hi = std::max<uint64_t>(h_hi, d_off[f1]);
    }
    if (h_hi <= h_lo)
        h_lo = h_hi = d0;
    b.h_from = h_lo - d0;
    b.h_len = h_hi - h_lo;
    return b;
}

}   // namespace zsk
