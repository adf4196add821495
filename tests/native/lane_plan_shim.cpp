// Test-only C shim over libzseek_amd/csrc/lane_plan.h (pure functions, no
// HIP): tests/test_lane_plan.py builds it with g++ and calls it via ctypes.
#include "../../libzseek_amd/csrc/lane_plan.h"

#include <algorithm>

extern "C" {

// frames are given by their decoded offsets d_off[0..nframes]; returns the
// number of lanes and writes their [fa, fb) into fa / fb
size_t lp_plan_lanes(size_t lanes, uint64_t offset, uint64_t end, const uint64_t *d_off, size_t nframes,
                     uint64_t per_lane, size_t *fa, size_t *fb)
{
    auto frame_of = [&](uint64_t x) -> size_t {   // the frame holding byte x
        return (size_t)(std::upper_bound(d_off, d_off + nframes + 1, x) - d_off) - 1;
    };
    const size_t f_first = frame_of(offset), f_last = frame_of(end - 1);
    const auto v = zsk::plan_lanes(lanes, offset, end, f_first, f_last, per_lane, frame_of);
    for (size_t i = 0; i < v.size(); i++) {
        fa[i] = v[i].fa;
        fb[i] = v[i].fb;
    }
    return v.size();
}

// out: route, dst_off, src_off, len, h_from, h_len
void lp_route_batch(int device_dst, int dst_dev, int lane_dev, uint64_t offset, uint64_t end, const uint64_t *d_off,
                    size_t f0, size_t f1, size_t cache_cap, uint64_t *out)
{
    const zsk::BatchRoute b = zsk::route_batch(device_dst != 0, dst_dev, lane_dev, offset, end, d_off, f0, f1,
                                               cache_cap);
    out[0] = (uint64_t)b.route;
    out[1] = b.dst_off;
    out[2] = b.src_off;
    out[3] = b.len;
    out[4] = b.h_from;
    out[5] = b.h_len;
}
}
