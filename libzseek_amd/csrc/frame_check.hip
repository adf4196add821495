// frame_check.hip — seek-table frame checksums verified on the GPU (gfx950).
//
// The seekable format's per-frame checksum (descriptor bit 7) is the low 32
// bits of XXH64(seed 0) of the frame's decompressed bytes; the reference
// parses it (src/seek_table.c:95-97, seekEntry_t.checksum :36-40; writer
// :392-396) and never checks it.  Here it is checked over the decoded frames
// already in HBM, after the decode grid, on the same stream.
//
// Mapping: four lanes per frame, one per XXH64 accumulator (16 frames per
// wave).  Lane k of a frame reads 8-byte word k of each 32-byte stripe, so a
// frame's four lanes together read consecutive 32-byte stripes and each line
// they touch is consumed whole over four consecutive stripes; four stripes'
// loads are issued before the dependent rounds.  The tail (< 32 bytes) and
// the avalanche run on the frame's lane 0, serially, as XXH64 defines them.
// Algorithmic bytes per frame: d_size read once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zseek_hip.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

constexpr uint64_t P1 = 0x9E3779B185EBCA87ull;
constexpr uint64_t P2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t P3 = 0x165667B19E3779F9ull;
constexpr uint64_t P4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t P5 = 0x27D4EB2F165667C5ull;

typedef uint64_t u64_ua __attribute__((aligned(1)));
typedef uint32_t u32_ua __attribute__((aligned(1)));

__device__ __forceinline__ uint64_t rotl(uint64_t x, int r)
{
    return (x << r) | (x >> (64 - r));
}

__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t v)
{
    acc += v * P2;
    return rotl(acc, 31) * P1;
}

__device__ __forceinline__ uint64_t xmerge(uint64_t h, uint64_t v)
{
    h ^= xround(0, v);
    return h * P1 + P4;
}

__device__ __forceinline__ uint64_t ld8(const uint8_t *p)
{
    return *reinterpret_cast<const u64_ua *>(p);
}

__global__ __launch_bounds__(256) void frame_xxh64_kernel(const FrameDesc *__restrict__ desc, uint32_t n,
                                                          const uint8_t *__restrict__ out,
                                                          const uint32_t *__restrict__ want,
                                                          int32_t *__restrict__ status)
{
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    const uint32_t f = t >> 2, k = t & 3;
    // the four lanes of a frame agree on `on`: they read the same status
    const bool on = f < n && status[f] == ST_OK;
    uint32_t len = 0;
    const uint8_t *p = out;
    if (on) {
        const FrameDesc d = desc[f];
        len = d.d_size;
        p = out + d.d_off;
    }
    const uint32_t stripes = len / 32;
    uint64_t acc = k == 0 ? P1 + P2 : k == 1 ? P2 : k == 2 ? 0 : 0ull - P1;
    const uint8_t *q = p + 8 * k;
    uint32_t s = 0;
    for (; s + 4 <= stripes; s += 4) {
        const uint64_t v0 = ld8(q + 32 * s), v1 = ld8(q + 32 * s + 32);
        const uint64_t v2 = ld8(q + 32 * s + 64), v3 = ld8(q + 32 * s + 96);
        acc = xround(acc, v0);
        acc = xround(acc, v1);
        acc = xround(acc, v2);
        acc = xround(acc, v3);
    }
    for (; s < stripes; s++)
        acc = xround(acc, ld8(q + 32 * s));
    // accumulators 1..3 of this frame to its lane 0 (every lane shuffles)
    const int base = (int)(threadIdx.x & 60u);
    const uint64_t a1 = __shfl(acc, base + 1, 64), a2 = __shfl(acc, base + 2, 64),
                   a3 = __shfl(acc, base + 3, 64);
    if (!on || k != 0)
        return;
    uint64_t h;
    if (len >= 32) {
        h = rotl(acc, 1) + rotl(a1, 7) + rotl(a2, 12) + rotl(a3, 18);
        h = xmerge(h, acc);
        h = xmerge(h, a1);
        h = xmerge(h, a2);
        h = xmerge(h, a3);
    } else {
        h = P5;
    }
    h += len;
    uint32_t i = stripes * 32;
    for (; i + 8 <= len; i += 8) {
        h ^= xround(0, ld8(p + i));
        h = rotl(h, 27) * P1 + P4;
    }
    if (i + 4 <= len) {
        h ^= (uint64_t)*reinterpret_cast<const u32_ua *>(p + i) * P1;
        h = rotl(h, 23) * P2 + P3;
        i += 4;
    }
    for (; i < len; i++) {
        h ^= p[i] * P5;
        h = rotl(h, 11) * P1;
    }
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    if ((uint32_t)h != want[f])
        status[f] = ST_SEEK_CHECKSUM;
}

}   // namespace

int launch_frame_checksums(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_out,
                           const uint32_t *d_want, int32_t *d_status, hipStream_t stream)
{
    if (nframes == 0)
        return 0;
    const uint32_t blocks = (uint32_t)(((uint64_t)nframes * 4 + 255) / 256);
    hipLaunchKernelGGL(frame_xxh64_kernel, dim3(blocks), dim3(256), 0, stream, d_desc, nframes, d_out,
                       d_want, d_status);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk

extern "C" ZSEEK_EXPORT int zsk_verify_frame_checksums(const zsk_frame_desc_t *d_desc, uint32_t nframes,
                                                       const void *d_out, const uint32_t *d_checksums,
                                                       int32_t *d_status, void *stream)
{
    return zsk::launch_frame_checksums(reinterpret_cast<const zsk::FrameDesc *>(d_desc), nframes,
                                       static_cast<const uint8_t *>(d_out), d_checksums, d_status,
                                       static_cast<hipStream_t>(stream));
}
