// lz4_wave.hip — wave-per-frame LZ4-frame decoder for CDNA4 (gfx950).
//
// Replaces the per-frame liblz4 call of the reference hot path
// (/root/reference/src/decompress.c:752-773, LZ4F_decompress in a loop) with
// ONE grid over every frame a zseek_pread range covers.
//
// Mapping:
//   * one wave64 decodes one seek-table frame; WAVES independent waves per
//     workgroup, frames dealt one per wave in grid order;
//   * the compressed frame streams through a 1 KiB register window per wave
//     (4 VGPRs x 64 lanes x 4 B, coalesced 256-B buffer loads, 2 windows of
//     prefetch); the token parse runs wave-uniform on the scalar unit, bytes
//     picked out of the window with v_readlane;
//   * literal runs move window -> LDS with ds_bpermute (lane i takes byte i);
//   * decoded bytes land in a per-wave LDS ring (RING bytes); matches whose
//     source is still in the ring are copied LDS -> LDS, older ones are
//     re-read from the frame's already-flushed output in HBM;
//   * completed 256-B ring chunks are flushed with one coalesced dword store
//     per lane.
//   * every global access goes through a per-frame buffer resource whose
//     num_records is the frame's seek-table size: hardware range checking
//     keeps a corrupt frame from touching any byte outside its own slot.
//
// Validation follows liblz4 1.9.3 (the library the reference links) so that
// success/failure matches the reference; oracle/lz4_oracle.c restates the same
// rules on the CPU.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4_wave_dev.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4w;

// DEFERRED (hand-offs after the two-phase decoder): each wave owns per_wave
// consecutive frames, reads their statuses at once (one lane each) and
// decodes the ones the parse left ST_NOT_RUN in turn -- a batch with no
// hand-off costs one status load per wave instead of one wave per frame
// (round 3: 262,144 workgroups, 83 us, for 1,048,576 frames of 4 KiB).
template <int RING, int WAVES, bool DEFERRED = false>
__global__ __launch_bounds__(64 * WAVES) void lz4_wave_kernel(const FrameDesc *__restrict__ desc,
                                                                uint32_t nframes,
                                                                const uint8_t *__restrict__ comp,
                                                                uint8_t *__restrict__ out,
                                                                int32_t *__restrict__ status,
                                                                uint32_t *__restrict__ fail_at,
                                                                uint32_t per_wave)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[WAVES * RING];
    const uint32_t wave = uni(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t g = DEFERRED ? per_wave : 1;
    const uint32_t f0 = uni((blockIdx.x * WAVES + wave) * g);
    if (f0 >= nframes)
        return;
    uint64_t todo = 1;
    if (DEFERRED)
        todo = __ballot(lane < g && f0 + lane < nframes && status[f0 + lane] == ST_NOT_RUN);
    for (; todo; todo &= todo - 1)
        wave_frame<RING>(desc, f0 + (uint32_t)__builtin_ctzll(todo), comp, out, status, fail_at, lds + wave * RING);
}

}   // namespace

int launch_lz4_wave_deferred(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                             uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at,
                             hipStream_t stream)
{
    if (nframes == 0)
        return 0;
    // frames per wave: enough waves (>= 16,384) to fill the chip when every
    // frame is a hand-off, at most 64 (one status per lane)
    const uint32_t per = min(64u, max(1u, nframes / 16384));
    const uint32_t waves = (nframes + per - 1) / per;
    hipLaunchKernelGGL((lz4_wave_kernel<4096, 4, true>), dim3((waves + 3) / 4), dim3(256), 0, stream, d_desc,
                       nframes, d_comp, d_out, d_status, d_fail_at, per);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_lz4_wave(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                    uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream)
{
    if (nframes == 0)
        return 0;
    hipLaunchKernelGGL((lz4_wave_kernel<4096, 4>), dim3((nframes + 3) / 4), dim3(256), 0, stream, d_desc,
                       nframes, d_comp, d_out, d_status, d_fail_at, 1u);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk
