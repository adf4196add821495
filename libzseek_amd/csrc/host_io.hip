// host_io.hip — a request's small upload by the GPU itself (gfx950).
//
// A single-frame read uploads ~30 KB (the frame's compressed bytes, its
// descriptor and, for zstd, the host plan) before its first kernel.  Through
// hipMemcpyAsync that is a DMA-engine copy (6 us on the request timeline)
// and then a cross-engine hand-off before the first kernel may start (~8 us
// more).  Here the copy is a kernel on the request's own stream that reads
// the pinned staging through its device mapping (pinned host memory is
// mapped into the GPU's address space) with every load of a thread issued
// before its stores, so the first decode kernel follows it like any other
// kernel on the stream.  Big uploads (the throughput path's batches) keep the
// DMA engine: PCIe bandwidth, not latency, is their bound.  The download of a
// small batch (its status words and the request's bytes) likewise: one
// kernel writing the pinned buffers in place of two copies.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "zsk_internal.h"

namespace zsk {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kUpT = 256;   // threads per workgroup
// 16-byte pieces per thread: one -- a ~32 KB upload spread over 8
// workgroups (8 CUs' load paths to the host) takes 3.3 us (median over a
// latency trace; 5.2 us average), against 7.6 us with four pieces per thread
// over 2 workgroups (64 x 1 over 32: 3.6 us average, no better per request)
constexpr uint32_t kUpV = 1;

template <uint32_t T, uint32_t V>
__global__ __launch_bounds__(T) void h2d_small_kernel(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst,
                                                      uint32_t n16)
{
    const uint32_t i0 = blockIdx.x * T * V + threadIdx.x;
    u32x4 v[V];
#pragma unroll
    for (uint32_t k = 0; k < V; k++) {
        const uint32_t i = i0 + k * T;
        if (i < n16)
            v[k] = src[i];
    }
#pragma unroll
    for (uint32_t k = 0; k < V; k++) {
        const uint32_t i = i0 + k * T;
        if (i < n16)
            dst[i] = v[k];
    }
}

// The batch's download in one kernel: the status words (aligned u32s) and
// the request's bytes [src, src + len) -- src at any byte, dst 16-aligned --
// written straight into pinned host memory through its device mapping.
// Each thread builds 16 bytes from five aligned dwords (v_alignbyte): the
// last thread's 20 bytes start at most 15 bytes before src + len rounded down
// to a dword, so it reads up to 19 bytes past src + len, and it writes up to
// 15 past dst + len (both buffers' slack: grow_dev / grow_host add 256).
__global__ __launch_bounds__(kUpT) void d2h_small_kernel(uint32_t *__restrict__ hst, const uint32_t *__restrict__ dst_,
                                                         uint32_t nst, u32x4 *__restrict__ hout,
                                                         const uint8_t *__restrict__ src, uint32_t len)
{
    const uint32_t t = blockIdx.x * kUpT + threadIdx.x;
    if (t < nst)
        hst[t] = dst_[t];
    if (16 * t >= len)
        return;
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3);
    const uint32_t *a = reinterpret_cast<const uint32_t *>(src - sh) + 4 * t;
    uint32_t d[5];
#pragma unroll
    for (int k = 0; k < 5; k++)
        d[k] = a[k];
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
    v.y = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
    v.z = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
    v.w = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
    hout[t] = v;
}

// The same download with the batch's completion posted to the host: one
// 1,024-thread workgroup writes everything (<= kFlagMax bytes), each wave
// waits for its stores and releases them at system scope, then, after the
// barrier, thread 0 writes `seq` to the pinned flag -- the reader spins on
// that word instead of waiting for the stream's completion signal (the
// kernel's end, the end-of-pipe flush, the signal, the runtime's wake-up).
constexpr uint32_t kFlagT = 1024;
__global__ __launch_bounds__(kFlagT) void d2h_flag_kernel(uint32_t *__restrict__ hst, const uint32_t *__restrict__ dst_,
                                                          uint32_t nst, u32x4 *__restrict__ hout,
                                                          const uint8_t *__restrict__ src, uint32_t len,
                                                          uint32_t *__restrict__ hflag, uint32_t seq)
{
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < nst; i += kFlagT)
        hst[i] = dst_[i];
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3);
    for (uint32_t i = t; 16 * i < len; i += kFlagT) {
        const uint32_t *a = reinterpret_cast<const uint32_t *>(src - sh) + 4 * i;
        uint32_t d[5];
#pragma unroll
        for (int k = 0; k < 5; k++)
            d[k] = a[k];
        u32x4 v;
        v.x = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
        v.y = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
        v.z = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
        v.w = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
        hout[i] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // (system scope: this wave's stores complete)
    __syncthreads();
    if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(hflag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}   // namespace

int download_flagged(uint32_t *h_status, void *hs, const uint32_t *d_status, uint32_t nst, uint8_t *h_out, void *ho,
                     const uint8_t *d_src, size_t len, void *hflag_dev, uint32_t seq, hipStream_t stream)
{
    if (!hs || !hflag_dev || len > kFlagMax || nst > kFlagMaxStatus ||
        (len && (!ho || (reinterpret_cast<uintptr_t>(ho) & 15))))
        return 1;
    hipLaunchKernelGGL(d2h_flag_kernel, dim3(1), dim3(kFlagT), 0, stream, static_cast<uint32_t *>(hs), d_status, nst,
                       static_cast<u32x4 *>(ho), d_src, (uint32_t)len, static_cast<uint32_t *>(hflag_dev), seq);
    (void)h_status;
    (void)h_out;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int download_small(uint32_t *h_status, void *hs, const uint32_t *d_status, uint32_t nst, uint8_t *h_out, void *ho,
                   const uint8_t *d_src, size_t len, hipStream_t stream)
{
    const bool small = len <= kDownloadSmallMax && hs && (!len || (ho && !(reinterpret_cast<uintptr_t>(ho) & 15)));
    if (!small) {
        if (hipMemcpyAsync(h_status, d_status, nst * sizeof(uint32_t), hipMemcpyDeviceToHost, stream) != hipSuccess)
            return -1;
        return !len || hipMemcpyAsync(h_out, d_src, len, hipMemcpyDeviceToHost, stream) == hipSuccess ? 0 : -1;
    }
    const uint32_t th = std::max<uint32_t>(nst, (uint32_t)((len + 15) / 16));
    hipLaunchKernelGGL(d2h_small_kernel, dim3((th + kUpT - 1) / kUpT), dim3(kUpT), 0, stream,
                       static_cast<uint32_t *>(hs), d_status, nst, static_cast<u32x4 *>(ho), d_src, (uint32_t)len);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int upload_small(void *d_dst, const void *h_src, const void *src, size_t bytes, hipStream_t stream)
{
    if (bytes == 0)
        return 0;
    if (bytes > kUploadSmallMax || !src || (reinterpret_cast<uintptr_t>(src) & 15) ||
        (reinterpret_cast<uintptr_t>(d_dst) & 15))
        return hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, stream) == hipSuccess ? 0 : -1;
    // whole 16-byte pieces: both buffers carry >= 256 bytes of slack past
    // their capacity (grow_host / grow_dev)
    const uint32_t n16 = (uint32_t)((bytes + 15) / 16);
    hipLaunchKernelGGL((h2d_small_kernel<kUpT, kUpV>), dim3((n16 + kUpT * kUpV - 1) / (kUpT * kUpV)), dim3(kUpT), 0,
                       stream, static_cast<const u32x4 *>(src), static_cast<u32x4 *>(d_dst), n16);
    (void)h_src;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk
