// Piece-owner computation of seq_exec.hip copy_scan, in isolation: lanes
// with np pieces each; owners[t] must be the lane whose pieces cover t.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../libzseek_amd/csrc/lz4_dev.h"

using namespace zsk::lz4d;

constexpr uint32_t K = 6;

template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T *lp(uint32_t a)
{
    return (__attribute__((address_space(3))) T *)(uintptr_t)a;
}

__global__ void k(const uint32_t *in, uint32_t *out, uint32_t *incl)
{
    __shared__ __attribute__((aligned(16))) uint32_t own_[64 * K + 64];
    const uint32_t lane = threadIdx.x;
    const uint32_t own = (uint32_t)(uintptr_t)own_;
    // stale content
    for (uint32_t i = lane; i < 64 * K; i += 64)
        own_[i] = 0xdead;
    __syncthreads();
    const uint32_t np = in[lane];
    const uint32_t inc = wave_incl_add(np);
    const uint32_t T = lane_val(inc, 63);
    const uint32_t x = inc - np;
    const uint32_t ob = own + 4 * K * lane;
    // one access type for the owner array (uint32_t): a mixed-width
    // access would let the compiler forward the cleared value past the marks
#pragma unroll
    for (uint32_t j = 0; j < K; j++)
        *lp<uint32_t>(ob + 4 * j) = 0;
    if (np)
        *lp<uint32_t>(own + 4 * x) = lane + 1;
    wave_lds_sync();
    uint32_t o[K];
#pragma unroll
    for (uint32_t j = 0; j < K; j++)
        o[j] = *lp<uint32_t>(ob + 4 * j);
#pragma unroll
    for (uint32_t j = 1; j < K; j++)
        o[j] = max(o[j], o[j - 1]);
    const uint32_t wi = wave_incl_max(o[K - 1]);
    incl[lane] = wi;
    const uint32_t carry = dpp_prev(wi, 0);
#pragma unroll
    for (uint32_t j = 0; j < K; j++)
        *lp<uint32_t>(ob + 4 * j) = max(o[j], carry);
    wave_lds_sync();
    for (uint32_t t = lane; t < 64 * K; t += 64)
        out[t] = t < T ? *lp<uint32_t>(own + 4 * t) - 1 : 0xFFFFFFFFu;
}

int main()
{
    uint32_t h[64], o[64 * K], inc[64];
    unsigned s = 12345;
    int bad = 0;
    for (int rep = 0; rep < 50; rep++) {
        uint32_t tot = 0;
        for (int i = 0; i < 64; i++) {
            s = s * 1103515245u + 12345u;
            uint32_t v = (s >> 16) % 7;
            if (rep % 5 == 0 && i == 3)
                v = 40;
            if (tot + v > 64 * K)
                v = 0;
            h[i] = v;
            tot += v;
        }
        uint32_t *d, *e, *f;
        hipMalloc(&d, sizeof(h));
        hipMalloc(&e, sizeof(o));
        hipMalloc(&f, sizeof(inc));
        hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, e, f);
        hipMemcpy(o, e, sizeof(o), hipMemcpyDeviceToHost);
        hipMemcpy(inc, f, sizeof(inc), hipMemcpyDeviceToHost);
        uint32_t t = 0;
        for (int i = 0; i < 64; i++)
            for (uint32_t j = 0; j < h[i]; j++, t++)
                if (o[t] != (uint32_t)i) {
                    if (bad < 8)
                        printf("rep %d piece %u: owner %u want %d\n", rep, t, o[t], i);
                    bad++;
                }
        hipFree(d);
        hipFree(e);
        hipFree(f);
    }
    printf("owner scan bad=%d\n", bad);
    return bad != 0;
}
