// Microtest: LDS-DMA (global_load_lds_dwordx4) from 4-byte-aligned, not
// 16-byte-aligned per-lane global addresses; unaligned ds_write_b32.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void k(const uint8_t *src, uint32_t *out, uint32_t *out2)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[2048];
    const uint32_t lane = threadIdx.x;
    const uint8_t *g = src + 4 * (lane * 3 + 1);   // 4-aligned, not 16-aligned
    uint32_t base = (uint32_t)(uintptr_t)lds;
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off\n\ts_waitcnt vmcnt(0)"
                 :: "v"(g), "s"(base) : "memory", "m0");
    __syncthreads();
    const uint32_t *w = reinterpret_cast<const uint32_t *>(lds + 16 * lane);
    for (int i = 0; i < 4; i++)
        out[4 * lane + i] = w[i];
    __syncthreads();
    // unaligned 4-byte LDS store then byte readback
    uint32_t v = 0x11223344u + lane;
    *reinterpret_cast<volatile uint32_t *>(lds + 1024 + 5 * lane + 1) = v;
    __syncthreads();
    out2[lane] = (uint32_t)lds[1024 + 5 * lane + 1] | ((uint32_t)lds[1024 + 5 * lane + 2] << 8) |
                 ((uint32_t)lds[1024 + 5 * lane + 3] << 16) | ((uint32_t)lds[1024 + 5 * lane + 4] << 24);
}

int main()
{
    const int n = 4096;
    uint8_t h[n];
    for (int i = 0; i < n; i++)
        h[i] = (uint8_t)(i * 7 + 3);
    uint8_t *d;
    uint32_t *o, *o2;
    hipMalloc(&d, n);
    hipMalloc(&o, 64 * 16);
    hipMalloc(&o2, 64 * 4);
    hipMemcpy(d, h, n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, o2);
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("kernel failed\n");
        return 2;
    }
    uint32_t ho[64 * 4], ho2[64];
    hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
    hipMemcpy(ho2, o2, sizeof(ho2), hipMemcpyDeviceToHost);
    int bad = 0, bad2 = 0;
    for (int l = 0; l < 64; l++) {
        const uint8_t *e = h + 4 * (l * 3 + 1);
        if (memcmp(&ho[4 * l], e, 16))
            bad++;
        if (ho2[l] != 0x11223344u + l)
            bad2++;
    }
    printf("lds_dma_4aligned bad=%d  unaligned_ds_write_b32 bad=%d\n", bad, bad2);
    return (bad || bad2) ? 1 : 0;
}
