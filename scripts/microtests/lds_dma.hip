// Microtests for the two-phase LZ4 decoder's hardware assumptions (gfx950):
//  1. LDS-DMA (global_load_lds_dwordx4) from 4-aligned, non-16-aligned
//     per-lane global addresses lands the right bytes.
//  2. DS 32-bit and 128-bit reads/writes at byte-misaligned LDS addresses:
//     correctness, and cycles per wave-instruction vs aligned.
//  3. global_load_dwordx4 / global_store_dwordx4 at byte-misaligned
//     addresses: correctness.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_dma(const uint8_t *src, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[1024];
    const uint32_t lane = threadIdx.x;
    const uint8_t *g = src + 4 * (lane * 3 + 1);
    uint32_t base = (uint32_t)(uintptr_t)lds;
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off\n\ts_waitcnt vmcnt(0)"
                 :: "v"(g), "s"(base) : "memory", "m0");
    __syncthreads();
    const uint32_t *w = reinterpret_cast<const uint32_t *>(lds + 16 * lane);
    for (int i = 0; i < 4; i++)
        out[4 * lane + i] = w[i];
}

// mode: 0 = b32 write+read at lane*20+mis, 1 = b128 write+read
__global__ void k_ds(int mode, uint32_t mis, uint32_t *out, long long *cyc)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[4096];
    const uint32_t lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64)
        reinterpret_cast<uint32_t *>(lds)[i] = 0;
    __syncthreads();
    uint32_t a = (uint32_t)(uintptr_t)lds + lane * 20 + mis;
    u32x4 v = {0x01020304u * (lane + 1), 0x11121314u + lane, 0x21222324u + lane, 0x31323334u + lane};
    u32x4 r;
    long long t0 = __builtin_amdgcn_s_memtime();
    if (mode == 0) {
        for (int it = 0; it < 256; it++) {
            asm volatile("ds_write_b32 %0, %1\n\tds_write_b32 %0, %2 offset:4\n\t"
                         "ds_write_b32 %0, %3 offset:8\n\tds_write_b32 %0, %4 offset:12"
                         :: "v"(a), "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w) : "memory");
            asm volatile("ds_read_b32 %0, %4\n\tds_read_b32 %1, %4 offset:4\n\t"
                         "ds_read_b32 %2, %4 offset:8\n\tds_read_b32 %3, %4 offset:12\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(r.x), "=v"(r.y), "=v"(r.z), "=v"(r.w) : "v"(a) : "memory");
            v.x ^= r.x & 0;
        }
    } else {
        for (int it = 0; it < 256; it++) {
            asm volatile("ds_write_b128 %0, %1" :: "v"(a), "v"(v) : "memory");
            asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
            v.x ^= r.x & 0;
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[4 * lane + 0] = r.x;
    out[4 * lane + 1] = r.y;
    out[4 * lane + 2] = r.z;
    out[4 * lane + 3] = r.w;
    // byte-level check of what landed in LDS
    __syncthreads();
    uint32_t ok = 1;
    const uint8_t *vb = reinterpret_cast<const uint8_t *>(&v);
    for (int i = 0; i < 16; i++)
        ok &= lds[lane * 20 + mis + i] == vb[i];
    out[256 + lane] = ok;
    if (lane == 0)
        cyc[0] = t1 - t0;
}

__global__ void k_glob(const uint8_t *src, uint8_t *dst, uint32_t *out)
{
    const uint32_t lane = threadIdx.x;
    u32x4 v;
    const uint8_t *s = src + lane * 19 + 3;
    asm volatile("global_load_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(s) : "memory");
    uint8_t *d = dst + lane * 21 + 5;
    asm volatile("global_store_dwordx4 %0, %1, off\n\ts_waitcnt vmcnt(0)" :: "v"(d), "v"(v) : "memory");
    out[lane] = v.x;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)

int main()
{
    const int n = 4096;
    static uint8_t h[n];
    for (int i = 0; i < n; i++)
        h[i] = (uint8_t)(i * 7 + 3);
    uint8_t *d, *d2;
    uint32_t *o;
    long long *cyc;
    CK(hipMalloc(&d, n));
    CK(hipMalloc(&d2, n));
    CK(hipMalloc(&o, 4096));
    CK(hipMalloc(&cyc, 64));
    CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
    int fails = 0;

    hipLaunchKernelGGL(k_dma, dim3(1), dim3(64), 0, 0, d, o);
    CK(hipDeviceSynchronize());
    uint32_t ho[512];
    CK(hipMemcpy(ho, o, 64 * 16, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; l++)
        bad += memcmp(&ho[4 * l], h + 4 * (l * 3 + 1), 16) != 0;
    printf("lds_dma 4-aligned src: bad lanes %d\n", bad);
    fails += bad != 0;

    for (int mode = 0; mode < 2; mode++)
        for (uint32_t mis = 0; mis < 4; mis++) {
            hipLaunchKernelGGL(k_ds, dim3(1), dim3(64), 0, 0, mode, mis, o, cyc);
            CK(hipDeviceSynchronize());
            long long c;
            CK(hipMemcpy(ho, o, 320 * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            int badr = 0, badl = 0;
            for (int l = 0; l < 64; l++) {
                uint32_t e[4] = {0x01020304u * (l + 1), 0x11121314u + l, 0x21222324u + l, 0x31323334u + l};
                badr += memcmp(&ho[4 * l], e, 16) != 0;
                badl += ho[256 + l] != 1;
            }
            printf("ds %s mis=%u: read-bad %d lds-bad %d  cycles/iter %.1f\n", mode ? "b128" : "4xb32", mis,
                   badr, badl, c / 256.0);
            fails += badr || badl;
        }

    CK(hipMemset(d2, 0, n));
    hipLaunchKernelGGL(k_glob, dim3(1), dim3(64), 0, 0, d, d2, o);
    CK(hipDeviceSynchronize());
    static uint8_t h2[n];
    CK(hipMemcpy(h2, d2, n, hipMemcpyDeviceToHost));
    bad = 0;
    for (int l = 0; l < 64; l++)
        bad += memcmp(h2 + l * 21 + 5, h + l * 19 + 3, 16) != 0;
    printf("global dwordx4 misaligned load/store: bad lanes %d\n", bad);
    fails += bad != 0;
    printf(fails ? "MICROTEST FAIL\n" : "MICROTEST OK\n");
    return fails ? 1 : 0;
}
