// latency micro-benchmark (diagnostic, not product): one wave, a dependent
// chain of (a) scalar loads of a 8 KB table (K$ hits after the first pass),
// (b) LDS reads of the same table, (c) vector global loads (L1/L2 hits);
// cycles per step by s_memtime.  Loads only.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void chase(const uint32_t *__restrict__ tab, uint32_t n, uint32_t steps, unsigned long long *out)
{
    __shared__ uint32_t lt[2048];
    for (uint32_t i = threadIdx.x; i < 2048; i += 64)
        lt[i] = tab[i];
    __syncthreads();
    // (a) scalar: the index stays uniform (readfirstlane keeps it in an SGPR)
    const __attribute__((address_space(4))) uint32_t *ct = (const __attribute__((address_space(4))) uint32_t *)tab;
    uint32_t x = 0;
    for (uint32_t i = 0; i < 256; i++)
        x = ct[x];
    uint64_t t0 = __builtin_readcyclecounter();
    for (uint32_t i = 0; i < steps; i++)
        x = ct[x];
    uint64_t t1 = __builtin_readcyclecounter();
    // (b) LDS, the index in a VGPR (an opaque zero keeps it there)
    uint32_t zv;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zv));
    uint32_t y = x & 2047;
    for (uint32_t i = 0; i < steps; i++)
        y = lt[y + zv];
    uint64_t t2 = __builtin_readcyclecounter();
    // (c) vector global loads
    uint32_t z = y & 2047;
    for (uint32_t i = 0; i < steps; i++)
        z = tab[z + zv];
    uint64_t t3 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = t2 - t1;
        out[2] = t3 - t2;
        out[3] = x + y + z;
    }
}

int main()
{
    const uint32_t n = 2048, steps = 4096;
    uint32_t h[2048];
    // a random cycle over the table
    uint32_t perm[2048];
    for (uint32_t i = 0; i < n; i++)
        perm[i] = i;
    uint32_t s = 12345;
    for (uint32_t i = n - 1; i > 0; i--) {
        s = s * 1103515245u + 12345u;
        uint32_t j = (s >> 8) % (i + 1);
        uint32_t t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
    for (uint32_t i = 0; i < n; i++)
        h[perm[i]] = perm[(i + 1) % n];
    uint32_t *d;
    unsigned long long *o, ho[4];
    hipMalloc(&d, sizeof(h));
    hipMalloc(&o, sizeof(ho));
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, n, steps, o);
        hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
        printf("cycles per dependent load: scalar %.1f  lds %.1f  vector-global %.1f\n", (double)ho[0] / steps,
               (double)ho[1] / steps, (double)ho[2] / steps);
    }
    return 0;
}
