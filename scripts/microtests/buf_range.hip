// Microtest: raw buffer_load_dwordx4 range checking at unaligned offsets
// straddling num_records (which bytes come back, which read as zero).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const uint8_t *src, uint32_t nrec, uint32_t *out)
{
    uint32_t lane = threadIdx.x;   // offset = lane
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, (int)nrec, 0x00020000);
    u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane, 0, 0));
    out[lane * 4 + 0] = v.x;
    out[lane * 4 + 1] = v.y;
    out[lane * 4 + 2] = v.z;
    out[lane * 4 + 3] = v.w;
}

int main()
{
    uint8_t h[256];
    for (int i = 0; i < 256; i++)
        h[i] = (uint8_t)(i + 1);
    uint8_t *d;
    uint32_t *o;
    hipMalloc(&d, 256);
    hipMalloc(&o, 64 * 16);
    hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
    for (uint32_t nrec : {21u, 24u, 32u}) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, nrec, o);
        hipDeviceSynchronize();
        uint8_t ho[64 * 16];
        hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
        printf("num_records=%u\n", nrec);
        for (int off = 0; off < 28; off++) {
            printf(" off %2d:", off);
            for (int b = 0; b < 16; b++)
                printf(" %c", ho[off * 16 + b] == 0 ? '.' : (ho[off * 16 + b] == (uint8_t)(off + b + 1) ? 'v' : '?'));
            printf("\n");
        }
    }
    return 0;
}
