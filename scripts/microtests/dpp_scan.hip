#include <hip/hip_runtime.h>
#include <stdint.h>
// inclusive wave64 prefix sum via DPP (gfx9: row_shr, row_bcast)
__device__ __forceinline__ uint32_t wave_incl(uint32_t v)
{
    uint32_t x = v;
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return x;
}
__global__ void k(const uint32_t* in, uint32_t* out) {
  out[threadIdx.x] = wave_incl(in[threadIdx.x]);
}
int main() {
  uint32_t h[64], o[64]; for (int i = 0; i < 64; i++) h[i] = i * 3 + 1;
  uint32_t *d, *e; hipMalloc(&d, 256); hipMalloc(&e, 256);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, e);
  hipMemcpy(o, e, 256, hipMemcpyDeviceToHost);
  int bad = 0; uint32_t s = 0;
  for (int i = 0; i < 64; i++) { s += h[i]; if (o[i] != s) { bad++; if (bad < 5) printf("lane %d got %u want %u\n", i, o[i], s); } }
  printf("dpp scan bad=%d\n", bad);
  return bad != 0;
}
