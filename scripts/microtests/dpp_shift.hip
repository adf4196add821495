#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__global__ void k(uint32_t* out) {
  uint32_t x = threadIdx.x + 100;
  out[threadIdx.x] = __builtin_amdgcn_update_dpp(7u, x, 0x130, 0xf, 0xf, false);       // wave_shl1
  out[64 + threadIdx.x] = __builtin_amdgcn_update_dpp(7u, x, 0x138, 0xf, 0xf, false);  // wave_shr1
}
int main() {
  uint32_t o[128]; uint32_t *e; hipMalloc(&e, 512);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, e);
  hipMemcpy(o, e, 512, hipMemcpyDeviceToHost);
  printf("shl: lane0=%u lane1=%u lane15=%u lane16=%u lane62=%u lane63=%u\n", o[0], o[1], o[15], o[16], o[62], o[63]);
  printf("shr: lane0=%u lane1=%u lane15=%u lane16=%u lane62=%u lane63=%u\n", o[64], o[65], o[79], o[80], o[126], o[127]);
  return 0;
}
