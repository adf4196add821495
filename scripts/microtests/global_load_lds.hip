#include <hip/hip_runtime.h>
#include <stdint.h>
__global__ void k(const uint32_t *src, uint32_t *out) {
  __shared__ uint32_t buf[256];
  __builtin_amdgcn_global_load_lds((const void *)(src + threadIdx.x * 3), (__attribute__((address_space(3))) void *)buf, 4, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  out[threadIdx.x] = buf[threadIdx.x];
}
int main() {
  uint32_t h[256*3], o[64]; for (int i = 0; i < 256*3; i++) h[i] = i;
  uint32_t *d, *e; hipMalloc(&d, sizeof(h)); hipMalloc(&e, 256);
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, e);
  hipMemcpy(o, e, 256, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 64; i++) if (o[i] != (uint32_t)(3*i)) { bad++; if (bad < 4) printf("lane %d got %u\n", i, o[i]); }
  printf("global_load_lds dword bad=%d\n", bad); return bad != 0;
}
