// Checks the lane semantics of gfx950 v_permlane16_swap / v_permlane32_swap
// (used by max_over_groups in common.h): hipcc --offload-arch=gfx950 permlane_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  int l = threadIdx.x;
  int x = l * 10;
  auto a = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  out[l * 4 + 0] = a[0]; out[l * 4 + 1] = a[1];
  out[l * 4 + 2] = b[0]; out[l * 4 + 3] = b[1];
}
int main() {
  int* d; hipMalloc(&d, 64 * 4 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  int h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 7) printf("lane %2d: p32 = (%d, %d)  p16 = (%d, %d)\n", l, h[l*4]/10, h[l*4+1]/10, h[l*4+2]/10, h[l*4+3]/10);
  return 0;
}
