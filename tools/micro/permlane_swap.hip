// Micro-test: semantics of gfx950 v_permlane32_swap / v_permlane16_swap as the builtins expose them.
// hipcc --offload-arch=gfx950 -O3 tools/micro/permlane_swap.hip -o exp/permlane_swap && exp/permlane_swap
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(int* out) {
  const int l = threadIdx.x;
  const unsigned a = 1000 + l, b = 2000 + l;
  auto s32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  auto s16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  out[l] = s32[0]; out[64 + l] = s32[1]; out[128 + l] = s16[0]; out[192 + l] = s16[1];
}
int main() {
  int* d; hipMalloc(&d, 256 * 4);
  k<<<1, 64>>>(d);
  int h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[4] = {"s32[0]", "s32[1]", "s16[0]", "s16[1]"};
  for (int j = 0; j < 4; ++j) {
    printf("%s:", nm[j]);
    for (int l = 0; l < 64; l += 8) printf(" l%d=%d", l, h[64 * j + l]);
    printf("\n");
  }
  return 0;
}
