// Micro-test: rt_partial_swap (csrc/mr_bwd.h) against a host sum of the 12 per-lane values.
// hipcc --offload-arch=gfx950 -O3 -I torch_renderer_amd/csrc tools/micro/rt_swap.hip -o exp/rt_swap
#include <hip/hip_runtime.h>
#include <stdio.h>
#define MR_DEV __device__ __forceinline__
template <int CTRL, int ROW_MASK>
MR_DEV float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf, false));
}
// gfx950 v_permlane32_swap / v_permlane16_swap as inline asm: lanes 32-63 of x trade with lanes 0-31 of y
// (x = {x.lo, y.lo}, y = {x.hi, y.hi}); the 16-lane form trades x's odd rows with y's even rows. (The
// compiler's builtins returned a pair whose two halves it treated as one register when both feed one add:
// v_add_f32 v4, v4, v4 after the swap — tools/micro/rt_swap.hip.) The s_nop covers the VALU-write ->
// swap-read hazard the compiler cannot see through the asm.
MR_DEV void lane_swap32(float& x, float& y) { asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y)); }
MR_DEV void lane_swap16(float& x, float& y) { asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y)); }
#define RT_VALUE(j, r) (4 * (j) + (((r) & 1) << 1) + ((r) >> 1))
MR_DEV void rt_partial_swap(const float (&gR)[9], const float (&gT)[3], float (&o)[3]) {
  float h[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float a = 2 * i < 9 ? gR[2 * i] : gT[2 * i - 9];
    const float b = 2 * i + 1 < 9 ? gR[2 * i + 1] : gT[2 * i + 1 - 9];
    float x = a, y = b;
    lane_swap32(x, y);
    h[i] = x + y;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float x = h[2 * j], y = h[2 * j + 1];
    lane_swap16(x, y);
    float v = x + y;
    v += dppf<0xB1, 0xf>(v);
    v += dppf<0x4E, 0xf>(v);
    v += dppf<0x141, 0xf>(v);
    v += dppf<0x140, 0xf>(v);
    o[j] = v;
  }
}
__global__ void k(const float* in, float* out) {
  const int lane = threadIdx.x;
  float gR[9], gT[3];
  for (int i = 0; i < 9; ++i) gR[i] = in[i * 64 + lane];
  for (int i = 0; i < 3; ++i) gT[i] = in[(9 + i) * 64 + lane];
  float o[3];
  rt_partial_swap(gR, gT, o);
  if ((lane & 15) == 0) {
    const int r = lane >> 4;
    for (int j = 0; j < 3; ++j) out[RT_VALUE(j, r)] = o[j];
  }
}
int main() {
  float h[12 * 64], ref[12] = {0}, got[12];
  for (int i = 0; i < 12 * 64; ++i) { h[i] = (float)((i * 37) % 101) - 50.0f; ref[i / 64] += h[i]; }
  float *d, *o;
  hipMalloc(&d, sizeof(h)); hipMalloc(&o, sizeof(got));
  hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, o);
  hipMemcpy(got, o, sizeof(got), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 12; ++i) { printf("%d: got %g ref %g\n", i, got[i], ref[i]); bad += got[i] != ref[i]; }
  printf(bad ? "MISMATCH\n" : "OK\n");
  return 0;
}
