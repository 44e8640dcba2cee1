// Cycles per face iteration of the real raster kernel: one view, F tiny faces piled into
// one 8x8 tile (the "blob"), or spread so that each tile holds ~80 faces (the cow case).
// Usage: rc F spread N
#include "../../torch_renderer_amd/csrc/mr_raster.hip"
#include <stdlib.h>
#include <vector>

int main(int argc, char** argv) {
  const int F = argc > 1 ? atoi(argv[1]) : 4096;
  const int spread = argc > 2 ? atoi(argv[2]) : 0;  // 0: blob in one tile; 1: spread over the image
  const int N = argc > 3 ? atoi(argv[3]) : 1;
  const int H = 512, W = 512;
  std::vector<float> fv((size_t)N * F * 9);
  srand(1);
  for (int n = 0; n < N; ++n)
    for (int f = 0; f < F; ++f) {
      float cx = 0.f, cy = 0.f;
      if (spread) {
        cx = ((rand() % 10000) / 10000.f - 0.5f) * 0.5f;
        cy = ((rand() % 10000) / 10000.f - 0.5f) * 0.5f;
      }
      const float s = 3.0f / 256.0f;  // ~3 px triangles
      float* v = &fv[((size_t)n * F + f) * 9];
      for (int c = 0; c < 3; ++c) {
        v[3 * c + 0] = cx + s * ((rand() % 1000) / 1000.f - 0.5f);
        v[3 * c + 1] = cy + s * ((rand() % 1000) / 1000.f - 0.5f);
        v[3 * c + 2] = 1.0f + (rand() % 1000) / 1000.f;
      }
    }
  float* dfv; int64_t *first, *count, *p2f; float *zbuf, *bary, *dists;
  hipMalloc(&dfv, fv.size() * 4);
  hipMemcpy(dfv, fv.data(), fv.size() * 4, hipMemcpyHostToDevice);
  std::vector<int64_t> hf(N), hc(N, F);
  for (int n = 0; n < N; ++n) hf[n] = (int64_t)n * F;
  hipMalloc(&first, N * 8); hipMalloc(&count, N * 8);
  hipMemcpy(first, hf.data(), N * 8, hipMemcpyHostToDevice);
  hipMemcpy(count, hc.data(), N * 8, hipMemcpyHostToDevice);
  const size_t P = (size_t)N * H * W;
  hipMalloc(&p2f, P * 8); hipMalloc(&zbuf, P * 4); hipMalloc(&bary, P * 12); hipMalloc(&dists, P * 4);
  mr_raster_settings_t s = {H, W, 1, 0.0f, 1, 0, 0, 0};
  size_t wsb = mr_rasterize_meshes_workspace(N, (int64_t)N * F, H, W, 0);
  void* ws; hipMalloc(&ws, wsb);
  mr_timing_enable(1);
  for (int it = 0; it < 6; ++it)
    if (mr_rasterize_meshes(dfv, first, count, N, (int64_t)N * F, &s, p2f, zbuf, bary, dists, ws, wsb, 0)) {
      printf("error %s\n", mr_last_error()); return 1;
    }
  hipDeviceSynchronize();
  int32_t l[KID_COUNT]; double t[KID_COUNT];
  mr_timing_read(l, t, KID_COUNT);
  const double us = t[KID_RASTER_FRAG] / l[KID_RASTER_FRAG] * 1e3;
  printf("F=%d spread=%d N=%d raster %.1f us", F, spread, N, us);
  if (!spread) printf("  => %.0f cycles/face/wave @2.4GHz", us * 2400.0 / (F / 8.0));
  printf("\n");
  return 0;
}
