// Microbenchmark: what makes short-lived 512-thread workgroups slow on MI355X?
// Variants share the grid of the empty-view raster (32768 WGs x 512 threads) and write
// the same 24 B/pixel of outputs (16.7M pixels).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Out { float* depth; float* sil; float* rgb; int* p2f; const int* cnt; };

template <int LDSB, bool READ_CNT, bool SYNC>
__global__ void __launch_bounds__(512) k_strip(Out o, int W, int H, int GX) {
  __shared__ float lds[LDSB > 0 ? LDSB / 4 : 1];
  const int n = blockIdx.y;
  const int gx = blockIdx.x % GX, ty = blockIdx.x / GX;
  const int t = threadIdx.x;
  int c = 0;
  if (READ_CNT) {
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    c = o.cnt[(n * (H / 8) + ty) * (W / 8) + gx * 8 + wave];
  }
  if (LDSB > 0) { lds[t] = (float)c; }
  if (SYNC) __syncthreads();
  const int row = t >> 6, col = t & 63;
  const int px = gx * 64 + col, py = ty * 8 + row;
  const long long pix = ((long long)n * H + py) * W + px;
  float v = LDSB > 0 ? lds[t ^ 1] : (float)c;
  o.depth[pix] = v;
  o.sil[pix] = v;
  o.p2f[pix] = -1;
  for (int j = t; j < 8 * 192; j += 512) {
    const int rr = j / 192, q = j - rr * 192;
    o.rgb[(((long long)n * H + ty * 8 + rr) * W + gx * 64) * 3 + q] = v;
  }
}

// same outputs, grid-stride over strips with a fixed grid (persistent style)
__global__ void __launch_bounds__(512) k_strip_persist(Out o, int W, int H, int GX, int nstrips) {
  for (int s = blockIdx.x; s < nstrips; s += gridDim.x) {
    const int n = s / (GX * (H / 8));
    const int b = s % (GX * (H / 8));
    const int gx = b % GX, ty = b / GX;
    const int t = threadIdx.x;
    const int row = t >> 6, col = t & 63;
    const int px = gx * 64 + col, py = ty * 8 + row;
    const long long pix = ((long long)n * H + py) * W + px;
    o.depth[pix] = 0.f;
    o.sil[pix] = 0.f;
    o.p2f[pix] = -1;
    for (int j = t; j < 8 * 192; j += 512) {
      const int rr = j / 192, q = j - rr * 192;
      o.rgb[(((long long)n * H + ty * 8 + rr) * W + gx * 64) * 3 + q] = 0.f;
    }
  }
}

// trivial exit, like the empty backward: read one int, write 12 floats
template <int LDSB>
__global__ void __launch_bounds__(256) k_exit(const int* cnt, float* part) {
  __shared__ float lds[LDSB / 4];
  if (cnt[blockIdx.y] <= (int)blockIdx.x * 1024) {
    if (threadIdx.x < 12) part[(blockIdx.y * gridDim.x + blockIdx.x) * 12 + threadIdx.x] = 0.f;
    return;
  }
  lds[threadIdx.x] = 1.f;
  __syncthreads();
  part[threadIdx.x] = lds[threadIdx.x ^ 1];
}

template <typename F>
float timeit(F f, int iters = 10) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f(); hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i) f();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / iters;
}

int main() {
  const int N = 64, H = 512, W = 512, GX = W / 64;
  const long long P = (long long)N * H * W;
  Out o;
  CHECK(hipMalloc(&o.depth, P * 4)); CHECK(hipMalloc(&o.sil, P * 4)); CHECK(hipMalloc(&o.rgb, P * 12));
  CHECK(hipMalloc(&o.p2f, P * 4));
  int* cnt; CHECK(hipMalloc(&cnt, (N * (H / 8) * (W / 8) + 64) * 4)); CHECK(hipMemset(cnt, 0, (N * (H / 8) * (W / 8) + 64) * 4));
  o.cnt = cnt;
  float* part; CHECK(hipMalloc(&part, 4096 * 64 * 12 * 4));
  dim3 g(GX * (H / 8), N);
  printf("plain stores            : %8.1f us\n", timeit([&] { k_strip<0, false, false><<<g, 512>>>(o, W, H, GX); }));
  printf("+ read cnt              : %8.1f us\n", timeit([&] { k_strip<0, true, false><<<g, 512>>>(o, W, H, GX); }));
  printf("+ 2KB LDS + sync        : %8.1f us\n", timeit([&] { k_strip<2048, true, true><<<g, 512>>>(o, W, H, GX); }));
  printf("+ 48KB LDS + sync       : %8.1f us\n", timeit([&] { k_strip<49152, true, true><<<g, 512>>>(o, W, H, GX); }));
  printf("persistent 2048 WGs     : %8.1f us\n", timeit([&] { k_strip_persist<<<2048, 512>>>(o, W, H, GX, GX * (H / 8) * N); }));
  printf("persistent 768 WGs      : %8.1f us\n", timeit([&] { k_strip_persist<<<768, 512>>>(o, W, H, GX, GX * (H / 8) * N); }));
  dim3 ge(32, 64);
  printf("exit 2048 WGs, 1KB LDS  : %8.1f us\n", timeit([&] { k_exit<1024><<<ge, 256>>>(cnt, part); }));
  printf("exit 2048 WGs, 40KB LDS : %8.1f us\n", timeit([&] { k_exit<40960><<<ge, 256>>>(cnt, part); }));
  dim3 ge2(256, 64);
  printf("exit 16384 WGs, 1KB LDS : %8.1f us\n", timeit([&] { k_exit<1024><<<ge2, 256>>>(cnt, part); }));
  return 0;
}
