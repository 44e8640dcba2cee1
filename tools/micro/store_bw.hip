// Store-bandwidth microbenchmark: the fused render's background (depth, sil f32 + rgb 3xf32 =
// 20 B/px) and the fragment background (p2f i64 + zbuf + dists f32 + bary 3xf32 = 28 B/px) for
// 64 x 512 x 512 pixels, written with different store schedules. Prints us and GB/s per variant.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Arr { float4* p[8]; long long n4[8]; int na; };  // arrays as float4 streams

// A: every array in the same chunk loop (current fill_chunk): chunk c -> 64 lanes x 16 B of each array
// (arrays with more float4 per pixel-quad write several consecutive float4 per lane)
__global__ void __launch_bounds__(256) k_interleaved(Arr a, long long nq, int per_lane_mult_mask) {
  const long long G = (long long)gridDim.x * blockDim.x;
  const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += G) {
    for (int i = 0; i < a.na; ++i) {
      const int m = (int)(a.n4[i] / nq);
      for (int k = 0; k < m; ++k) a.p[i][q * m + k] = v;
    }
  }
}
// B: every array in the same loop, but lane-contiguous: array i with m float4 per quad is
// written as m wave-contiguous 1-KB blocks (q*m + k -> base*m + k*64 + lane)
__global__ void __launch_bounds__(256) k_interleaved_coal(Arr a, long long nq) {
  const long long G = (long long)gridDim.x * blockDim.x;
  const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  const int lane = threadIdx.x & 63;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += G) {
    const long long base = q - lane;
    for (int i = 0; i < a.na; ++i) {
      const int m = (int)(a.n4[i] / nq);
      for (int k = 0; k < m; ++k) a.p[i][base * m + k * 64 + lane] = v;
    }
  }
}
// C: arrays one after another (array-major index space), grid-stride
__global__ void __launch_bounds__(256) k_sequential(Arr a) {
  const long long G = (long long)gridDim.x * blockDim.x;
  const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  for (int i = 0; i < a.na; ++i)
    for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < a.n4[i]; q += G) a.p[i][q] = v;
}
// D: non-temporal variant of B
__global__ void __launch_bounds__(256) k_interleaved_nt(Arr a, long long nq) {
  const long long G = (long long)gridDim.x * blockDim.x;
  const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  const int lane = threadIdx.x & 63;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += G) {
    const long long base = q - lane;
    for (int i = 0; i < a.na; ++i) {
      const int m = (int)(a.n4[i] / nq);
      for (int k = 0; k < m; ++k) { typedef float f4v __attribute__((ext_vector_type(4))); f4v w = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(w, (f4v*)&a.p[i][base * m + k * 64 + lane]); }
    }
  }
}
// E: each wave owns a contiguous block of quads (not grid-stride): wave w writes quads [w*B, (w+1)*B)
__global__ void __launch_bounds__(256) k_blocked(Arr a, long long nq, int B) {
  const float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
  const int lane = threadIdx.x & 63;
  const long long w = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  for (long long b = w * B; b < (w + 1) * B && b < nq; b += 64) {
    const long long q = b + lane;
    if (q >= nq) break;
    for (int i = 0; i < a.na; ++i) {
      const int m = (int)(a.n4[i] / nq);
      for (int k = 0; k < m; ++k) a.p[i][b * m + k * 64 + lane] = v;
    }
  }
}

int main() {
  const long long npx = 64ll * 512 * 512, nq = npx / 4;
  float* buf;
  const long long total = 28 * npx;
  CHECK(hipMalloc(&buf, total + 4096));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (int cfg = 0; cfg < 3; ++cfg) {
    Arr a = {};
    const char* name;
    // render: depth (1 f4/quad), sil (1), rgb (3); fragments: p2f (2), zbuf (1), dists (1), bary (3); single: 5 f4/quad one array
    int ms_r[] = {1, 1, 3}, ms_f[] = {2, 1, 1, 3}, ms_s[] = {5};
    int* ms; 
    if (cfg == 0) { ms = ms_r; a.na = 3; name = "render 20B/px"; }
    else if (cfg == 1) { ms = ms_f; a.na = 4; name = "frags 28B/px"; }
    else { ms = ms_s; a.na = 1; name = "single 20B/px"; }
    long long off = 0, bytes = 0;
    for (int i = 0; i < a.na; ++i) { a.p[i] = (float4*)((char*)buf + off); a.n4[i] = nq * ms[i]; off += a.n4[i] * 16; bytes += a.n4[i] * 16; }
    for (int var = 0; var < 12; ++var) {
      int grid; const char* vn;
      auto launch = [&]() {
        switch (var) {
          case 0: grid = 1024; vn = "interleaved g1024"; k_interleaved<<<grid, 256>>>(a, nq, 0); break;
          case 1: grid = 1024; vn = "coal g1024"; k_interleaved_coal<<<grid, 256>>>(a, nq); break;
          case 2: grid = 2048; vn = "coal g2048"; k_interleaved_coal<<<grid, 256>>>(a, nq); break;
          case 3: grid = 4096; vn = "coal g4096"; k_interleaved_coal<<<grid, 256>>>(a, nq); break;
          case 4: grid = 512; vn = "coal g512"; k_interleaved_coal<<<grid, 256>>>(a, nq); break;
          case 5: grid = 1024; vn = "sequential g1024"; k_sequential<<<grid, 256>>>(a); break;
          case 6: grid = 4096; vn = "sequential g4096"; k_sequential<<<grid, 256>>>(a); break;
          case 7: grid = 2048; vn = "nt g2048"; k_interleaved_nt<<<grid, 256>>>(a, nq); break;
          case 8: { const int B = 4096; grid = (int)((nq + (long long)B * 4 - 1) / ((long long)B * 4)); vn = "blocked 4096q/wave"; k_blocked<<<grid, 256>>>(a, nq, B); break; }
          case 9: { const int B = 1024; grid = (int)((nq + (long long)B * 4 - 1) / ((long long)B * 4)); vn = "blocked 1024q/wave"; k_blocked<<<grid, 256>>>(a, nq, B); break; }
          case 10: { const int B = 256; grid = (int)((nq + (long long)B * 4 - 1) / ((long long)B * 4)); vn = "blocked 256q/wave"; k_blocked<<<grid, 256>>>(a, nq, B); break; }
          default: { const int B = 64; grid = (int)((nq + (long long)B * 4 - 1) / ((long long)B * 4)); vn = "blocked 64q/wave"; k_blocked<<<grid, 256>>>(a, nq, B); break; }
        }
      };
      for (int w = 0; w < 3; ++w) launch();
      CHECK(hipDeviceSynchronize());
      CHECK(hipEventRecord(e0));
      const int it = 20;
      for (int w = 0; w < it; ++w) launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms_ = 0; CHECK(hipEventElapsedTime(&ms_, e0, e1));
      const double us = ms_ * 1e3 / it;
      printf("%-14s %-22s %8.1f us  %7.0f GB/s\n", name, vn, us, bytes / us / 1e3);
    }
  }
  return 0;
}
