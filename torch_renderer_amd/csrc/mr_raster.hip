// mi355r — MI355X (gfx950, CDNA4) rasterizer kernels + C ABI.
//
// Pipeline for a batch of N views (one launch each, all async on one stream):
//   1. k_setup_*   : one thread per (view, face): project (or read face_verts),
//                    build a 64-B FaceRec, and append the face id to every
//                    32x32-pixel super-tile its (conservative) bbox touches
//                    (global atomics on per-tile counters; order irrelevant).
//   2. k_raster<M> : one 256-thread workgroup per (super-tile, view). Face
//                    records of the tile's list are staged in LDS in chunks of
//                    256; each wave owns a 16x16 region = 4 sub-tiles of 8x8
//                    (lane = pixel). Per face: wave-uniform sub-tile bbox test,
//                    then the exact per-pixel test (cheap edge-sign reject,
//                    then the CPU-identical barycentric/depth evaluation).
//                    K=1 keeps the lexicographic (z, face) minimum == the CPU
//                    tie-break, so the result is independent of list order.
//                    Epilogue: M=0 writes PyTorch3D Fragments; M=1 shades
//                    (depth relu, sigmoid silhouette, Phong + softmax blend)
//                    and writes only the requested images + int32 face ids.
//   3. backward    : k_render_bwd / k_raster_bwd — one workgroup per
//                    (super-tile, view); per covered pixel the forward is
//                    recomputed, the analytic backward produces per-face
//                    gradient rows that are pre-reduced in an LDS hash table
//                    (ds_add_f32) and flushed with one global atomic per
//                    (workgroup, face, component); per-view R/T gradients are
//                    reduced in-workgroup and written without atomics.
//   4. vertex kernels gather per-face rows through a CSR vertex adjacency
//      (deterministic order) and chain the vertex-normal backward.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdarg.h>

#include "../../include/mi355r.h"
#include "mr_common.h"
#include "mr_shade.h"

#define MR_ST 32      // super-tile edge (pixels)
#define MR_CH 256     // face records staged in LDS per chunk
#define MR_HT 512     // LDS hash slots in the backward
#define MR_DEFAULT_CAP 2048

static thread_local char g_err[512];
static int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
#define MR_CHECK_LAUNCH(name)                                                         \
  do {                                                                                \
    hipError_t _e = hipGetLastError();                                                \
    if (_e != hipSuccess) return set_err(MR_ELAUNCH, "%s: %s", name, hipGetErrorString(_e)); \
  } while (0)

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
static inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

struct TileGeom {
  int NSTX, NSTY, NST, cap;
};
static TileGeom tile_geom(int H, int W, int64_t max_faces_per_view, int32_t mfpb) {
  TileGeom g;
  g.NSTX = ceil_div(W, MR_ST);
  g.NSTY = ceil_div(H, MR_ST);
  g.NST = g.NSTX * g.NSTY;
  int64_t cap = mfpb > 0 ? mfpb : MR_DEFAULT_CAP;
  if (cap > max_faces_per_view) cap = max_faces_per_view;
  if (cap < 1) cap = 1;
  g.cap = (int)cap;
  return g;
}

struct RasterWS {
  FaceRec* recs;
  int* bin_count;
  int* bin_faces;
  size_t bytes;
};
static RasterWS carve_raster_ws(void* base, int64_t N, int64_t Ftot, const TileGeom& g) {
  RasterWS w;
  size_t off = 0;
  char* b = (char*)base;
  w.recs = (FaceRec*)(b + off);
  off = align_up(off + sizeof(FaceRec) * (size_t)Ftot, 256);
  w.bin_count = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)N * g.NST, 256);
  w.bin_faces = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)N * g.NST * g.cap, 256);
  w.bytes = off;
  return w;
}

// ---------------------------------------------------------------------------
// 1. setup + binning
// ---------------------------------------------------------------------------
struct SetupParams {
  int H, W, NSTX, NSTY, NST, cap;
  float bbox_pad;
  int persp, cull;
  FaceRec* recs;
  int* bin_count;
  int* bin_faces;
};

// Inverse of col_ndc/row_ndc (approximate, widened by one pixel; the raster
// kernel repeats the exact per-pixel bbox test, so a superset is all we need).
MR_DEV void ndc_range_to_pix(float lo, float hi, int S1, int S2, int& p0, int& p1) {
  float range = 2.0f;
  if (S1 > S2) range = ((float)S1 * range) / (float)S2;
  const float off = range / 2.0f;
  // i = ((ndc + off) * S1 - off) / range ; pixel = S1 - 1 - i
  float i_hi = ((hi + off) * (float)S1 - off) / range;
  float i_lo = ((lo + off) * (float)S1 - off) / range;
  float pf0 = (float)(S1 - 1) - i_hi - 1.0f;
  float pf1 = (float)(S1 - 1) - i_lo + 1.0f;
  pf0 = fminf(fmaxf(pf0, -2.0f), (float)S1 + 1.0f);
  pf1 = fminf(fmaxf(pf1, -2.0f), (float)S1 + 1.0f);
  p0 = (int)floorf(pf0);
  p1 = (int)ceilf(pf1);
  if (p0 < 0) p0 = 0;
  if (p1 > S1 - 1) p1 = S1 - 1;
}

MR_DEV void setup_one(const SetupParams& P, int n, int64_t rec, uint32_t face, const float v[3][3]) {
  FaceRec r;
  r.x0 = v[0][0]; r.y0 = v[0][1]; r.z0 = v[0][2];
  r.x1 = v[1][0]; r.y1 = v[1][1]; r.z1 = v[1][2];
  r.x2 = v[2][0]; r.y2 = v[2][1]; r.z2 = v[2][2];
  r.face = face;
  const bool fin = rec_finite(r);
  const float face_area = edge_fn(r.x0, r.y0, r.x1, r.y1, r.x2, r.y2);  // ComputeFaceAreas: E(v0,v1,v2)
  r.area = (float)((double)edge_fn(r.x2, r.y2, r.x0, r.y0, r.x1, r.y1) + MR_KEPS_D);
  r.xmin = smin(r.x0, smin(r.x1, r.x2));
  r.xmax = smax(r.x0, smax(r.x1, r.x2));
  r.ymin = smin(r.y0, smin(r.y1, r.y2));
  r.ymax = smax(r.y0, smax(r.y1, r.y2));
  const float zmax = smax(r.z0, smax(r.z1, r.z2));
  bool valid = fin;
  if (P.cull && face_area < 0.0f) valid = false;
  if ((double)face_area <= MR_KEPS_D && (double)face_area >= -1.0f * MR_KEPS_D) valid = false;
  if (zmax < 0.0f) valid = false;
  bool fast = valid && __builtin_isfinite(r.area) && r.area != 0.0f;
  if (P.persp) fast = fast && r.z0 > 0.0f && r.z1 > 0.0f && r.z2 > 0.0f;
  r.flags = (valid ? FR_VALID : 0u) | (fast ? FR_FAST : 0u);
  P.recs[rec] = r;
  if (!valid) return;
  int cx0, cx1, cy0, cy1;
  ndc_range_to_pix(r.xmin - P.bbox_pad, r.xmax + P.bbox_pad, P.W, P.H, cx0, cx1);
  ndc_range_to_pix(r.ymin - P.bbox_pad, r.ymax + P.bbox_pad, P.H, P.W, cy0, cy1);
  if (cx0 > cx1 || cy0 > cy1) return;
  const int tx0 = cx0 / MR_ST, tx1 = cx1 / MR_ST, ty0 = cy0 / MR_ST, ty1 = cy1 / MR_ST;
  for (int ty = ty0; ty <= ty1; ++ty)
    for (int tx = tx0; tx <= tx1; ++tx) {
      const int b = n * P.NST + ty * P.NSTX + tx;
      const int slot = atomicAdd(&P.bin_count[b], 1);
      if (slot < P.cap) P.bin_faces[(int64_t)b * P.cap + slot] = (int)rec;
    }
}

// World mode: one mesh shared by all views (Meshes.extend(N)); rec = n*F + f.
__global__ void __launch_bounds__(256) k_setup_world(SetupParams P, const float* __restrict__ verts,
                                                     const int32_t* __restrict__ faces, int64_t F,
                                                     const ViewRec* __restrict__ views) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = blockIdx.y;
  if (f >= F) return;
  const ViewRec V = views[n];
  float v[3][3];
  for (int c = 0; c < 3; ++c) {
    const int32_t vi = faces[3 * f + c];
    const float X[3] = {verts[3 * (int64_t)vi], verts[3 * (int64_t)vi + 1], verts[3 * (int64_t)vi + 2]};
    float vx, vy, vz;
    project_point(V, X, vx, vy, vz, v[c][0], v[c][1]);
    v[c][2] = vz;
  }
  setup_one(P, n, (int64_t)n * F + f, (uint32_t)f, v);
}

// face_verts mode (PyTorch3D _C boundary): rec = packed face id.
__global__ void __launch_bounds__(256) k_setup_fv(SetupParams P, const float* __restrict__ fv, int64_t Ftot,
                                                  const int64_t* __restrict__ first, int64_t N) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= Ftot) return;
  // mesh owning f: last n with first[n] <= f (packed, ascending)
  int64_t lo = 0, hi = N - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (first[mid] <= f) lo = mid;
    else hi = mid - 1;
  }
  float v[3][3];
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 3; ++k) v[c][k] = fv[9 * f + 3 * c + k];
  setup_one(P, (int)lo, f, (uint32_t)f, v);
}

// ---------------------------------------------------------------------------
// 2. raster (+ fused shading)
// ---------------------------------------------------------------------------
struct RasterParams {
  int N, H, W, NSTX, NSTY, NST, cap;
  float blur, bbox_pad;
  int persp, clipb;
  const FaceRec* recs;
  const int* bin_count;
  const int* bin_faces;
  const int64_t* view_first;  // NULL: shared mode (first = n*F, count = F)
  const int64_t* view_count;
  int64_t F;
  // MODE 0 outputs
  int64_t* p2f;
  float* zbuf;
  float* bary;
  float* dists;
  // MODE 1
  ShadeParams S;
  int out_flags, rgb_ch;
  float* depth;
  float* sil;
  float* rgb;
  int32_t* p2f32;
};

template <int MODE>
__global__ void __launch_bounds__(256) k_raster(RasterParams P) {
  __shared__ FaceRec srec[MR_CH];
  __shared__ int sid[MR_CH];
  const int n = blockIdx.y, st = blockIdx.x;
  const int stx = st % P.NSTX, sty = st / P.NSTX;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int rx0 = stx * MR_ST + (wave & 1) * 16, ry0 = sty * MR_ST + (wave >> 1) * 16;
  const int lx = lane & 7, ly = lane >> 3;
  const int H = P.H, W = P.W;

  float xf[4], yf[4], bz[4];
  int bf[4];
  bool pv[4];
  float sxl[4], sxh[4], syl[4], syh[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int sx = rx0 + (p & 1) * 8, sy = ry0 + (p >> 1) * 8;
    const int px = sx + lx, py = sy + ly;
    pv[p] = px < W && py < H;
    xf[p] = col_ndc(px < W ? px : W - 1, H, W);
    yf[p] = row_ndc(py < H ? py : H - 1, H, W);
    bz[p] = __builtin_inff();
    bf[p] = -1;
    if (sx < W && sy < H) {
      const int cx1 = sx + 7 < W ? sx + 7 : W - 1, cy1 = sy + 7 < H ? sy + 7 : H - 1;
      sxh[p] = col_ndc(sx, H, W);
      sxl[p] = col_ndc(cx1, H, W);
      syh[p] = row_ndc(sy, H, W);
      syl[p] = row_ndc(cy1, H, W);
    } else {  // empty sub-tile: bounds that reject every face
      sxh[p] = -__builtin_inff();
      sxl[p] = __builtin_inff();
      syh[p] = -__builtin_inff();
      syl[p] = __builtin_inff();
    }
  }

  const int bidx = n * P.NST + st;
  const int cnt = P.bin_count[bidx];
  const bool ovf = cnt > P.cap;
  const int64_t vfirst = P.view_first ? P.view_first[n] : (int64_t)n * P.F;
  const int64_t vcount = P.view_first ? P.view_count[n] : P.F;
  const int total = ovf ? (int)vcount : cnt;
  const float pad = P.bbox_pad;
  const bool fast_ok = !(P.blur > 0.0f);

  for (int base = 0; base < total; base += MR_CH) {
    const int m = (total - base) < MR_CH ? (total - base) : MR_CH;
    __syncthreads();
    if (tid < m) {
      const int rid = ovf ? (int)(vfirst + base + tid) : P.bin_faces[(int64_t)bidx * P.cap + base + tid];
      srec[tid] = P.recs[rid];
      sid[tid] = rid;
    }
    __syncthreads();
    for (int j = 0; j < m; ++j) {
      const FaceRec r = srec[j];
      if (!(r.flags & FR_VALID)) continue;
      const int rid = sid[j];
      const bool fast = fast_ok && (r.flags & FR_FAST);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if (r.xmax + pad < sxl[p] || r.xmin - pad > sxh[p] || r.ymax + pad < syl[p] || r.ymin - pad > syh[p])
          continue;
        if (!pv[p]) continue;
        const float x = xf[p], y = yf[p];
        if (x > r.xmax + pad || x < r.xmin - pad || y > r.ymax + pad || y < r.ymin - pad) continue;
        if (fast && fast_reject(r, x, y)) continue;
        FragEval e;
        if (eval_face(r, x, y, pad, P.blur, P.persp, P.clipb, e) && frag_less(e.pz, rid, bz[p], bf[p])) {
          bz[p] = e.pz;
          bf[p] = rid;
        }
      }
    }
  }

  // epilogue
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (!pv[p]) continue;
    const int px = rx0 + (p & 1) * 8 + lx, py = ry0 + (p >> 1) * 8 + ly;
    const int64_t pix = ((int64_t)n * H + py) * W + px;
    FragEval e;
    FaceRec r;
    bool hit = bf[p] >= 0;
    if (hit) {
      r = P.recs[bf[p]];
      hit = eval_face(r, xf[p], yf[p], pad, P.blur, P.persp, P.clipb, e);  // recompute (deterministic)
    }
    if (MODE == 0) {
      if (hit) {
        P.p2f[pix] = bf[p];
        P.zbuf[pix] = e.pz;
        P.bary[3 * pix + 0] = e.b0;
        P.bary[3 * pix + 1] = e.b1;
        P.bary[3 * pix + 2] = e.b2;
        P.dists[pix] = e.sdist;
      } else {
        P.p2f[pix] = -1;
        P.zbuf[pix] = -1.0f;
        P.bary[3 * pix + 0] = -1.0f;
        P.bary[3 * pix + 1] = -1.0f;
        P.bary[3 * pix + 2] = -1.0f;
        P.dists[pix] = -1.0f;
      }
    } else {
      PixGeom G;
      ShadeOut o;
      ShadeCache C;
      if (hit) gather_geom(P.S, r.face, G);
      shade_fwd(P.S, n, hit, G, hit ? e.b0 : 0.f, hit ? e.b1 : 0.f, hit ? e.b2 : 0.f, hit ? e.pz : 0.f,
                hit ? e.sdist : 0.f, o, C);
      if (P.out_flags & MR_OUT_DEPTH) P.depth[pix] = o.depth;
      if (P.out_flags & MR_OUT_SIL) P.sil[pix] = o.sil;
      if (P.out_flags & MR_OUT_RGB) {
        float* q = P.rgb + pix * P.rgb_ch;
        q[0] = o.rgb[0];
        q[1] = o.rgb[1];
        q[2] = o.rgb[2];
        if (P.rgb_ch == 4) q[3] = o.alpha;
      }
      P.p2f32[pix] = hit ? bf[p] : -1;
    }
  }
}

// ---------------------------------------------------------------------------
// 3. backward
// ---------------------------------------------------------------------------
// LDS hash: face key -> slot holding ACC partial sums.
template <int ACC>
struct LdsAcc {
  int keys[MR_HT];
  float acc[MR_HT * ACC];
};

MR_DEV int ht_slot(int* keys, int key) {
  unsigned h = ((unsigned)key * 2654435761u) >> (32 - 9);
#pragma unroll 1
  for (int probe = 0; probe < 16; ++probe) {
    const int k = keys[h];
    if (k == key) return (int)h;
    if (k == -1) {
      const int old = atomicCAS(&keys[h], -1, key);
      if (old == -1 || old == key) return (int)h;
    }
    h = (h + 1) & (MR_HT - 1);
  }
  return -1;
}

template <int ACC>
MR_DEV void acc_add(LdsAcc<ACC>& L, float* __restrict__ gdst, int key, const float* v) {
  const int s = ht_slot(L.keys, key);
  if (s >= 0) {
#pragma unroll
    for (int i = 0; i < ACC; ++i)
      if (v[i] != 0.0f) atomicAdd(&L.acc[s * ACC + i], v[i]);
  } else {
#pragma unroll
    for (int i = 0; i < ACC; ++i)
      if (v[i] != 0.0f) atomicAdd(&gdst[(int64_t)key * ACC + i], v[i]);
  }
}

template <int ACC>
MR_DEV void acc_init(LdsAcc<ACC>& L) {
  for (int i = threadIdx.x; i < MR_HT; i += blockDim.x) L.keys[i] = -1;
  for (int i = threadIdx.x; i < MR_HT * ACC; i += blockDim.x) L.acc[i] = 0.0f;
}

template <int ACC>
MR_DEV void acc_flush(LdsAcc<ACC>& L, float* __restrict__ gdst) {
  for (int i = threadIdx.x; i < MR_HT * ACC; i += blockDim.x) {
    const int s = i / ACC;
    const int k = L.keys[s];
    const float v = L.acc[i];
    if (k >= 0 && v != 0.0f) atomicAdd(&gdst[(int64_t)k * ACC + (i - s * ACC)], v);
  }
}

// Modular backward (PyTorch3D _C.rasterize_meshes_backward), K = 1.
struct RasterBwdParams {
  int N, H, W, NSTX, NST;
  int persp, clipb;
  const float* fv;
  const int64_t* p2f;
  const float* gz;
  const float* gb;
  const float* gd;
  float* gfv;
};

__global__ void __launch_bounds__(256) k_raster_bwd(RasterBwdParams P) {
  __shared__ LdsAcc<9> L;
  acc_init(L);
  __syncthreads();
  const int n = blockIdx.y, st = blockIdx.x;
  const int stx = st % P.NSTX, sty = st / P.NSTX;
  const int px = stx * MR_ST + (threadIdx.x & 31);
  for (int k = 0; k < 4; ++k) {
    const int py = sty * MR_ST + (threadIdx.x >> 5) + 8 * k;
    if (px >= P.W || py >= P.H) continue;
    const int64_t pix = ((int64_t)n * P.H + py) * P.W + px;
    const int64_t f = P.p2f[pix];
    if (f < 0) continue;
    FaceRec r;
    const float* v = P.fv + 9 * f;
    r.x0 = v[0]; r.y0 = v[1]; r.z0 = v[2];
    r.x1 = v[3]; r.y1 = v[4]; r.z1 = v[5];
    r.x2 = v[6]; r.y2 = v[7]; r.z2 = v[8];
    r.area = (float)((double)edge_fn(r.x2, r.y2, r.x0, r.y0, r.x1, r.y1) + MR_KEPS_D);
    const float gb[3] = {P.gb[3 * pix], P.gb[3 * pix + 1], P.gb[3 * pix + 2]};
    float g[3][3];
    raster_bwd_pixel(r, col_ndc(px, P.H, P.W), row_ndc(py, P.H, P.W), P.persp, P.clipb, P.gz[pix], gb, P.gd[pix], g);
    acc_add<9>(L, P.gfv, (int)f, &g[0][0]);
  }
  __syncthreads();
  acc_flush(L, P.gfv);
}

// Fused render backward.
struct RenderBwdParams {
  int N, H, W, NSTX, NST;
  float blur, bbox_pad;
  int persp, clipb;
  const FaceRec* recs;
  const int32_t* p2f32;
  const float* gD;
  const float* gS;
  const float* gRGB;
  int rgb_ch;
  ShadeParams S;
  const ViewRec* views;
  float* gface;   // (F, ACC)
  float* rt_part; // (N*NST, 12)
};

template <int ACC>
__global__ void __launch_bounds__(256) k_render_bwd(RenderBwdParams P) {
  __shared__ LdsAcc<ACC> L;
  __shared__ float red[4][12];
  acc_init(L);
  __syncthreads();
  const int n = blockIdx.y, st = blockIdx.x;
  const int stx = st % P.NSTX, sty = st / P.NSTX;
  const int px = stx * MR_ST + (threadIdx.x & 31);
  const ViewRec V = P.views[n];
  float gR[9], gT[3];
  for (int i = 0; i < 9; ++i) gR[i] = 0.0f;
  for (int i = 0; i < 3; ++i) gT[i] = 0.0f;
  for (int k = 0; k < 4; ++k) {
    const int py = sty * MR_ST + (threadIdx.x >> 5) + 8 * k;
    if (px >= P.W || py >= P.H) continue;
    const int64_t pix = ((int64_t)n * P.H + py) * P.W + px;
    const int rid = P.p2f32[pix];
    if (rid < 0) continue;
    const FaceRec r = P.recs[rid];
    const float xf = col_ndc(px, P.H, P.W), yf = row_ndc(py, P.H, P.W);
    FragEval e;
    if (!eval_face(r, xf, yf, P.bbox_pad, P.blur, P.persp, P.clipb, e)) continue;
    PixGeom G;
    gather_geom(P.S, r.face, G);
    ShadeOut o;
    ShadeCache C;
    shade_fwd(P.S, n, true, G, e.b0, e.b1, e.b2, e.pz, e.sdist, o, C);
    const float gD = P.gD ? P.gD[pix] : 0.0f;
    const float gS = P.gS ? P.gS[pix] : 0.0f;
    float gC[3] = {0.f, 0.f, 0.f}, gA = 0.0f;
    if (P.gRGB) {
      const float* q = P.gRGB + pix * P.rgb_ch;
      gC[0] = q[0];
      gC[1] = q[1];
      gC[2] = q[2];
      if (P.rgb_ch == 4) gA = q[3];
    }
    ShadeGrad SG;
    shade_bwd(P.S, G, e.b0, e.b1, e.b2, e.pz, C, gD, gS, gC, gA, SG);
    float gfv[3][3];
    raster_bwd_pixel(r, xf, yf, P.persp, P.clipb, SG.gz, SG.gb, SG.gsd, gfv);
    float row[ACC];
    for (int c = 0; c < 3; ++c) {
      float gX[3];
      project_bwd(V, G.X[c], gfv[c], gX, gR, gT);
      for (int a = 0; a < 3; ++a) {
        row[3 * c + a] = SG.gX[c][a] + gX[a];
        row[9 + 3 * c + a] = SG.gN[c][a];
        if (ACC == 27) row[18 + 3 * c + a] = SG.gC[c][a];
      }
    }
    acc_add<ACC>(L, P.gface, (int)r.face, row);
  }
  // per-view R/T partial sums: wave shuffle + LDS across the 4 waves
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = 0; i < 12; ++i) {
    float v = i < 9 ? gR[i] : gT[i - 9];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wave][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < 12) {
    const int i = threadIdx.x;
    P.rt_part[((int64_t)n * P.NST + st) * 12 + i] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
  }
  acc_flush(L, P.gface);
}

__global__ void __launch_bounds__(256) k_rt_reduce(const float* __restrict__ part, int NST, float* __restrict__ out) {
  __shared__ float s[256];
  const int n = blockIdx.x;
  for (int i = 0; i < 12; ++i) {
    float v = 0.0f;
    for (int t = threadIdx.x; t < NST; t += 256) v += part[((int64_t)n * NST + t) * 12 + i];
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (threadIdx.x < o) s[threadIdx.x] += s[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) out[n * 12 + i] = s[0];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// 4. vertex kernels (CSR adjacency, entries (face << 2 | corner) sorted by (corner, face))
// ---------------------------------------------------------------------------
MR_DEV void face_normal(const float* verts, const int32_t* faces, int f, float nf[3]) {
  const int32_t i0 = faces[3 * f], i1 = faces[3 * f + 1], i2 = faces[3 * f + 2];
  float a[3], b[3];
  for (int k = 0; k < 3; ++k) {
    a[k] = verts[3 * i2 + k] - verts[3 * i1 + k];
    b[k] = verts[3 * i0 + k] - verts[3 * i1 + k];
  }
  nf[0] = a[1] * b[2] - a[2] * b[1];
  nf[1] = a[2] * b[0] - a[0] * b[2];
  nf[2] = a[0] * b[1] - a[1] * b[0];
}

__global__ void __launch_bounds__(256) k_vertex_normals(const float* __restrict__ verts, int64_t V,
                                                        const int32_t* __restrict__ faces,
                                                        const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj,
                                                        float* __restrict__ vn, float* __restrict__ vraw) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  float s[3] = {0.f, 0.f, 0.f};
  for (int e = ptr[v]; e < ptr[v + 1]; ++e) {
    float nf[3];
    face_normal(verts, faces, adj[e] >> 2, nf);
    s[0] += nf[0];
    s[1] += nf[1];
    s[2] += nf[2];
  }
  float y[3], nrm, den;
  normalize3(s, y, nrm, den);
  for (int k = 0; k < 3; ++k) {
    vn[3 * v + k] = y[k];
    vraw[3 * v + k] = s[k];
  }
}

// A: gNu[v] = normalize_bwd(raw[v], sum of gface normal rows)
template <int ACC>
__global__ void __launch_bounds__(256) k_vgrad_a(int64_t V, const int32_t* __restrict__ ptr,
                                                 const int32_t* __restrict__ adj, const float* __restrict__ gface,
                                                 const float* __restrict__ vraw, float* __restrict__ gnu) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  float g[3] = {0.f, 0.f, 0.f};
  for (int e = ptr[v]; e < ptr[v + 1]; ++e) {
    const int f = adj[e] >> 2, c = adj[e] & 3;
    for (int k = 0; k < 3; ++k) g[k] += gface[(int64_t)f * ACC + 9 + 3 * c + k];
  }
  const float x[3] = {vraw[3 * v], vraw[3 * v + 1], vraw[3 * v + 2]};
  const float nrm = sqrtf(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  const float den = smax(nrm, 1e-6f);
  float gx[3];
  normalize3_bwd(x, nrm, den, g, gx);
  for (int k = 0; k < 3; ++k) gnu[3 * v + k] = gx[k];
}

// B: grad_verts[v] = sum over incident (f, c) of position rows + cross-product backward of the face normal.
template <int ACC>
__global__ void __launch_bounds__(256) k_vgrad_b(int64_t V, const float* __restrict__ verts,
                                                 const int32_t* __restrict__ faces, const int32_t* __restrict__ ptr,
                                                 const int32_t* __restrict__ adj, const float* __restrict__ gface,
                                                 const float* __restrict__ gnu, int use_normals,
                                                 float* __restrict__ gverts, float* __restrict__ gcol) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  float g[3] = {0.f, 0.f, 0.f}, gc[3] = {0.f, 0.f, 0.f};
  for (int e = ptr[v]; e < ptr[v + 1]; ++e) {
    const int f = adj[e] >> 2, c = adj[e] & 3;
    for (int k = 0; k < 3; ++k) g[k] += gface[(int64_t)f * ACC + 3 * c + k];
    if (ACC == 27)
      for (int k = 0; k < 3; ++k) gc[k] += gface[(int64_t)f * ACC + 18 + 3 * c + k];
    if (use_normals) {
      const int32_t i0 = faces[3 * f], i1 = faces[3 * f + 1], i2 = faces[3 * f + 2];
      float gn[3], a[3], b[3];
      for (int k = 0; k < 3; ++k) {
        gn[k] = (gnu[3 * i0 + k] + gnu[3 * i1 + k]) + gnu[3 * i2 + k];
        a[k] = verts[3 * i2 + k] - verts[3 * i1 + k];
        b[k] = verts[3 * i0 + k] - verts[3 * i1 + k];
      }
      // n = a x b : ga = b x gn, gb = gn x a
      const float ga[3] = {b[1] * gn[2] - b[2] * gn[1], b[2] * gn[0] - b[0] * gn[2], b[0] * gn[1] - b[1] * gn[0]};
      const float gb[3] = {gn[1] * a[2] - gn[2] * a[1], gn[2] * a[0] - gn[0] * a[2], gn[0] * a[1] - gn[1] * a[0]};
      for (int k = 0; k < 3; ++k) {
        if (c == 0) g[k] += gb[k];
        else if (c == 1) g[k] += -(ga[k] + gb[k]);
        else g[k] += ga[k];
      }
    }
  }
  for (int k = 0; k < 3; ++k) gverts[3 * v + k] = g[k];
  if (ACC == 27 && gcol)
    for (int k = 0; k < 3; ++k) gcol[3 * v + k] = gc[k];
}

// projection: face_verts[n*F+f][c] = ndc(view n, X)
__global__ void __launch_bounds__(256) k_project_faces(const float* __restrict__ verts, const int32_t* __restrict__ faces,
                                                       int64_t F, const ViewRec* __restrict__ views, float* __restrict__ fv) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = blockIdx.y;
  if (f >= F) return;
  const ViewRec V = views[n];
  for (int c = 0; c < 3; ++c) {
    const int32_t vi = faces[3 * f + c];
    const float X[3] = {verts[3 * (int64_t)vi], verts[3 * (int64_t)vi + 1], verts[3 * (int64_t)vi + 2]};
    float vx, vy, vz, nx, ny;
    project_point(V, X, vx, vy, vz, nx, ny);
    float* o = fv + (((int64_t)n * F + f) * 3 + c) * 3;
    o[0] = nx;
    o[1] = ny;
    o[2] = vz;
  }
}

// projection backward: thread per (n, v); grads summed over incident faces (CSR order).
__global__ void __launch_bounds__(256) k_project_faces_bwd(const float* __restrict__ verts, int64_t V, int64_t F,
                                                           const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj,
                                                           const ViewRec* __restrict__ views,
                                                           const float* __restrict__ gfv, float* __restrict__ gverts,
                                                           float* __restrict__ gviews) {
  __shared__ float red[4][12];
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = blockIdx.y;
  const ViewRec Vw = views[n];
  float gR[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, gT[3] = {0, 0, 0};
  if (v < V) {
    float gn[3] = {0.f, 0.f, 0.f};
    for (int e = ptr[v]; e < ptr[v + 1]; ++e) {
      const int f = adj[e] >> 2, c = adj[e] & 3;
      const float* q = gfv + (((int64_t)n * F + f) * 3 + c) * 3;
      gn[0] += q[0];
      gn[1] += q[1];
      gn[2] += q[2];
    }
    const float X[3] = {verts[3 * v], verts[3 * v + 1], verts[3 * v + 2]};
    float gX[3];
    project_bwd(Vw, X, gn, gX, gR, gT);
    for (int k = 0; k < 3; ++k) atomicAdd(&gverts[3 * v + k], gX[k]);
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = 0; i < 12; ++i) {
    float x = i < 9 ? gR[i] : gT[i - 9];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane == 0) red[wave][i] = x;
  }
  __syncthreads();
  if (threadIdx.x < 12) {
    const int i = threadIdx.x;
    atomicAdd(&gviews[n * 12 + i], ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i]);
  }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* mr_last_error(void) { return g_err; }
int32_t mr_version(void) { return 1; }

static int check_settings(const mr_raster_settings_t* s) {
  if (!s) return set_err(MR_EINVAL, "settings is NULL");
  if (s->H <= 0 || s->W <= 0) return set_err(MR_EINVAL, "image size must be positive (got %d x %d)", s->H, s->W);
  if (s->H > 8192 || s->W > 8192) return set_err(MR_EUNSUPPORTED, "image size above 8192");
  if (s->faces_per_pixel != 1)
    return set_err(MR_EUNSUPPORTED, "faces_per_pixel=%d: only 1 is implemented on the MI355X path", s->faces_per_pixel);
  if (!(s->blur_radius >= 0.0f) || !__builtin_isfinite(s->blur_radius))
    return set_err(MR_EINVAL, "blur_radius must be finite and >= 0");
  return MR_OK;
}

size_t mr_rasterize_meshes_workspace(int64_t num_meshes, int64_t total_faces, int32_t H, int32_t W,
                                     int32_t max_faces_per_bin) {
  TileGeom g = tile_geom(H, W, total_faces, max_faces_per_bin);
  return carve_raster_ws(nullptr, num_meshes, total_faces, g).bytes;
}

static SetupParams make_setup(const mr_raster_settings_t* s, const TileGeom& g, const RasterWS& w) {
  SetupParams P;
  P.H = s->H; P.W = s->W; P.NSTX = g.NSTX; P.NSTY = g.NSTY; P.NST = g.NST; P.cap = g.cap;
  P.bbox_pad = sqrtf(s->blur_radius);
  P.persp = s->perspective_correct;
  P.cull = s->cull_backfaces;
  P.recs = w.recs;
  P.bin_count = w.bin_count;
  P.bin_faces = w.bin_faces;
  return P;
}

static RasterParams make_raster(const mr_raster_settings_t* s, const TileGeom& g, const RasterWS& w, int64_t N) {
  RasterParams P;
  memset(&P, 0, sizeof(P));
  P.N = (int)N; P.H = s->H; P.W = s->W;
  P.NSTX = g.NSTX; P.NSTY = g.NSTY; P.NST = g.NST; P.cap = g.cap;
  P.blur = s->blur_radius;
  P.bbox_pad = sqrtf(s->blur_radius);
  P.persp = s->perspective_correct;
  P.clipb = s->clip_barycentric_coords;
  P.recs = w.recs;
  P.bin_count = w.bin_count;
  P.bin_faces = w.bin_faces;
  return P;
}

int32_t mr_rasterize_meshes(const float* face_verts, const int64_t* first, const int64_t* count, int64_t N,
                            int64_t Ftot, const mr_raster_settings_t* s, int64_t* p2f, float* zbuf, float* bary,
                            float* dists, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "num_meshes must be in [1, 65535] (got %lld)", (long long)N);
  if (Ftot < 0 || Ftot >= (1ll << 31)) return set_err(MR_EINVAL, "total_faces out of range");
  if (!p2f || !zbuf || !bary || !dists || !first || !count || (Ftot > 0 && !face_verts))
    return set_err(MR_EINVAL, "NULL tensor argument");
  hipStream_t st = (hipStream_t)stream;
  const int64_t Fbound = Ftot > 0 ? Ftot : 1;
  TileGeom g = tile_geom(s->H, s->W, Fbound, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws(ws, N, Fbound, g);
  if (ws_bytes < w.bytes) return set_err(MR_EWORKSPACE, "workspace too small: %zu < %zu", ws_bytes, w.bytes);
  if (hipMemsetAsync(w.bin_count, 0, sizeof(int) * (size_t)N * g.NST, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  if (Ftot > 0) {
    SetupParams SP = make_setup(s, g, w);
    k_setup_fv<<<ceil_div(Ftot, 256), 256, 0, st>>>(SP, face_verts, Ftot, first, N);
    MR_CHECK_LAUNCH("k_setup_fv");
  }
  RasterParams P = make_raster(s, g, w, N);
  P.view_first = first;
  P.view_count = count;
  P.F = 0;
  P.p2f = p2f; P.zbuf = zbuf; P.bary = bary; P.dists = dists;
  dim3 grid(g.NST, (unsigned)N);
  k_raster<0><<<grid, 256, 0, st>>>(P);
  MR_CHECK_LAUNCH("k_raster<0>");
  return MR_OK;
}

int32_t mr_rasterize_meshes_backward(const float* fv, const int64_t* p2f, const float* gz, const float* gb,
                                     const float* gd, int64_t N, int64_t Ftot, const mr_raster_settings_t* s,
                                     float* gfv, void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "num_meshes out of range");
  if (!p2f || !gz || !gb || !gd || !gfv) return set_err(MR_EINVAL, "NULL tensor argument");
  hipStream_t st = (hipStream_t)stream;
  if (Ftot > 0 && hipMemsetAsync(gfv, 0, sizeof(float) * 9 * (size_t)Ftot, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  if (Ftot == 0) return MR_OK;
  TileGeom g = tile_geom(s->H, s->W, Ftot, s->max_faces_per_bin);
  RasterBwdParams P;
  P.N = (int)N; P.H = s->H; P.W = s->W; P.NSTX = g.NSTX; P.NST = g.NST;
  P.persp = s->perspective_correct; P.clipb = s->clip_barycentric_coords;
  P.fv = fv; P.p2f = p2f; P.gz = gz; P.gb = gb; P.gd = gd; P.gfv = gfv;
  dim3 grid(g.NST, (unsigned)N);
  k_raster_bwd<<<grid, 256, 0, st>>>(P);
  MR_CHECK_LAUNCH("k_raster_bwd");
  return MR_OK;
}

int32_t mr_project_faces(const float* verts, int64_t V, const int32_t* faces, int64_t F, const mr_view_t* views,
                         int64_t N, float* fv, void* stream) {
  if (N <= 0 || N > 65535 || F < 0 || V < 0) return set_err(MR_EINVAL, "bad sizes");
  if (F == 0) return MR_OK;
  if (!verts || !faces || !views || !fv) return set_err(MR_EINVAL, "NULL argument");
  dim3 grid(ceil_div(F, 256), (unsigned)N);
  k_project_faces<<<grid, 256, 0, (hipStream_t)stream>>>(verts, faces, F, (const ViewRec*)views, fv);
  MR_CHECK_LAUNCH("k_project_faces");
  return MR_OK;
}

int32_t mr_project_faces_backward(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                                  const int32_t* ptr, const int32_t* adj, const mr_view_t* views, int64_t N,
                                  const float* gfv, float* gverts, float* gviews, void* stream) {
  (void)faces;
  if (N <= 0 || N > 65535 || F < 0 || V < 0) return set_err(MR_EINVAL, "bad sizes");
  hipStream_t st = (hipStream_t)stream;
  if (V > 0 && hipMemsetAsync(gverts, 0, sizeof(float) * 3 * (size_t)V, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  if (hipMemsetAsync(gviews, 0, sizeof(float) * 12 * (size_t)N, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  if (V == 0) return MR_OK;
  dim3 grid(ceil_div(V, 256), (unsigned)N);
  k_project_faces_bwd<<<grid, 256, 0, st>>>(verts, V, F, ptr, adj, (const ViewRec*)views, gfv, gverts, gviews);
  MR_CHECK_LAUNCH("k_project_faces_bwd");
  return MR_OK;
}

int32_t mr_vertex_normals(const float* verts, int64_t V, const int32_t* faces, int64_t F, const int32_t* ptr,
                          const int32_t* adj, float* vn, float* vraw, void* stream) {
  (void)F;
  if (V <= 0) return MR_OK;
  k_vertex_normals<<<ceil_div(V, 256), 256, 0, (hipStream_t)stream>>>(verts, V, faces, ptr, adj, vn, vraw);
  MR_CHECK_LAUNCH("k_vertex_normals");
  return MR_OK;
}

static ShadeParams make_shade(const mr_mesh_t* m, const mr_shade_params_t* sp, const float* cc, int64_t ncc) {
  ShadeParams S;
  memset(&S, 0, sizeof(S));
  S.verts = m->verts;
  S.faces = m->faces;
  S.vnormals = m->vnormals;
  S.tex_kind = m->tex_kind;
  S.vcolors = m->vcolors;
  S.verts_uvs = m->verts_uvs;
  S.faces_uvs = m->faces_uvs;
  S.tex = (const float4*)m->tex_rgba;
  S.tex_h = m->tex_h;
  S.tex_w = m->tex_w;
  S.light_kind = sp->light_kind;
  for (int k = 0; k < 3; ++k) {
    S.light_loc[k] = sp->light_location[k];
    S.light_amb[k] = sp->light_ambient[k];
    S.light_diff[k] = sp->light_diffuse[k];
    S.light_spec[k] = sp->light_specular[k];
    S.mat_amb[k] = sp->mat_ambient[k];
    S.mat_diff[k] = sp->mat_diffuse[k];
    S.mat_spec[k] = sp->mat_specular[k];
    S.bg[k] = sp->background[k];
  }
  S.shininess = sp->shininess;
  S.cam_centers = cc;
  S.cam_center_stride = ncc > 1 ? 3 : 0;
  S.sigma_rgb = sp->sigma_rgb;
  S.gamma = sp->gamma;
  S.znear = sp->znear;
  S.zfar = sp->zfar;
  S.sigma_sil = sp->sigma_sil;
  return S;
}

static int check_mesh(const mr_mesh_t* m, const mr_shade_params_t* sp) {
  if (!m || !sp) return set_err(MR_EINVAL, "NULL mesh/shade params");
  if (m->V <= 0 || m->F <= 0) return set_err(MR_EINVAL, "empty mesh");
  if (m->F >= (1ll << 29)) return set_err(MR_EUNSUPPORTED, "too many faces");
  if (!m->verts || !m->faces || !m->vadj_ptr || !m->vadj) return set_err(MR_EINVAL, "NULL mesh array");
  if (sp->light_kind == 0 && !m->vnormals) return set_err(MR_EINVAL, "point lights need vertex normals");
  if (m->tex_kind == 1 && !m->vcolors) return set_err(MR_EINVAL, "vertex texture without colours");
  if (m->tex_kind == 2 && (!m->verts_uvs || !m->faces_uvs || !m->tex_rgba || m->tex_h < 1 || m->tex_w < 1))
    return set_err(MR_EINVAL, "UV texture arrays missing");
  if (sp->rgb_channels != 3 && sp->rgb_channels != 4) return set_err(MR_EINVAL, "rgb_channels must be 3 or 4");
  return MR_OK;
}

size_t mr_render_workspace(int64_t N, int64_t F, int32_t H, int32_t W, int32_t max_faces_per_bin) {
  TileGeom g = tile_geom(H, W, F, max_faces_per_bin);
  return carve_raster_ws(nullptr, N, N * F, g).bytes;
}

int32_t mr_render_forward(const mr_mesh_t* m, const mr_view_t* views, int64_t N, const float* cc, int64_t ncc,
                          const mr_raster_settings_t* s, const mr_shade_params_t* sp, float* depth, float* sil,
                          float* rgb, int32_t* p2f32, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  rc = check_mesh(m, sp);
  if (rc) return rc;
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "N out of range");
  if ((int64_t)N * m->F >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "N*F >= 2^31");
  if (!p2f32 || !views) return set_err(MR_EINVAL, "NULL output");
  if ((sp->out_flags & MR_OUT_DEPTH) && !depth) return set_err(MR_EINVAL, "depth output NULL");
  if ((sp->out_flags & MR_OUT_SIL) && !sil) return set_err(MR_EINVAL, "silhouette output NULL");
  if ((sp->out_flags & MR_OUT_RGB) && !rgb) return set_err(MR_EINVAL, "rgb output NULL");
  if (sp->light_kind == 0 && (!cc || (ncc != 1 && ncc != N))) return set_err(MR_EINVAL, "camera centres");
  hipStream_t st = (hipStream_t)stream;
  TileGeom g = tile_geom(s->H, s->W, m->F, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws(ws, N, N * m->F, g);
  if (ws_bytes < w.bytes) return set_err(MR_EWORKSPACE, "workspace too small: %zu < %zu", ws_bytes, w.bytes);
  if (hipMemsetAsync(w.bin_count, 0, sizeof(int) * (size_t)N * g.NST, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  SetupParams SP = make_setup(s, g, w);
  dim3 sgrid(ceil_div(m->F, 256), (unsigned)N);
  k_setup_world<<<sgrid, 256, 0, st>>>(SP, m->verts, m->faces, m->F, (const ViewRec*)views);
  MR_CHECK_LAUNCH("k_setup_world");
  RasterParams P = make_raster(s, g, w, N);
  P.view_first = nullptr;
  P.view_count = nullptr;
  P.F = m->F;
  P.S = make_shade(m, sp, cc, ncc);
  P.out_flags = sp->out_flags;
  P.rgb_ch = sp->rgb_channels;
  P.depth = depth;
  P.sil = sil;
  P.rgb = rgb;
  P.p2f32 = p2f32;
  dim3 grid(g.NST, (unsigned)N);
  k_raster<1><<<grid, 256, 0, st>>>(P);
  MR_CHECK_LAUNCH("k_raster<1>");
  return MR_OK;
}

size_t mr_render_backward_workspace(int64_t N, int64_t V, int64_t F, int32_t H, int32_t W) {
  const int NST = ceil_div(W, MR_ST) * ceil_div(H, MR_ST);
  size_t off = align_up(sizeof(float) * 27 * (size_t)F, 256);
  off = align_up(off + sizeof(float) * 12 * (size_t)N * NST, 256);
  off = align_up(off + sizeof(float) * 3 * (size_t)V, 256);
  return off;
}

int32_t mr_render_backward(const mr_mesh_t* m, const float* vraw, const mr_view_t* views, int64_t N, const float* cc,
                           int64_t ncc, const mr_raster_settings_t* s, const mr_shade_params_t* sp,
                           const int32_t* p2f32, const float* gD, const float* gS, const float* gRGB,
                           const void* fws, void* bws, size_t bws_bytes, float* gverts, float* gviews, float* gcol,
                           void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  rc = check_mesh(m, sp);
  if (rc) return rc;
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "N out of range");
  if (!p2f32 || !fws || !bws || !gverts || !gviews) return set_err(MR_EINVAL, "NULL argument");
  if (sp->light_kind == 0 && !vraw) return set_err(MR_EINVAL, "raw vertex normals required");
  const size_t need = mr_render_backward_workspace(N, m->V, m->F, s->H, s->W);
  if (bws_bytes < need) return set_err(MR_EWORKSPACE, "backward workspace too small");
  hipStream_t st = (hipStream_t)stream;
  TileGeom g = tile_geom(s->H, s->W, m->F, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws((void*)fws, N, N * m->F, g);
  const bool vcol = m->tex_kind == 1;
  const int ACC = vcol ? 27 : 18;
  char* b = (char*)bws;
  float* gface = (float*)b;
  size_t off = align_up(sizeof(float) * 27 * (size_t)m->F, 256);
  float* rt_part = (float*)(b + off);
  off = align_up(off + sizeof(float) * 12 * (size_t)N * g.NST, 256);
  float* gnu = (float*)(b + off);
  if (hipMemsetAsync(gface, 0, sizeof(float) * ACC * (size_t)m->F, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  RenderBwdParams P;
  memset(&P, 0, sizeof(P));
  P.N = (int)N; P.H = s->H; P.W = s->W; P.NSTX = g.NSTX; P.NST = g.NST;
  P.blur = s->blur_radius; P.bbox_pad = sqrtf(s->blur_radius);
  P.persp = s->perspective_correct; P.clipb = s->clip_barycentric_coords;
  P.recs = w.recs;
  P.p2f32 = p2f32;
  P.gD = (sp->out_flags & MR_OUT_DEPTH) ? gD : nullptr;
  P.gS = (sp->out_flags & MR_OUT_SIL) ? gS : nullptr;
  P.gRGB = (sp->out_flags & MR_OUT_RGB) ? gRGB : nullptr;
  P.rgb_ch = sp->rgb_channels;
  P.S = make_shade(m, sp, cc, ncc);
  P.views = (const ViewRec*)views;
  P.gface = gface;
  P.rt_part = rt_part;
  dim3 grid(g.NST, (unsigned)N);
  if (vcol) k_render_bwd<27><<<grid, 256, 0, st>>>(P);
  else k_render_bwd<18><<<grid, 256, 0, st>>>(P);
  MR_CHECK_LAUNCH("k_render_bwd");
  k_rt_reduce<<<(unsigned)N, 256, 0, st>>>(rt_part, g.NST, gviews);
  MR_CHECK_LAUNCH("k_rt_reduce");
  const int use_n = sp->light_kind == 0;
  const int vb = ceil_div(m->V, 256);
  if (vcol) {
    if (use_n) k_vgrad_a<27><<<vb, 256, 0, st>>>(m->V, m->vadj_ptr, m->vadj, gface, vraw, gnu);
    k_vgrad_b<27><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, gface, gnu, use_n, gverts, gcol);
  } else {
    if (use_n) k_vgrad_a<18><<<vb, 256, 0, st>>>(m->V, m->vadj_ptr, m->vadj, gface, vraw, gnu);
    k_vgrad_b<18><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, gface, gnu, use_n, gverts, gcol);
  }
  MR_CHECK_LAUNCH("k_vgrad");
  return MR_OK;
}

}  // extern "C"
