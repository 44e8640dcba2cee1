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

#define MR_TS 8         // raster tile edge: one 64-lane wave per 8x8 tile (lane = pixel)
#define MR_BT 32        // tile edge of the modular (fragments) backward
#define MR_HT 512       // LDS hash slots in the backward
#define MR_LDS_HIST 16384  // per-view tiles binned through an LDS histogram (else global atomics)

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

// ---------------------------------------------------------------------------
// Optional per-kernel timing: HIP events recorded on the launch stream around
// every kernel while enabled (bench.py reads them to price the dominant kernel).
// ---------------------------------------------------------------------------
enum KernelId { KID_BIN_COUNT, KID_BIN_SCAN, KID_BIN_FILL, KID_RASTER_FRAG, KID_RASTER_RENDER, KID_RASTER_BWD,
                KID_RENDER_BWD, KID_RT_REDUCE, KID_VGRAD_A, KID_VGRAD_B, KID_VNORMALS, KID_PROJECT, KID_PROJECT_BWD,
                KID_BG, KID_COUNT };
static const char* kKernelNames[KID_COUNT] = {"k_bin_count", "k_bin_scan", "k_bin_fill", "k_raster<0>", "k_raster<1>",
                                              "k_raster_bwd", "k_render_bwd", "k_rt_reduce", "k_vgrad_a",
                                              "k_vgrad_b", "k_vertex_normals", "k_project_faces",
                                              "k_project_faces_bwd", "k_bg"};
#define MR_TPOOL 4096
static struct {
  int enabled;
  int created;
  hipEvent_t ev[2 * MR_TPOOL];
  int kid[MR_TPOOL];
  int used;
  int dropped;
} g_t;

static int timing_begin(hipStream_t st) {
  if (!g_t.enabled || g_t.used >= MR_TPOOL) {
    if (g_t.enabled) g_t.dropped++;
    return -1;
  }
  const int i = g_t.used++;
  (void)hipEventRecord(g_t.ev[2 * i], st);
  return i;
}
static void timing_end(int i, int kid, hipStream_t st) {
  if (i < 0) return;
  g_t.kid[i] = kid;
  (void)hipEventRecord(g_t.ev[2 * i + 1], st);
}
#define MR_TIMED(kid, st, launch)              \
  do {                                         \
    const int _ti = timing_begin(st);          \
    launch;                                    \
    timing_end(_ti, kid, st);                  \
  } while (0)

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
static inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------------------
// Workspace: face records, per-(view, 8x8 tile) face lists (count -> scan ->
// fill), and the compact per-view list of covered pixels (fused path).
// ---------------------------------------------------------------------------
struct BinGeom {
  int TX, TY, T;
  int GX, S;  // 64x8-pixel strips: GX per strip row, S = GX * TY per view
  int64_t list_cap;
};
static BinGeom bin_geom(int H, int W, int64_t N, int64_t Ftot, int32_t mfpb) {
  BinGeom g;
  g.TX = ceil_div(W, MR_TS);
  g.TY = ceil_div(H, MR_TS);
  g.T = g.TX * g.TY;
  g.GX = ceil_div(g.TX, 8);
  g.S = g.GX * g.TY;
  // Expected entries: ~(1 + 2*edge/8)^2 tiles per face + large faces; overflowing tiles take
  // the exact full-view path. max_faces_per_bin (if given) scales the reservation.
  int64_t cap = 6 * Ftot + 2 * N * (int64_t)g.T + 65536;
  if (mfpb > 0) cap = (int64_t)mfpb * N * 16 + 65536;
  g.list_cap = cap;
  return g;
}

struct RasterWS {
  FaceRec* recs;
  int* cnt;    // (N*T) zeroed per call
  int* start;  // (N*T + 1)
  int* cur;    // (N*T)
  int* list;   // list_cap
  int* pcnt;   // (N) covered-pixel counts, zeroed per call (pcnt sits right after cnt)
  int* wctr;   // (4) strips per work bucket [3] + the raster's work counter, zeroed with cnt
  int* scount; // (N*S) entries per strip (0: background strip)
  int* work;   // (3 * N*S) non-empty strip ids per bucket (heavy, medium, light)
  int* vtot;   // (N) per-view list entries
  int* vbase;  // (N+1) exclusive prefix of vtot
  int* plist;  // (N*H*W) covered pixel indices, view-major regions
  size_t bytes;
};
static RasterWS carve_raster_ws(void* base, int64_t N, int64_t Ftot, int H, int W, const BinGeom& g, bool pixlist) {
  RasterWS w;
  size_t off = 0;
  char* b = (char*)base;
  w.recs = (FaceRec*)(b + off);
  off = align_up(off + sizeof(FaceRec) * (size_t)(Ftot > 0 ? Ftot : 1), 256);
  w.cnt = (int*)(b + off);
  w.pcnt = w.cnt + (size_t)N * g.T;
  w.wctr = w.pcnt + N;
  off = align_up(off + sizeof(int) * ((size_t)N * g.T + (size_t)N + 4), 256);
  w.start = (int*)(b + off);
  off = align_up(off + sizeof(int) * ((size_t)N * g.T + 1), 256);
  w.vtot = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)N, 256);
  w.vbase = (int*)(b + off);
  off = align_up(off + sizeof(int) * ((size_t)N + 1), 256);
  w.cur = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)N * g.T, 256);
  w.scount = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)N * g.S, 256);
  w.work = (int*)(b + off);
  off = align_up(off + sizeof(int) * 3 * (size_t)N * g.S, 256);
  w.list = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)g.list_cap, 256);
  w.plist = (int*)(b + off);
  if (pixlist) off = align_up(off + sizeof(int) * (size_t)N * H * W, 256);
  w.bytes = off;
  return w;
}
static size_t zero_bytes(int64_t N, const BinGeom& g) { return sizeof(int) * ((size_t)N * g.T + (size_t)N + 4); }

// ---------------------------------------------------------------------------
// 1. binning: count -> scan -> fill
// ---------------------------------------------------------------------------
struct SetupParams {
  int H, W, TX, TY, T;
  float bbox_pad;
  int persp, cull;
  int64_t list_cap;
  FaceRec* recs;
  int* cnt;
  int* cur;
  int* list;
  const int* vbase;
};

// Inverse of col_ndc/row_ndc (approximate, widened by 0.05 px; the raster
// kernel repeats the exact per-pixel bbox test, so a superset is all we need).
MR_DEV void ndc_range_to_pix(float lo, float hi, int S1, int S2, int& p0, int& p1) {
  float range = 2.0f;
  if (S1 > S2) range = ((float)S1 * range) / (float)S2;
  const float off = range / 2.0f;
  // i = ((ndc + off) * S1 - off) / range ; pixel = S1 - 1 - i
  float i_hi = ((hi + off) * (float)S1 - off) / range;
  float i_lo = ((lo + off) * (float)S1 - off) / range;
  float pf0 = (float)(S1 - 1) - i_hi - 0.05f;  // inverse error is ~1e-4 px; 0.05 px is ample
  float pf1 = (float)(S1 - 1) - i_lo + 0.05f;
  pf0 = fminf(fmaxf(pf0, -2.0f), (float)S1 + 1.0f);
  pf1 = fminf(fmaxf(pf1, -2.0f), (float)S1 + 1.0f);
  p0 = (int)floorf(pf0);
  p1 = (int)ceilf(pf1);
  if (p0 < 0) p0 = 0;
  if (p1 > S1 - 1) p1 = S1 - 1;
}

MR_DEV bool rec_tiles(const SetupParams& P, const FaceRec& r, int& tx0, int& tx1, int& ty0, int& ty1) {
  if (!(r.flags & FR_VALID)) return false;
  int cx0, cx1, cy0, cy1;
  ndc_range_to_pix(r.xmin - P.bbox_pad, r.xmax + P.bbox_pad, P.W, P.H, cx0, cx1);
  ndc_range_to_pix(r.ymin - P.bbox_pad, r.ymax + P.bbox_pad, P.H, P.W, cy0, cy1);
  if (cx0 > cx1 || cy0 > cy1) return false;
  tx0 = cx0 / MR_TS; tx1 = cx1 / MR_TS;
  ty0 = cy0 / MR_TS; ty1 = cy1 / MR_TS;
  return true;
}

MR_DEV FaceRec make_rec(const SetupParams& P, uint32_t face, const float v[3][3]) {
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
  return r;
}

MR_DEV void world_face_verts(const float* __restrict__ verts, const int32_t* __restrict__ faces, int64_t f,
                             const ViewRec& V, float v[3][3]) {
  for (int c = 0; c < 3; ++c) {
    const int32_t vi = faces[3 * f + c];
    const float X[3] = {verts[3 * (int64_t)vi], verts[3 * (int64_t)vi + 1], verts[3 * (int64_t)vi + 2]};
    float vx, vy, vz;
    project_point(V, X, vx, vy, vz, v[c][0], v[c][1]);
    v[c][2] = vz;
  }
}

// World mode (one mesh shared by N views, rec = n*F + f): project, write the record,
// count tile overlaps through an LDS histogram, flush one global atomic per touched tile.
template <bool LDS>
__global__ void __launch_bounds__(256) k_bin_count_world(SetupParams P, const float* __restrict__ verts,
                                                         const int32_t* __restrict__ faces, int64_t F,
                                                         const ViewRec* __restrict__ views) {
  extern __shared__ __attribute__((aligned(16))) int hist[];
  const int n = blockIdx.y;
  if (LDS) {
    for (int i = threadIdx.x; i < P.T; i += blockDim.x) hist[i] = 0;
    __syncthreads();
  }
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f < F) {
    const ViewRec V = views[n];
    float v[3][3];
    world_face_verts(verts, faces, f, V, v);
    const FaceRec r = make_rec(P, (uint32_t)f, v);
    P.recs[(int64_t)n * F + f] = r;
    int tx0, tx1, ty0, ty1;
    if (rec_tiles(P, r, tx0, tx1, ty0, ty1))
      for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) {
          const int t = ty * P.TX + tx;
          if (LDS) atomicAdd(&hist[t], 1);
          else atomicAdd(&P.cnt[(int64_t)n * P.T + t], 1);
        }
  }
  if (LDS) {
    __syncthreads();
    for (int i = threadIdx.x; i < P.T; i += blockDim.x)
      if (hist[i]) atomicAdd(&P.cnt[(int64_t)n * P.T + i], hist[i]);
  }
}

template <bool LDS>
__global__ void __launch_bounds__(256) k_bin_fill_world(SetupParams P, int64_t F) {
  extern __shared__ __attribute__((aligned(16))) int hist[];
  const int n = blockIdx.y;
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  FaceRec r;
  int tx0 = 0, tx1 = -1, ty0 = 0, ty1 = -1;
  bool ok = false;
  if (f < F) {
    r = P.recs[(int64_t)n * F + f];
    ok = rec_tiles(P, r, tx0, tx1, ty0, ty1);
  }
  const int rid = (int)((int64_t)n * F + f);
  if (LDS) {
    for (int i = threadIdx.x; i < P.T; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    if (ok)
      for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) atomicAdd(&hist[ty * P.TX + tx], 1);
    __syncthreads();
    const int vb = P.vbase[n];
    for (int i = threadIdx.x; i < P.T; i += blockDim.x)
      if (hist[i]) hist[i] = vb + atomicAdd(&P.cur[(int64_t)n * P.T + i], hist[i]);  // reserve a block
    __syncthreads();
    if (ok)
      for (int ty = ty0; ty <= ty1; ++ty)
        for (int tx = tx0; tx <= tx1; ++tx) {
          const int pos = atomicAdd(&hist[ty * P.TX + tx], 1);
          if (pos < P.list_cap) P.list[pos] = rid;
        }
  } else if (ok) {
    for (int ty = ty0; ty <= ty1; ++ty)
      for (int tx = tx0; tx <= tx1; ++tx) {
        const int pos = P.vbase[n] + atomicAdd(&P.cur[(int64_t)n * P.T + ty * P.TX + tx], 1);
        if (pos < P.list_cap) P.list[pos] = rid;
      }
  }
}

MR_DEV int mesh_of_face(const int64_t* __restrict__ first, int64_t N, int64_t f) {
  int64_t lo = 0, hi = N - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (first[mid] <= f) lo = mid;
    else hi = mid - 1;
  }
  return (int)lo;
}

// face_verts mode (PyTorch3D _C boundary): rec = packed face id; global atomics.
__global__ void __launch_bounds__(256) k_bin_count_fv(SetupParams P, const float* __restrict__ fv, int64_t Ftot,
                                                      const int64_t* __restrict__ first, int64_t N) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= Ftot) return;
  const int n = mesh_of_face(first, N, f);
  float v[3][3];
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 3; ++k) v[c][k] = fv[9 * f + 3 * c + k];
  const FaceRec r = make_rec(P, (uint32_t)f, v);
  P.recs[f] = r;
  int tx0, tx1, ty0, ty1;
  if (rec_tiles(P, r, tx0, tx1, ty0, ty1))
    for (int ty = ty0; ty <= ty1; ++ty)
      for (int tx = tx0; tx <= tx1; ++tx) atomicAdd(&P.cnt[(int64_t)n * P.T + ty * P.TX + tx], 1);
}

__global__ void __launch_bounds__(256) k_bin_fill_fv(SetupParams P, int64_t Ftot, const int64_t* __restrict__ first,
                                                     int64_t N) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= Ftot) return;
  const int n = mesh_of_face(first, N, f);
  const FaceRec r = P.recs[f];
  int tx0, tx1, ty0, ty1;
  if (rec_tiles(P, r, tx0, tx1, ty0, ty1))
    for (int ty = ty0; ty <= ty1; ++ty)
      for (int tx = tx0; tx <= tx1; ++tx) {
        const int pos = P.vbase[n] + atomicAdd(&P.cur[(int64_t)n * P.T + ty * P.TX + tx], 1);
        if (pos < P.list_cap) P.list[pos] = (int)f;
      }
}

// Per-view exclusive scan of the T tile counts (one 1024-thread workgroup per view):
// start[n*T+t] = cur[n*T+t] = offset inside view n's region; vtot[n] = entries of view n.
__global__ void __launch_bounds__(1024) k_bin_scan_views(const int* __restrict__ cnt, int T, int* __restrict__ start,
                                                         int* __restrict__ cur, int* __restrict__ vtot, int TX,
                                                         int GX, int S, int64_t NS, int* __restrict__ scount,
                                                         int* __restrict__ work, int* __restrict__ wctr) {
  __shared__ int part[1024];
  const int n = blockIdx.x;
  const int per = (T + 1023) / 1024;
  const int b0 = threadIdx.x * per;
  const int* c = cnt + (int64_t)n * T;
  int loc[16];
  int s = 0;
  if (per <= 16) {
    for (int i = 0; i < per; ++i) {
      loc[i] = b0 + i < T ? c[b0 + i] : 0;
      s += loc[i];
    }
  } else {
    for (int i = b0; i < b0 + per && i < T; ++i) s += c[i];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
    const int v = threadIdx.x >= o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int run = part[threadIdx.x] - s;
  for (int i = 0; i < per; ++i) {
    const int t = b0 + i;
    if (t >= T) break;
    start[(int64_t)n * T + t] = run;
    cur[(int64_t)n * T + t] = run;
    run += per <= 16 ? loc[i] : c[t];
  }
  if (threadIdx.x == 1023) vtot[n] = part[1023];
  // Strip table: entries per 64x8 strip; non-empty strips go to one of three work buckets
  // by size, so the persistent raster takes the heaviest strips first (shorter tail).
  for (int sidx = threadIdx.x; sidx < S; sidx += 1024) {
    const int ty = sidx / GX, gx = sidx - ty * GX;
    int e = 0;
    for (int k = 0; k < 8; ++k) {
      const int tx = gx * 8 + k;
      if (tx < TX) e += c[ty * TX + tx];
    }
    scount[(int64_t)n * S + sidx] = e;
    if (e > 0) {
      const int b = e >= 384 ? 0 : e >= 96 ? 1 : 2;
      work[(int64_t)b * NS + atomicAdd(&wctr[b], 1)] = n * S + sidx;
    }
  }
}

// vbase = exclusive prefix of per-view totals (saturating at INT_MAX: tiles beyond the
// list capacity take the exact overflow path).
__global__ void __launch_bounds__(64) k_bin_scan_base(const int* __restrict__ vtot, int N, int* __restrict__ vbase) {
  if (threadIdx.x != 0) return;
  long long run = 0;
  for (int n = 0; n < N; ++n) {
    vbase[n] = (int)(run < 0x7fffffffll ? run : 0x7fffffffll);
    run += vtot[n];
  }
  vbase[N] = (int)(run < 0x7fffffffll ? run : 0x7fffffffll);
}

// ---------------------------------------------------------------------------
// 2. raster (+ fused shading): one wave per 8x8 tile
// ---------------------------------------------------------------------------
struct RasterParams {
  int N, H, W, TX, TY, T;
  int64_t list_cap;
  float blur, bbox_pad;
  int persp, clipb;
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
  int* pcnt;
  int* plist;
};

// Exact per-(pixel, face) decision and depth: eval_face's return value and pz, without
// the point-triangle distance unless blur > 0 and the pixel is outside. On the fast path
// (blur == 0, FR_FAST) the edge signs reject before any division: a pixel whose edge
// functions do not all carry the area's strict sign has some w_i <= 0, hence c_i <= 0
// (all z > 0), hence is not inside, hence eval_face rejects it too.
MR_DEV bool frag_keep(const FaceRec& r, float x, float y, float pad, float blur, bool persp, bool clipb,
                      bool fast, float& pz) {
  if (x > r.xmax + pad || x < r.xmin - pad || y > r.ymax + pad || y < r.ymin - pad) return false;
  const float e0 = edge_fn(x, y, r.x1, r.y1, r.x2, r.y2);
  const float e1 = edge_fn(x, y, r.x2, r.y2, r.x0, r.y0);
  const float e2 = edge_fn(x, y, r.x0, r.y0, r.x1, r.y1);
  if (fast) {
    const bool inp = (e0 > 0.0f) & (e1 > 0.0f) & (e2 > 0.0f);
    const bool inn = (e0 < 0.0f) & (e1 < 0.0f) & (e2 < 0.0f);
    if (!(r.area > 0.0f ? inp : inn)) return false;
  }
  const float w0 = e0 / r.area, w1 = e1 / r.area, w2 = e2 / r.area;
  float c0, c1, c2, b0, b1, b2;
  if (persp) persp_fwd(w0, w1, w2, r.z0, r.z1, r.z2, c0, c1, c2);
  else { c0 = w0; c1 = w1; c2 = w2; }
  if (clipb) clip_fwd(c0, c1, c2, b0, b1, b2);
  else { b0 = c0; b1 = c1; b2 = c2; }
  pz = b0 * r.z0 + b1 * r.z1 + b2 * r.z2;
  if (pz < 0.0f) return false;
  const bool inside = c0 > 0.0f && c1 > 0.0f && c2 > 0.0f;
  if (!inside) {
    if (!(blur > 0.0f)) return false;
    if (pt_tri_dist(x, y, r) >= blur) return false;
  }
  return true;
}

#define MR_WGT 8                    // tiles (= waves) per workgroup
#define MR_SPX (MR_WGT * MR_TS * MR_TS)  // 512 pixels per strip
#define MR_NONE 0x7fffffff          // "no face" sentinel, larger than any face id

// (z, face) packed so that unsigned order == frag_less order on the depths that are ever
// kept (pz >= 0; -0 folds onto +0, which the CPU compares equal). The empty key sorts
// after every kept fragment, +inf depth included.
#define MR_KEY_EMPTY ((0x7f800000ull << 32) | (unsigned long long)MR_NONE)
MR_DEV unsigned long long frag_key(float z, int f) {
  const unsigned zb = z == 0.0f ? 0u : __float_as_uint(z);
  return ((unsigned long long)zb << 32) | (unsigned)f;
}

// Wave-wide inclusive scans on DPP: row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 carry row totals across rows (GFX9 DPP).
MR_DEV int wave_incl_sum(int v) {
#ifdef MR_DBG_SHFL
  for (int o = 1; o < 64; o <<= 1) { const int u = __shfl_up(v, o, 64); if ((threadIdx.x & 63) >= o) v += u; }
  return v;
#endif
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}
MR_DEV int wave_incl_max(int v) {
#ifdef MR_DBG_SHFL
  for (int o = 1; o < 64; o <<= 1) { const int u = __shfl_up(v, o, 64); if ((threadIdx.x & 63) >= o) v = max(v, u); }
  return v;
#endif
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xa, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xc, 0xf, false));
  return v;
}

// Wave-local LDS hand-off (the 64 lanes of one wave write, then every lane reads).
MR_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// ---- output staging for the 64x8-pixel strip of one raster workgroup ----
// Rows padded to 72 entries so the 8 rows one wave's tile touches land in different banks.
#define MR_SROW 72
#define MR_SSZ (MR_TS * MR_SROW)
MR_DEV int strip_slot(int row, int col) { return row * MR_SROW + col; }

struct StageOut {  // 18 KB, union over the two modes
  union {
    struct { float depth[MR_SSZ], sil[MR_SSZ], rgb[MR_SSZ * 4]; int p2f[MR_SSZ]; } m1;
    struct { long long p2f[MR_SSZ]; float zbuf[MR_SSZ], bary[MR_SSZ * 3], dists[MR_SSZ]; } m0;
  };
};

// One wave's batch of up to 64 (tile, face) entries, expanded into (face, pixel) pairs.
struct PairStage {
  FaceRec rec[64];
  int id[64];
  int meta[64];  // first pair index | (rect width - 1) << 13 | strip col << 16 | strip row << 22
  int mark[64];  // pass-local: pair slot -> entry lane that starts there
};

struct RasterSmem {
  union {
    PairStage ps[MR_WGT];  // 39 KB, face loop only
    StageOut out;          // epilogue only
  };
  unsigned long long key[MR_SPX];  // per-pixel (z, face) minimum
  float xs[64], ys[MR_TS];         // pixel-centre NDC of the strip's columns / rows
};

template <int MODE>
MR_DEV void stage_pixel(const RasterParams& P, StageOut& O, int n, int sp, bool hit, int f, const FaceRec& r,
                        const FragEval& e) {
  if (MODE == 0) {
    O.m0.p2f[sp] = hit ? (long long)f : -1ll;
    O.m0.zbuf[sp] = hit ? e.pz : -1.0f;
    O.m0.bary[3 * sp + 0] = hit ? e.b0 : -1.0f;
    O.m0.bary[3 * sp + 1] = hit ? e.b1 : -1.0f;
    O.m0.bary[3 * sp + 2] = hit ? e.b2 : -1.0f;
    O.m0.dists[sp] = hit ? e.sdist : -1.0f;
  } else {
    PixGeom G;
    ShadeOut o;
    ShadeCache C;
    if (hit) gather_geom(P.S, r.face, G);
    shade_fwd(P.S, n, hit, G, hit ? e.b0 : 0.f, hit ? e.b1 : 0.f, hit ? e.b2 : 0.f, hit ? e.pz : 0.f,
              hit ? e.sdist : 0.f, o, C);
    O.m1.depth[sp] = o.depth;
    O.m1.sil[sp] = o.sil;
    O.m1.rgb[4 * sp + 0] = o.rgb[0];
    O.m1.rgb[4 * sp + 1] = o.rgb[1];
    O.m1.rgb[4 * sp + 2] = o.rgb[2];
    O.m1.rgb[4 * sp + 3] = o.alpha;
    O.m1.p2f[sp] = hit ? f : -1;
  }
}

// Coalesced strip write: thread t owns strip row t/64, column t%64 (one wave = one 256-B row);
// multi-channel rows (bary, rgb) go out as flat float streams, 64 consecutive floats per
// wave instruction. With O == nullptr the strip is empty and the background is written
// straight from registers (no LDS round trip).
template <int MODE, int CH>
MR_DEV void write_strip(const RasterParams& P, const StageOut* O, int n, int x0, int y0) {
  const int t = threadIdx.x;
  const int row = t >> 6, col = t & 63;
  const int px = x0 + col, py = y0 + row;
  const int sp = strip_slot(row, col);
  float bgv[4] = {-1.0f, -1.0f, -1.0f, -1.0f}, bgd = -1.0f, bgs = -1.0f;
  if (MODE == 1 && !O) {
    PixGeom G;
    ShadeOut o;
    ShadeCache C;
    shade_fwd(P.S, n, false, G, 0.f, 0.f, 0.f, 0.f, 0.f, o, C);
    bgd = o.depth;
    bgs = o.sil;
    bgv[0] = o.rgb[0]; bgv[1] = o.rgb[1]; bgv[2] = o.rgb[2]; bgv[3] = o.alpha;
  }
  if (px < P.W && py < P.H) {
    const int64_t pix = ((int64_t)n * P.H + py) * P.W + px;
    if (MODE == 0) {
      P.p2f[pix] = O ? O->m0.p2f[sp] : -1ll;
      P.zbuf[pix] = O ? O->m0.zbuf[sp] : -1.0f;
      P.dists[pix] = O ? O->m0.dists[sp] : -1.0f;
    } else {
      if (P.out_flags & MR_OUT_DEPTH) P.depth[pix] = O ? O->m1.depth[sp] : bgd;
      if (P.out_flags & MR_OUT_SIL) P.sil[pix] = O ? O->m1.sil[sp] : bgs;
      P.p2f32[pix] = O ? O->m1.p2f[sp] : -1;
    }
  }
  constexpr int ch = CH;  // compile-time channel count: the flat-stream index math is shifts/multiplies
  if (MODE == 1 && !(P.out_flags & MR_OUT_RGB)) return;
  const int rowlen = 64 * ch;
  const int ncols = (P.W - x0) < 64 ? (P.W - x0) : 64;
  for (int j = t; j < MR_TS * rowlen; j += MR_SPX) {
    const int rr = j / rowlen, q = j - rr * rowlen;
    const int cc = q / ch, k = q - cc * ch;
    const int yy = y0 + rr;
    if (cc >= ncols || yy >= P.H) continue;
    const int64_t base = ((int64_t)n * P.H + yy) * P.W + x0;
    const int s = strip_slot(rr, cc);
    if (MODE == 0) P.bary[base * 3 + q] = O ? O->m0.bary[3 * s + k] : -1.0f;
    else P.rgb[base * ch + q] = O ? O->m1.rgb[4 * s + k] : (k == 0 ? bgv[0] : k == 1 ? bgv[1] : k == 2 ? bgv[2] : bgv[3]);
  }
}

// Optional phase timestamps (build with -DMR_PROF; tools/raster_phases.py): per wave 16 slots,
// s_memtime at phase boundaries, s_memrealtime at start/end, entry/pass counts.
#ifdef MR_PROF
__device__ unsigned long long* g_prof = nullptr;
#define PROF_AT(i, v)                                                                                 \
  do {                                                                                                \
    if (g_prof && lane == 0)                                                                          \
      g_prof[((size_t)prof_slot * MR_WGT + wave) * 16 + (i)] = (v);                                 \
  } while (0)
#define PROF_T(i) PROF_AT(i, __builtin_amdgcn_s_memtime())
#else
#define PROF_AT(i, v) do {} while (0)
#define PROF_T(i) do {} while (0)
#endif

// One 512-thread workgroup = 8 waves rasterizes one 64x8-pixel strip (8 tiles of 8x8):
//  (1) the strip's 8 tile lists are concatenated and dealt to the waves 64 entries at a
//      time, one per lane; each lane clips its face's pixel bbox to its tile (<= 64 pixels);
//  (2) a wave prefix sum over the rectangle sizes numbers the (face, pixel) pairs, and
//      64 pairs per pass are evaluated exactly (frag_keep), one per lane — so a ~3-pixel
//      face costs ~3 lanes, not a whole wave;
//  (3) kept fragments meet in a per-pixel LDS atomicMin on the packed (z, face) key, which
//      is order-independent and equals the CPU's "strictly nearer, earlier face wins";
//  (4) wave k finalises tile k (exact recompute + shading) and the strip is written row-wise.
template <int MODE, int CH>
__device__ __attribute__((noinline)) void raster_strip(const RasterParams& P, RasterSmem& sm, const FaceRec* __restrict__ recs,
                         const int* __restrict__ list, const int* __restrict__ cnt, const int* __restrict__ start,
                         const int* __restrict__ vbase, int n, int gx, int ty, int prof_slot) {
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  PROF_AT(8, __builtin_amdgcn_s_memrealtime());
  PROF_T(0);
  const int H = P.H, W = P.W;
  const int x0 = gx * MR_WGT * MR_TS, y0 = ty * MR_TS;
  const int64_t vb = vbase[n];
  const int64_t vfirst = P.view_first ? P.view_first[n] : (int64_t)n * P.F;
  const int64_t vcount = P.view_first ? P.view_count[n] : P.F;

  // lanes 0..7 <-> tiles 0..7 of the strip: entry count, list start, overflow flag
  int tc = 0, ts = 0, tovf = 0;
  {
    const int txl = gx * MR_WGT + lane;
    if (lane < MR_WGT && txl < P.TX) {
      const int64_t bt = (int64_t)n * P.T + (int64_t)ty * P.TX + txl;
      const int c = cnt[bt];
      ts = start[bt];
      // overflowed list: the tile's entries are every face of the view (bbox-filtered below);
      // counts are exact, so an empty tile stays empty
      if (c > 0 && vb + ts + c > P.list_cap) {
        tovf = 1;
        tc = (int)(vcount < 0x7fffffffll ? vcount : 0x7fffffffll);
      } else {
        tc = c;
      }
    }
  }
  const int tincl = wave_incl_sum(tc);
  const int E = __builtin_amdgcn_readlane(tincl, MR_WGT - 1);
  PROF_T(1);
  if (E == 0) {  // uniform over the workgroup (work lists only hold non-empty strips)
    write_strip<MODE, CH>(P, nullptr, n, x0, y0);
    return;
  }
  const int texcl = tincl - tc;

  if (t < 64) sm.xs[t] = col_ndc(x0 + t < W ? x0 + t : W - 1, H, W);
  else if (t < 64 + MR_TS) sm.ys[t - 64] = row_ndc(y0 + t - 64 < H ? y0 + t - 64 : H - 1, H, W);
  sm.key[t] = MR_KEY_EMPTY;
  PairStage& S = sm.ps[wave];
  S.mark[lane] = -1;
  __syncthreads();
  PROF_T(2);
#ifdef MR_PROF
  int prof_passes = 0;
#endif

  const float pad = P.bbox_pad, blur = P.blur;
  const bool persp = P.persp != 0, clipb = P.clipb != 0;
#ifdef MR_DBG_NOFAST
  const bool fast_ok = false;
#else
  const bool fast_ok = !(blur > 0.0f);
#endif
#pragma unroll 1
  for (int eb = 0; eb < E; eb += MR_WGT * 64) {
    // (1) one entry per lane, interleaved over the 8 waves so every wave gets ~E/8 of them
    const int e = eb + lane * MR_WGT + wave;
    int k = 0;
#pragma unroll
    for (int kk = 1; kk < MR_WGT; ++kk) k += e >= __builtin_amdgcn_readlane(texcl, kk) ? 1 : 0;
    // cross-lane reads at full EXEC (ds_bpermute from an inactive lane is undefined)
    const int kex = __shfl(texcl, k, 64);
    const int kst = __shfl(ts, k, 64);
    const int kovf = __shfl(tovf, k, 64);
    int np = 0, meta = 0;
    if (e < E) {
      const int i = e - kex;
      const int id = kovf ? (int)(vfirst + i) : list[vb + kst + i];
      const FaceRec r = recs[id];
      int cx0, cx1, cy0, cy1;
      ndc_range_to_pix(r.xmin - pad, r.xmax + pad, W, H, cx0, cx1);
      ndc_range_to_pix(r.ymin - pad, r.ymax + pad, H, W, cy0, cy1);
      const int tx0 = x0 + k * MR_TS;
      cx0 = cx0 > tx0 ? cx0 : tx0;
      cx1 = cx1 < tx0 + MR_TS - 1 ? cx1 : tx0 + MR_TS - 1;
      cy0 = cy0 > y0 ? cy0 : y0;
      cy1 = cy1 < y0 + MR_TS - 1 ? cy1 : y0 + MR_TS - 1;
      if ((r.flags & FR_VALID) && cx0 <= cx1 && cy0 <= cy1) {
        const int w = cx1 - cx0 + 1;
        np = w * (cy1 - cy0 + 1);
        meta = ((w - 1) << 13) | ((cx0 - x0) << 16) | ((cy0 - y0) << 22);
      }
      S.rec[lane] = r;
      S.id[lane] = id;
    }
    // (2) pair numbering
    const int pincl = wave_incl_sum(np);
    const int pexcl = pincl - np;
    const int NP = __builtin_amdgcn_readlane(pincl, 63);
    S.meta[lane] = meta | pexcl;
#pragma unroll 1
    for (int pb = 0; pb < NP; pb += 64) {
#ifdef MR_PROF
      ++prof_passes;
#endif
      wave_lds_sync();
      // entry starting inside this pass marks its first slot; slot 0 belongs to the entry
      // straddling pb (the last non-empty entry starting at or before it)
      if (np > 0 && pexcl > pb && pexcl < pb + 64) S.mark[pexcl - pb] = lane;
      const unsigned long long own = __ballot(np > 0 && pexcl <= pb);
      const int straddle = 63 - __builtin_clzll(own);
      wave_lds_sync();
      int m = S.mark[lane];
      S.mark[lane] = -1;
      if (lane == 0) m = straddle;
      m = wave_incl_max(m);
      const int q = pb + lane;
      if (q < NP) {
        // (3) one (face, pixel) pair per lane
        const int mt = S.meta[m];
        const int loc = q - (mt & 0x1fff);
        const int w = ((mt >> 13) & 7) + 1;
#ifdef MR_DBG_IDIV
        const int ly = loc / w;
#else
        const int ly = (int)((float)loc * __builtin_amdgcn_rcpf((float)w) + 1e-3f);
#endif
        const int lx = loc - ly * w;
        const int sx = ((mt >> 16) & 63) + lx, sy = ((mt >> 22) & 7) + ly;
        const FaceRec r = S.rec[m];
        float pz;
        if (frag_keep(r, sm.xs[sx], sm.ys[sy], pad, blur, persp, clipb, fast_ok && (r.flags & FR_FAST), pz))
          atomicMin(&sm.key[sy * 64 + sx], frag_key(pz, S.id[m]));
      }
    }
    wave_lds_sync();  // the stage is rewritten by the next batch
  }
  PROF_T(3);
  __syncthreads();
  PROF_T(4);

  // (4) wave k finalises tile k of the strip
  const int ly = lane >> 3, lx = wave * MR_TS + (lane & 7);
  const int px = x0 + lx, py = y0 + ly;
  const unsigned long long key = sm.key[ly * 64 + lx];
  const int f = (int)(unsigned)(key & 0xffffffffull);
  FragEval ev;
  FaceRec r;
  bool hit = f != MR_NONE && px < W && py < H;
  if (hit) {
    r = recs[f];
    hit = eval_face(r, sm.xs[lx], sm.ys[ly], P.bbox_pad, P.blur, P.persp, P.clipb, ev);
  }
  stage_pixel<MODE>(P, sm.out, n, strip_slot(ly, lx), hit, f, r, ev);
  if (MODE == 1) {  // compact list of covered pixels for the backward (one atomic per wave)
    const unsigned long long msk = __ballot(hit);
    if (msk) {
      int base = 0;
      if (lane == 0) base = atomicAdd(&P.pcnt[n], __popcll(msk));
      base = __shfl(base, 0, 64);
      if (hit) {
        const int rank = __popcll(msk & ((1ull << lane) - 1ull));
        P.plist[(int64_t)n * H * W + base + rank] = py * W + px;
      }
    }
  }
  PROF_T(5);
  __syncthreads();
  write_strip<MODE, CH>(P, &sm.out, n, x0, y0);
  PROF_T(6);
  PROF_AT(9, __builtin_amdgcn_s_memrealtime());
#ifdef MR_PROF
  PROF_AT(7, ((unsigned long long)E << 32) | (unsigned)prof_passes);
#endif
}

// Persistent raster: a grid sized to the resident capacity (CUs x workgroups per CU) pulls
// non-empty strips from the three work buckets (heaviest first) through one atomic counter;
// background strips never reach this kernel (k_bg writes them). Every workgroup leaves
// when the counter passes the total, so the grid always drains.
template <int MODE, int CH>
__global__ void __launch_bounds__(512, 6) k_raster(RasterParams P, const FaceRec* __restrict__ recs,
                                                const int* __restrict__ list, const int* __restrict__ cnt,
                                                const int* __restrict__ start, const int* __restrict__ vbase,
                                                const int* __restrict__ work, int* __restrict__ wctr, int64_t NS,
                                                int S, int GX) {
  __shared__ RasterSmem sm;
  __shared__ int s_item;
  const int c0 = wctr[0], c1 = wctr[1], c2 = wctr[2];
  const int total = c0 + c1 + c2;
  for (;;) {
    if (threadIdx.x == 0) s_item = atomicAdd(&wctr[3], 1);
    __syncthreads();  // also orders the previous strip's LDS reads before this strip's writes
    const int item = s_item;
    if (item >= total) break;
    const int sid = item < c0 ? work[item] : item < c0 + c1 ? work[NS + (item - c0)] : work[2 * NS + (item - c0 - c1)];
    const int n = sid / S, r = sid - n * S;
    const int ty = r / GX, gx = r - ty * GX;
    raster_strip<MODE, CH>(P, sm, recs, list, cnt, start, vbase, n, gx, ty, sid);
  }
}

// Background for every strip without entries: streaming vector stores, one workgroup per
// strip row (8 image rows) of one view; strips holding faces are skipped (k_raster writes them).
template <int MODE, int CH>
__global__ void __launch_bounds__(256) k_bg(RasterParams P, const int* __restrict__ scount, int S, int GX) {
  const int n = blockIdx.y, ty = blockIdx.x;
  float bgd = -1.0f, bgs = -1.0f, bgv[4] = {-1.0f, -1.0f, -1.0f, -1.0f};
  if (MODE == 1) {
    PixGeom G;
    ShadeOut o;
    ShadeCache C;
    shade_fwd(P.S, n, false, G, 0.f, 0.f, 0.f, 0.f, 0.f, o, C);
    bgd = o.depth;
    bgs = o.sil;
    bgv[0] = o.rgb[0]; bgv[1] = o.rgb[1]; bgv[2] = o.rgb[2]; bgv[3] = o.alpha;
  }
  const int* sc = scount + (int64_t)n * S + (int64_t)ty * GX;
  const int W = P.W, H = P.H;
  const bool vec = (W & 3) == 0;
  const int W4 = (W + 3) >> 2;
  const bool rgb = MODE == 1 && (P.out_flags & MR_OUT_RGB);
  for (int rr = threadIdx.x >> 7; rr < MR_TS; rr += 2) {
    const int y = ty * MR_TS + rr;
    if (y >= H) break;
    for (int x4 = threadIdx.x & 127; x4 < W4; x4 += 128) {
      if (sc[x4 >> 4] != 0) continue;  // 16 groups of 4 pixels per 64-pixel strip
      const int x = x4 * 4;
      const int64_t pix = ((int64_t)n * H + y) * W + x;
      if (vec) {
        if (MODE == 0) {
          longlong2* q = (longlong2*)(P.p2f + pix);
          q[0] = make_longlong2(-1ll, -1ll);
          q[1] = make_longlong2(-1ll, -1ll);
          const float4 m1 = make_float4(-1.f, -1.f, -1.f, -1.f);
          *(float4*)(P.zbuf + pix) = m1;
          *(float4*)(P.dists + pix) = m1;
          float4* b = (float4*)(P.bary + pix * 3);
          b[0] = m1; b[1] = m1; b[2] = m1;
        } else {
          if (P.out_flags & MR_OUT_DEPTH) *(float4*)(P.depth + pix) = make_float4(bgd, bgd, bgd, bgd);
          if (P.out_flags & MR_OUT_SIL) *(float4*)(P.sil + pix) = make_float4(bgs, bgs, bgs, bgs);
          *(int4*)(P.p2f32 + pix) = make_int4(-1, -1, -1, -1);
          if (rgb) {
            float4* c = (float4*)(P.rgb + pix * CH);
            if (CH == 4) {
              const float4 v = make_float4(bgv[0], bgv[1], bgv[2], bgv[3]);
              c[0] = v; c[1] = v; c[2] = v; c[3] = v;
            } else {
              c[0] = make_float4(bgv[0], bgv[1], bgv[2], bgv[0]);
              c[1] = make_float4(bgv[1], bgv[2], bgv[0], bgv[1]);
              c[2] = make_float4(bgv[2], bgv[0], bgv[1], bgv[2]);
            }
          }
        }
      } else {
        for (int k = 0; k < 4 && x + k < W; ++k) {
          const int64_t q = pix + k;
          if (MODE == 0) {
            P.p2f[q] = -1ll;
            P.zbuf[q] = -1.0f;
            P.dists[q] = -1.0f;
            for (int c = 0; c < 3; ++c) P.bary[q * 3 + c] = -1.0f;
          } else {
            if (P.out_flags & MR_OUT_DEPTH) P.depth[q] = bgd;
            if (P.out_flags & MR_OUT_SIL) P.sil[q] = bgs;
            P.p2f32[q] = -1;
            if (rgb)
              for (int c = 0; c < CH; ++c) P.rgb[q * CH + c] = bgv[c];
          }
        }
      }
    }
  }
}

// Resident workgroups of k_raster<MODE,CH> on the current device (persistent grid size).
template <int MODE, int CH>
static int raster_grid(int64_t strips_total) {
  static int cached = 0;
  if (!cached) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_raster<MODE, CH>, 512, 0) != hipSuccess || per <= 0)
      per = 2;
    cached = cus * per;
  }
  return (int)(strips_total < cached ? (strips_total > 0 ? strips_total : 1) : cached);
}

template <int MODE, int CH>
static int launch_raster(const RasterParams& P, const RasterWS& w, const BinGeom& g, int64_t N, int kid,
                         hipStream_t st) {
  dim3 bgrid((unsigned)g.TY, (unsigned)N);
  MR_TIMED(KID_BG, st, (k_bg<MODE, CH><<<bgrid, 256, 0, st>>>(P, w.scount, g.S, g.GX)));
  MR_CHECK_LAUNCH("k_bg");
  const int grid = raster_grid<MODE, CH>(N * g.S);
  MR_TIMED(kid, st, (k_raster<MODE, CH><<<grid, 512, 0, st>>>(P, w.recs, w.list, w.cnt, w.start, w.vbase, w.work,
                                                                w.wctr, N * g.S, g.S, g.GX)));
  MR_CHECK_LAUNCH("k_raster");
  return MR_OK;
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
  int N, H, W, NBX;
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
  const int n = blockIdx.y, bt = blockIdx.x;
  const int btx = bt % P.NBX, bty = bt / P.NBX;
  const int px = btx * MR_BT + (threadIdx.x & 31);
  for (int k = 0; k < 4; ++k) {
    const int py = bty * MR_BT + (threadIdx.x >> 5) + 8 * k;
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

// Fused render backward over the compact per-view list of covered pixels written by
// k_raster<1>: workgroup (b, n) handles entries [1024 b, 1024 b + 1024) of view n.
struct RenderBwdParams {
  int N, H, W, NB;
  float blur, bbox_pad;
  int persp, clipb;
  const FaceRec* recs;
  const int32_t* p2f32;
  const int* pcnt;
  const int* plist;
  const float* gD;
  const float* gS;
  const float* gRGB;
  int rgb_ch;
  ShadeParams S;
  const ViewRec* views;
  float* gface;   // (F, ACC)
  float* rt_part; // (N*NB, 12)
};

template <int ACC>
__global__ void __launch_bounds__(256) k_render_bwd(RenderBwdParams P) {
  __shared__ LdsAcc<ACC> L;
  __shared__ float red[4][12];
  const int n = blockIdx.y;
  const int cntp = P.pcnt[n];
  float gR[9], gT[3];
  for (int i = 0; i < 9; ++i) gR[i] = 0.0f;
  for (int i = 0; i < 3; ++i) gT[i] = 0.0f;
  if ((int64_t)blockIdx.x * 256 >= cntp) {  // uniform over the workgroup: nothing to do
    if (threadIdx.x < 12) P.rt_part[((int64_t)n * P.NB + blockIdx.x) * 12 + threadIdx.x] = 0.0f;
    return;
  }
  acc_init(L);
  __syncthreads();
  const ViewRec V = P.views[n];
  const int64_t HW = (int64_t)P.H * P.W;
  // grid-stride over 256-pixel chunks of view n's compact covered-pixel list (one pixel per thread)
  for (int64_t c0 = (int64_t)blockIdx.x * 256; c0 < cntp; c0 += (int64_t)gridDim.x * 256) {
    {
      const int64_t idx = c0 + threadIdx.x;
      if (idx >= cntp) continue;
      const int q = P.plist[n * HW + idx];
      const int px = q % P.W, py = q / P.W;
      const int64_t pix = n * HW + q;
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
        const float* g = P.gRGB + pix * P.rgb_ch;
        gC[0] = g[0];
        gC[1] = g[1];
        gC[2] = g[2];
        if (P.rgb_ch == 4) gA = g[3];
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
    P.rt_part[((int64_t)n * P.NB + blockIdx.x) * 12 + i] = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
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

#ifdef MR_PROF
// Debug-only (MR_PROF builds): device buffer of N*strips*8*16 u64 for k_raster phase stamps.
int32_t mr_debug_set_prof(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_prof), &buf, sizeof(buf)) == hipSuccess ? MR_OK : MR_ELAUNCH;
}
#endif
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
  const int64_t Ftot = total_faces > 0 ? total_faces : 1;
  BinGeom g = bin_geom(H, W, num_meshes, Ftot, max_faces_per_bin);
  return carve_raster_ws(nullptr, num_meshes, Ftot, H, W, g, false).bytes;
}

static SetupParams make_setup(const mr_raster_settings_t* s, const BinGeom& g, const RasterWS& w) {
  SetupParams P;
  P.H = s->H; P.W = s->W; P.TX = g.TX; P.TY = g.TY; P.T = g.T;
  P.bbox_pad = sqrtf(s->blur_radius);
  P.persp = s->perspective_correct;
  P.cull = s->cull_backfaces;
  P.list_cap = g.list_cap;
  P.recs = w.recs;
  P.cnt = w.cnt;
  P.cur = w.cur;
  P.list = w.list;
  P.vbase = w.vbase;
  return P;
}

static RasterParams make_raster(const mr_raster_settings_t* s, const BinGeom& g, int64_t N) {
  RasterParams P;
  memset(&P, 0, sizeof(P));
  P.N = (int)N; P.H = s->H; P.W = s->W;
  P.TX = g.TX; P.TY = g.TY; P.T = g.T;
  P.list_cap = g.list_cap;
  P.blur = s->blur_radius;
  P.bbox_pad = sqrtf(s->blur_radius);
  P.persp = s->perspective_correct;
  P.clipb = s->clip_barycentric_coords;
  return P;
}

static int launch_scan(const RasterWS& w, int64_t N, const BinGeom& g, hipStream_t st) {
  MR_TIMED(KID_BIN_SCAN, st, (k_bin_scan_views<<<(unsigned)N, 1024, 0, st>>>(w.cnt, g.T, w.start, w.cur, w.vtot, g.TX, g.GX, g.S,
                                                                   N * g.S, w.scount, w.work, w.wctr)));
  MR_CHECK_LAUNCH("k_bin_scan_views");
  MR_TIMED(KID_BIN_SCAN, st, (k_bin_scan_base<<<1, 64, 0, st>>>(w.vtot, (int)N, w.vbase)));
  MR_CHECK_LAUNCH("k_bin_scan_base");
  return MR_OK;
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
  const int64_t Fb = Ftot > 0 ? Ftot : 1;
  BinGeom g = bin_geom(s->H, s->W, N, Fb, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws(ws, N, Fb, s->H, s->W, g, false);
  if (ws_bytes < w.bytes) return set_err(MR_EWORKSPACE, "workspace too small: %zu < %zu", ws_bytes, w.bytes);
  if (hipMemsetAsync(w.cnt, 0, zero_bytes(N, g), st) != hipSuccess) return set_err(MR_ELAUNCH, "memset failed");
  SetupParams SP = make_setup(s, g, w);
  if (Ftot > 0) {
    MR_TIMED(KID_BIN_COUNT, st, (k_bin_count_fv<<<ceil_div(Ftot, 256), 256, 0, st>>>(SP, face_verts, Ftot, first, N)));
    MR_CHECK_LAUNCH("k_bin_count_fv");
  }
  if ((rc = launch_scan(w, N, g, st))) return rc;
  if (Ftot > 0) {
    MR_TIMED(KID_BIN_FILL, st, (k_bin_fill_fv<<<ceil_div(Ftot, 256), 256, 0, st>>>(SP, Ftot, first, N)));
    MR_CHECK_LAUNCH("k_bin_fill_fv");
  }
  RasterParams P = make_raster(s, g, N);
  P.view_first = first;
  P.view_count = count;
  P.p2f = p2f; P.zbuf = zbuf; P.bary = bary; P.dists = dists;
  if ((rc = launch_raster<0, 3>(P, w, g, N, KID_RASTER_FRAG, st))) return rc;
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
  RasterBwdParams P;
  P.N = (int)N; P.H = s->H; P.W = s->W; P.NBX = ceil_div(s->W, MR_BT);
  P.persp = s->perspective_correct; P.clipb = s->clip_barycentric_coords;
  P.fv = fv; P.p2f = p2f; P.gz = gz; P.gb = gb; P.gd = gd; P.gfv = gfv;
  dim3 grid(P.NBX * ceil_div(s->H, MR_BT), (unsigned)N);
  MR_TIMED(KID_RASTER_BWD, st, (k_raster_bwd<<<grid, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_raster_bwd");
  return MR_OK;
}

int32_t mr_project_faces(const float* verts, int64_t V, const int32_t* faces, int64_t F, const mr_view_t* views,
                         int64_t N, float* fv, void* stream) {
  if (N <= 0 || N > 65535 || F < 0 || V < 0) return set_err(MR_EINVAL, "bad sizes");
  if (F == 0) return MR_OK;
  if (!verts || !faces || !views || !fv) return set_err(MR_EINVAL, "NULL argument");
  dim3 grid(ceil_div(F, 256), (unsigned)N);
  MR_TIMED(KID_PROJECT, (hipStream_t)stream, (k_project_faces<<<grid, 256, 0, (hipStream_t)stream>>>(verts, faces, F, (const ViewRec*)views, fv)));
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
  MR_TIMED(KID_PROJECT_BWD, st, (k_project_faces_bwd<<<grid, 256, 0, st>>>(verts, V, F, ptr, adj, (const ViewRec*)views, gfv, gverts, gviews)));
  MR_CHECK_LAUNCH("k_project_faces_bwd");
  return MR_OK;
}

int32_t mr_vertex_normals(const float* verts, int64_t V, const int32_t* faces, int64_t F, const int32_t* ptr,
                          const int32_t* adj, float* vn, float* vraw, void* stream) {
  (void)F;
  if (V <= 0) return MR_OK;
  MR_TIMED(KID_VNORMALS, (hipStream_t)stream, (k_vertex_normals<<<ceil_div(V, 256), 256, 0, (hipStream_t)stream>>>(verts, V, faces, ptr, adj, vn, vraw)));
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
  BinGeom g = bin_geom(H, W, N, N * F, max_faces_per_bin);
  return carve_raster_ws(nullptr, N, N * F, H, W, g, true).bytes;
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
  if ((int64_t)N * s->H * s->W >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "N*H*W >= 2^31");
  if (!p2f32 || !views) return set_err(MR_EINVAL, "NULL output");
  if ((sp->out_flags & MR_OUT_DEPTH) && !depth) return set_err(MR_EINVAL, "depth output NULL");
  if ((sp->out_flags & MR_OUT_SIL) && !sil) return set_err(MR_EINVAL, "silhouette output NULL");
  if ((sp->out_flags & MR_OUT_RGB) && !rgb) return set_err(MR_EINVAL, "rgb output NULL");
  if (sp->light_kind == 0 && (!cc || (ncc != 1 && ncc != N))) return set_err(MR_EINVAL, "camera centres");
  hipStream_t st = (hipStream_t)stream;
  BinGeom g = bin_geom(s->H, s->W, N, N * m->F, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws(ws, N, N * m->F, s->H, s->W, g, true);
  if (ws_bytes < w.bytes) return set_err(MR_EWORKSPACE, "workspace too small: %zu < %zu", ws_bytes, w.bytes);
  if (hipMemsetAsync(w.cnt, 0, zero_bytes(N, g), st) != hipSuccess) return set_err(MR_ELAUNCH, "memset failed");
  SetupParams SP = make_setup(s, g, w);
  dim3 sgrid(ceil_div(m->F, 256), (unsigned)N);
  const bool lds = g.T <= MR_LDS_HIST;
  const size_t shm = lds ? sizeof(int) * (size_t)g.T : 0;
  if (lds)
    MR_TIMED(KID_BIN_COUNT, st, (k_bin_count_world<true><<<sgrid, 256, shm, st>>>(SP, m->verts, m->faces, m->F, (const ViewRec*)views)));
  else
    MR_TIMED(KID_BIN_COUNT, st, (k_bin_count_world<false><<<sgrid, 256, 0, st>>>(SP, m->verts, m->faces, m->F, (const ViewRec*)views)));
  MR_CHECK_LAUNCH("k_bin_count_world");
  if ((rc = launch_scan(w, N, g, st))) return rc;
  if (lds)
    MR_TIMED(KID_BIN_FILL, st, (k_bin_fill_world<true><<<sgrid, 256, shm, st>>>(SP, m->F)));
  else
    MR_TIMED(KID_BIN_FILL, st, (k_bin_fill_world<false><<<sgrid, 256, 0, st>>>(SP, m->F)));
  MR_CHECK_LAUNCH("k_bin_fill_world");
  RasterParams P = make_raster(s, g, N);
  P.F = m->F;
  P.S = make_shade(m, sp, cc, ncc);
  P.out_flags = sp->out_flags;
  P.rgb_ch = sp->rgb_channels;
  P.depth = depth;
  P.sil = sil;
  P.rgb = rgb;
  P.p2f32 = p2f32;
  P.pcnt = w.pcnt;
  P.plist = w.plist;
  if (P.rgb_ch == 4) rc = launch_raster<1, 4>(P, w, g, N, KID_RASTER_RENDER, st);
  else rc = launch_raster<1, 3>(P, w, g, N, KID_RASTER_RENDER, st);
  if (rc) return rc;
  return MR_OK;
}

// Backward workgroups per view: ~4096 in total, never more than the view's 256-pixel chunks.
static int bwd_blocks_per_view(int64_t N, int H, int W) {
  const int chunks = ceil_div((int64_t)H * W, 256);
  int nb = ceil_div(4096, N);
  if (nb > chunks) nb = chunks;
  return nb < 1 ? 1 : nb;
}

size_t mr_render_backward_workspace(int64_t N, int64_t V, int64_t F, int32_t H, int32_t W) {
  const int NB = bwd_blocks_per_view(N, H, W);
  size_t off = align_up(sizeof(float) * 27 * (size_t)F, 256);
  off = align_up(off + sizeof(float) * 12 * (size_t)N * NB, 256);
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
  BinGeom g = bin_geom(s->H, s->W, N, N * m->F, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws((void*)fws, N, N * m->F, s->H, s->W, g, true);
  const bool vcol = m->tex_kind == 1;
  const int ACC = vcol ? 27 : 18;
  const int NB = bwd_blocks_per_view(N, s->H, s->W);
  char* b = (char*)bws;
  float* gface = (float*)b;
  size_t off = align_up(sizeof(float) * 27 * (size_t)m->F, 256);
  float* rt_part = (float*)(b + off);
  off = align_up(off + sizeof(float) * 12 * (size_t)N * NB, 256);
  float* gnu = (float*)(b + off);
  if (hipMemsetAsync(gface, 0, sizeof(float) * ACC * (size_t)m->F, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  RenderBwdParams P;
  memset(&P, 0, sizeof(P));
  P.N = (int)N; P.H = s->H; P.W = s->W; P.NB = NB;
  P.blur = s->blur_radius; P.bbox_pad = sqrtf(s->blur_radius);
  P.persp = s->perspective_correct; P.clipb = s->clip_barycentric_coords;
  P.recs = w.recs;
  P.p2f32 = p2f32;
  P.pcnt = w.pcnt;
  P.plist = w.plist;
  P.gD = (sp->out_flags & MR_OUT_DEPTH) ? gD : nullptr;
  P.gS = (sp->out_flags & MR_OUT_SIL) ? gS : nullptr;
  P.gRGB = (sp->out_flags & MR_OUT_RGB) ? gRGB : nullptr;
  P.rgb_ch = sp->rgb_channels;
  P.S = make_shade(m, sp, cc, ncc);
  P.views = (const ViewRec*)views;
  P.gface = gface;
  P.rt_part = rt_part;
  dim3 grid(NB, (unsigned)N);
  if (vcol) MR_TIMED(KID_RENDER_BWD, st, (k_render_bwd<27><<<grid, 256, 0, st>>>(P)));
  else MR_TIMED(KID_RENDER_BWD, st, (k_render_bwd<18><<<grid, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_render_bwd");
  MR_TIMED(KID_RT_REDUCE, st, (k_rt_reduce<<<(unsigned)N, 256, 0, st>>>(rt_part, NB, gviews)));
  MR_CHECK_LAUNCH("k_rt_reduce");
  const int use_n = sp->light_kind == 0;
  const int vb = ceil_div(m->V, 256);
  if (vcol) {
    if (use_n) MR_TIMED(KID_VGRAD_A, st, (k_vgrad_a<27><<<vb, 256, 0, st>>>(m->V, m->vadj_ptr, m->vadj, gface, vraw, gnu)));
    MR_TIMED(KID_VGRAD_B, st, (k_vgrad_b<27><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, gface, gnu, use_n, gverts, gcol)));
  } else {
    if (use_n) MR_TIMED(KID_VGRAD_A, st, (k_vgrad_a<18><<<vb, 256, 0, st>>>(m->V, m->vadj_ptr, m->vadj, gface, vraw, gnu)));
    MR_TIMED(KID_VGRAD_B, st, (k_vgrad_b<18><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, gface, gnu, use_n, gverts, gcol)));
  }
  MR_CHECK_LAUNCH("k_vgrad");
  return MR_OK;
}

int32_t mr_timing_enable(int32_t enable) {
  if (enable && !g_t.created) {
    for (int i = 0; i < 2 * MR_TPOOL; ++i)
      if (hipEventCreate(&g_t.ev[i]) != hipSuccess) return set_err(MR_ELAUNCH, "hipEventCreate failed");
    g_t.created = 1;
  }
  g_t.enabled = enable ? 1 : 0;
  if (enable) {
    g_t.used = 0;
    g_t.dropped = 0;
  }
  return MR_OK;
}

int32_t mr_timing_read(int32_t* launches, double* total_ms, int32_t n) {
  if (!g_t.created) return set_err(MR_EINVAL, "timing never enabled");
  for (int k = 0; k < n && k < KID_COUNT; ++k) {
    launches[k] = 0;
    total_ms[k] = 0.0;
  }
  for (int i = 0; i < g_t.used; ++i) {
    if (hipEventSynchronize(g_t.ev[2 * i + 1]) != hipSuccess) return set_err(MR_ELAUNCH, "event sync failed");
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, g_t.ev[2 * i], g_t.ev[2 * i + 1]) != hipSuccess)
      return set_err(MR_ELAUNCH, "elapsed time failed");
    const int k = g_t.kid[i];
    if (k < n) {
      launches[k] += 1;
      total_ms[k] += ms;
    }
  }
  g_t.used = 0;
  return g_t.dropped ? set_err(MR_EWORKSPACE, "timing pool overflow (%d launches dropped)", g_t.dropped) : MR_OK;
}

const char* mr_timing_kernel_name(int32_t k) { return (k >= 0 && k < KID_COUNT) ? kKernelNames[k] : ""; }
int32_t mr_timing_kernel_count(void) { return KID_COUNT; }

}  // extern "C"
