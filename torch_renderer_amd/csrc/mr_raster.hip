// mi355r — MI355X (gfx950, CDNA4) rasterizer kernels + C ABI.
//
// Pipeline for a batch of N views (all launches async on one stream, no host sync):
//   1. binning     : k_bin_count (thread per (view, face): project or read face_verts,
//                    write a 64-B FaceRec, count the 8x8 tiles its padded bbox touches
//                    through an LDS histogram) -> k_bin_scan (one workgroup per view:
//                    entry offsets per tile, compact slot per non-empty tile, and work
//                    UNITS of <= 64 (tile, face) entries) -> k_bin_fill (tile lists).
//   2. k_tile_raster: persistent grid of independent waves (XCD-partitioned units, 3-deep
//                    unit/list/record prefetch): each lane clips one face's pixel bbox to
//                    the tile, the wave expands the (face, pixel) pairs 64 at a time (DPP
//                    prefix sums), evaluates each pair exactly and keeps the per-pixel
//                    minimum of the packed (z, face) key with ds_min_u64; the tile's 64
//                    winners go to its slot (a plain store, or a global u64 atomicMin merge
//                    when a tile has > 1 unit). The same waves stream the background.
//                    The minimum equals the CPU's "strictly nearer, earlier face wins".
//   3. k_shade<M>  : per covered tile, recompute each winner's fragment exactly and write
//                    M=0 PyTorch3D Fragments or M=1 shaded depth/silhouette/rgb.
//      K > 1 (modular): k_fill<0> then k_raster_k (per-lane sorted K-lists in LDS).
//   4. backward    : k_bwd_fused — per covered tile: shading backward (record handed over
//                    in LDS), raster + projection backward, per-face rows summed over runs
//                    of equal faces (segmented scan) with one atomic per run, per-slot R/T
//                    partials (k_rt_reduce). k_raster_bwd is the modular
//                    _C.rasterize_meshes_backward (any K).
//   5. vertex kernels gather per-face rows through a CSR vertex adjacency
//      (deterministic order) and chain the vertex-normal backward.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdarg.h>
#include <stdlib.h>

#include "../../include/mi355r.h"
#include "mr_common.h"
#include "mr_shade.h"

#define MR_TS 8         // raster tile edge: one 64-lane wave per 8x8 tile (lane = pixel)
#define MR_BT 32        // tile edge of the modular (fragments) backward
#define MR_HT 512       // LDS hash slots in the backward
#define MR_BIN_FPT 2     // faces per thread in the world-space binning kernels
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
enum KernelId { KID_BIN_COUNT, KID_BIN_SCAN, KID_BIN_FILL, KID_TILE_RASTER, KID_SHADE_FRAG, KID_SHADE_RENDER, KID_RASTER_BWD, KID_BWD_SHADE, KID_BWD_GEOM, KID_RT_REDUCE,
                KID_VGRAD_A, KID_VGRAD_B,
                KID_VNORMALS, KID_PROJECT, KID_PROJECT_BWD, KID_SHADE_REC, KID_FILL_FRAG,
                KID_RASTER_K, KID_BWD_FUSED, KID_RT_VGRAD_A, KID_FRAG_SHADE, KID_FRAG_SHADE_BWD, KID_SETUP, KID_BIN_RECT, KID_BIN_VIEW, KID_COUNT };
static const char* kKernelNames[KID_COUNT] = {"k_bin_count", "k_bin_scan", "k_bin_fill", "k_tile_raster",
                                              "k_shade<0>", "k_shade<1>",
                                              "k_raster_bwd", "k_bwd_shade(unused)", "k_bwd_geom(unused)", "k_rt_reduce",
                                              "k_vgrad_a", "k_vgrad_b",
                                              "k_vertex_normals", "k_project_faces", "k_project_faces_bwd",
                                              "k_shade_rec", "k_fill<0>", "k_raster_k", "k_bwd_fused",
                                              "k_rt_vgrad_a", "k_frag_shade_fwd", "k_frag_shade_bwd", "k_setup_zero",
                                              "k_bin_rect", "k_bin_view"};
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
// fill), work units, compact per-tile depth keys, and (fused path) the compact
// per-view list of covered (pixel, face) pairs.
// ---------------------------------------------------------------------------
#define MR_UE 64  // (tile, face) entries per raster work unit (one wave, one entry per lane)
// ctr[CTR_ENTRIES64 .. +2) is a u64: list entries allocated by the per-view binning (k_bin_view)
enum { CTR_UNITS = 0, CTR_SLOTS = 1, CTR_COVERED = 2, CTR_ENTRIES64 = 4, CTR_COUNT = 8 };

struct BinGeom {
  int TX, TY, T;
  int64_t list_cap;
  int64_t unit_cap;  // >= units the scan can emit: one per non-empty tile + list_cap / MR_UE
  int mfpb;          // max_faces_per_bin (0: none): a longer tile list takes the whole-view path
};
static BinGeom bin_geom(int H, int W, int64_t N, int64_t Ftot, int32_t mfpb) {
  BinGeom g;
  g.TX = ceil_div(W, MR_TS);
  g.TY = ceil_div(H, MR_TS);
  g.T = g.TX * g.TY;
  // Expected entries: ~(1 + 2*edge/8)^2 tiles per face + large faces; tiles whose list would
  // overflow take the exact full-view path (one unit scanning every face of the view).
  // max_faces_per_bin (if given) scales the reservation and caps each tile's list (PyTorch3D's per-bin cap).
  int64_t cap = 6 * Ftot + 2 * N * (int64_t)g.T + 65536;
  if (mfpb > 0) cap = (int64_t)mfpb * N * 16 + 65536;
  g.list_cap = cap < 0x40000000ll ? cap : 0x40000000ll;  // <= MR_CURSOR_OFF (k_bin_view); tiles past it take the exact path
  g.unit_cap = N * (int64_t)g.T + cap / MR_UE + 1;
  g.mfpb = mfpb > 0 ? mfpb : 0;
  return g;
}

struct RasterWS {
  FaceRec* recs;
  int* ctr;    // (CTR_COUNT) units / slots emitted by the scan, covered pixels, entries (u64)
  int* cnt;    // (N*T) entries per tile; zeroed per call together with ctr and vtot (count -> scan path)
  int* vtot;   // (N) list entries per view (count -> scan path)
  uint32_t* rects;  // (2 * Ftot) per record: tile rectangle (k_bin_view path)
  int* start;  // (N*T) entry offset of each tile inside its view's region
  int* cur;    // (N*T) fill cursors
  int* vbase;  // (N) first list entry of each view (saturating)
  int* tdone;  // (N*T) per slot: units of a shared slot still to finish (count-down; the last writes)
  int* vslot;  // (2N) first slot and number of slots of each view
  int* stile;  // (N*T) per slot: view * T + tile
  int4* units; // (unit_cap) {view*T + tile, first list entry (-1: every face of the view), entries, slot | multi<<31}
  int* list;   // list_cap
  unsigned long long* tkey;  // (N*T*64) per-slot (z, face) keys of tiles shared by several units
  int* sface;  // (N*T*64) per slot, per tile pixel (row-major 8x8): winning face record or -1
  ShadeRec* srec;  // (F) per-face shading inputs (fused path; F = faces of the shared mesh)
  float* grows;    // (F, 27) the fused backward's per-face gradient rows, cleared by the forward
  float4* frec;    // (N*T*64) fused path: per slot pixel the winner's fragment (b0, b1, b2, signed dist)
  ClipRec* crec;   // (2 * Ftot) barycentric conversion of near-plane sub-triangles (by record id)
  size_t bytes;
};
static RasterWS carve_raster_ws(void* base, int64_t N, int64_t Ftot, int H, int W, const BinGeom& g,
                                int64_t Fshade = 0) {
  (void)H; (void)W;
  RasterWS w;
  size_t off = 0;
  char* b = (char*)base;
  const size_t NT = (size_t)N * g.T;
  // face records: [0, Ftot) one per face instance, [Ftot, 2 Ftot) the second triangle of a face
  // split at the near plane (only written for such faces)
  w.recs = (FaceRec*)(b + off);
  off = align_up(off + sizeof(FaceRec) * 2 * (size_t)(Ftot > 0 ? Ftot : 1), 256);
  w.ctr = (int*)(b + off);  // 256-B aligned: the u64 entry counter at ctr + CTR_ENTRIES64
  w.cnt = w.ctr + CTR_COUNT;
  w.vtot = w.cnt + NT;
  off = align_up(off + sizeof(int) * (NT + (size_t)N + CTR_COUNT), 256);
  w.rects = (uint32_t*)(b + off);
  off = align_up(off + sizeof(uint32_t) * 2 * (size_t)(Ftot > 0 ? Ftot : 1), 256);
  w.start = (int*)(b + off);
  off = align_up(off + sizeof(int) * NT, 256);
  w.cur = (int*)(b + off);
  off = align_up(off + sizeof(int) * NT, 256);
  w.vbase = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)N, 256);
  w.tdone = (int*)(b + off);
  off = align_up(off + sizeof(int) * NT, 256);
  w.vslot = (int*)(b + off);
  off = align_up(off + sizeof(int) * 2 * (size_t)N, 256);
  w.stile = (int*)(b + off);
  off = align_up(off + sizeof(int) * NT, 256);
  w.units = (int4*)(b + off);
  off = align_up(off + sizeof(int4) * (size_t)g.unit_cap, 256);
  w.list = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)g.list_cap, 256);
  w.tkey = (unsigned long long*)(b + off);
  off = align_up(off + sizeof(unsigned long long) * 64 * NT, 256);
  w.sface = (int*)(b + off);
  off = align_up(off + sizeof(int) * 64 * NT, 256);
  w.srec = (ShadeRec*)(b + off);
  off = align_up(off + sizeof(ShadeRec) * (size_t)Fshade, 256);
  w.grows = (float*)(b + off);
  off = align_up(off + sizeof(float) * 27 * (size_t)Fshade, 256);
  w.frec = (float4*)(b + off);
  off = align_up(off + sizeof(float4) * (Fshade > 0 ? 64 * NT : 0), 256);
  w.crec = (ClipRec*)(b + off);
  off = align_up(off + sizeof(ClipRec) * 2 * (size_t)(Ftot > 0 ? Ftot : 1), 256);
  w.bytes = off;
  return w;
}
// Bytes to clear from w.ctr before a forward: the counters and, on the count -> scan path, the
// per-tile counts and per-view totals.
static size_t zero_bytes(int64_t N, const BinGeom& g, bool view_path) {
  return sizeof(int) * (view_path ? (size_t)CTR_COUNT : (size_t)N * g.T + (size_t)N + CTR_COUNT);
}

// ---------------------------------------------------------------------------
// 1. binning: count -> scan -> fill
// ---------------------------------------------------------------------------
struct SetupParams {
  int H, W, TX, TY, T;
  float bbox_pad;
  int persp, cull;
  int clipz;      // near-plane clipping on
  float zc;       // z_clip_value
  int64_t NF;     // face instances (record id of a pair's second triangle = NF + rid)
  ClipRec* crec;
  int64_t list_cap;
  FaceRec* recs;
  int* cnt;
  int* cur;
  int* list;
  int* vtot;
  const int* vbase;
  uint32_t* rects;  // k_bin_view path: per-record tile rectangles
  float* fv_out;    // k_bin_rect_world: face_verts (N*F,3,3) written beside the records (NULL: none)
  const int64_t* vff;  // world mode, distinct meshes: first union face of each view (N+1); NULL: shared mesh
};

// Wave-wide inclusive scans on DPP: row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 carry row totals across rows (GFX9 DPP). Full EXEC required.
MR_DEV int wave_incl_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}
MR_DEV int wave_incl_max(int v) {
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xa, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xc, 0xf, false));
  return v;
}
MR_DEV int wave_sum(int v) { return __builtin_amdgcn_readlane(wave_incl_sum(v), 63); }

// Sum of v over a 256-thread workgroup added to *dst with ONE atomic (thread 0). Uniform call.
MR_DEV void block_add_256(int v, int* dst) {
  __shared__ int part[4];
  const int w = wave_sum(v);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = ((part[0] + part[1]) + part[2]) + part[3];
    if (t) atomicAdd(dst, t);
  }
}

// A zero the compiler cannot see through, in a VGPR: a load indexed by it is a per-lane load
// whose wait sits at the first use, not a scalar-ised load + readfirstlane waited on at once.
MR_DEV int lane_zero() {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}

// Wave-local LDS hand-off (the 64 lanes of one wave write, then every lane reads). A wave's
// LDS operations execute in program order, so a wavefront-scope fence (no instructions, a
// compiler barrier) is all the ordering needed. A workgroup-scope fence here would emit
// s_waitcnt vmcnt(0) and stall on the wave's outstanding global stores every time.
MR_DEV void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS (and scalar) operations,
// not for its global stores (a __syncthreads waits vmcnt(0) too, i.e. a full memory round trip
// of every store in flight — expensive while other workgroups saturate HBM).
MR_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Inclusive scan over a 1024-thread workgroup (16 waves): DPP inside each wave, then the
// 16 wave totals scanned by every wave from LDS. `tot` = workgroup total. Uniform call only.
// LDSB: LDS-only barriers (the caller's global stores may stay in flight).
template <bool LDSB = false>
MR_DEV int block_incl_sum(int v, int* part16, int& tot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int w = wave_incl_sum(v);
  if (lane == 63) part16[wave] = w;
  if (LDSB) lds_barrier(); else __syncthreads();
  const int ws = wave_incl_sum(lane < 16 ? part16[lane] : 0);
  tot = __builtin_amdgcn_readlane(ws, 15);
  const int before = __shfl(ws, wave > 0 ? wave - 1 : 0, 64);
  if (LDSB) lds_barrier(); else __syncthreads();  // part16 is reused by the next call
  return w + (wave > 0 ? before : 0);
}

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

MR_DEV FaceRec make_rec_core(int cull, int persp, uint32_t face, const float v[3][3]);
MR_DEV FaceRec make_rec(const SetupParams& P, uint32_t face, const float v[3][3]) {
  return make_rec_core(P.cull, P.persp, face, v);
}
MR_DEV FaceRec make_rec_core(int cull, int persp, uint32_t face, const float v[3][3]) {
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
  if (cull && face_area < 0.0f) valid = false;
  if ((double)face_area <= MR_KEPS_D && (double)face_area >= -1.0f * MR_KEPS_D) valid = false;
  if (zmax < 0.0f) valid = false;
  bool fast = valid && __builtin_isfinite(r.area) && r.area != 0.0f;
  if (persp) fast = fast && r.z0 > 0.0f && r.z1 > 0.0f && r.z2 > 0.0f;
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

// The record(s) of face instance rid (mesh face `face`, projected corners v): the face itself,
// or with near-plane clipping its sub-triangle(s) (recs[rid] and, for a split quadrilateral,
// recs[NF + rid]) and their ClipRecs. Returns the second record through r1 (flags 0 if none).
MR_DEV FaceRec build_records(const SetupParams& P, int64_t rid, uint32_t face, const float v[3][3], FaceRec& r1) {
  r1.flags = 0u;
  if (!P.clipz) return make_rec(P, face, v);
  int i = 0;
  const int nb = clip_class(v, P.zc, i);
  if (nb == 0) return make_rec(P, face, v);
  FaceRec r0 = make_rec(P, face, v);
  if (nb == 3) {  // entirely behind the plane: culled
    r0.flags = 0u;
    return r0;
  }
  float sv[3][3];
  ClipRec cr;
  clip_sub(v, nb, i, 0, P.zc, P.persp != 0, sv, cr);
  r0 = make_rec(P, face, sv);
  r0.flags |= FR_CLIP | (nb == 1 ? FR_PAIR : 0u);
  P.crec[rid] = cr;
  if (nb == 1) {
    clip_sub(v, nb, i, 1, P.zc, P.persp != 0, sv, cr);
    r1 = make_rec(P, face, sv);
    r1.flags |= FR_CLIP | FR_PAIR;
    P.crec[P.NF + rid] = cr;
    P.recs[P.NF + rid] = r1;
  }
  return r0;
}

MR_DEV int rec_tile_count(const SetupParams& P, const FaceRec& r) {
  int tx0, tx1, ty0, ty1;
  if (!rec_tiles(P, r, tx0, tx1, ty0, ty1)) return 0;
  return (tx1 - tx0 + 1) * (ty1 - ty0 + 1);
}

// World mode (one mesh shared by N views, rec = n*F + f): project, write the record,
// count tile overlaps through an LDS histogram, flush one global atomic per touched tile
// and one per wave into the view's entry total.
template <bool LDS>
__global__ void __launch_bounds__(256) k_bin_count_world(SetupParams P, const float* __restrict__ verts,
                                                         const int32_t* __restrict__ faces, int64_t F,
                                                         const ViewRec* __restrict__ views, int fpt) {
  // fpt faces per thread: the per-block LDS histogram clear and flush (T entries each) are
  // paid once per 256 * fpt faces
  extern __shared__ __attribute__((aligned(16))) int hist[];
  const int n = blockIdx.y;
  if (LDS) {
    for (int i = threadIdx.x; i < P.T; i += blockDim.x) hist[i] = 0;
    __syncthreads();
  }
  int mine = 0;
  const ViewRec V = views[n];
  int64_t Fv = F, rbase = (int64_t)n * F, fbase = 0;  // as k_bin_rect_world
  if (P.vff) {
    rbase = fbase = P.vff[n];
    Fv = P.vff[n + 1] - rbase;
  }
  for (int k = 0; k < fpt; ++k) {
    const int64_t f = ((int64_t)blockIdx.x * fpt + k) * blockDim.x + threadIdx.x;
    if (f >= Fv) break;
    float v[3][3];
    world_face_verts(verts, faces, fbase + f, V, v);
    FaceRec r2;
    const FaceRec r = build_records(P, rbase + f, (uint32_t)(fbase + f), v, r2);
    P.recs[rbase + f] = r;
    for (int q = 0; q < 2; ++q) {
      const FaceRec& rq = q == 0 ? r : r2;
      int tx0, tx1, ty0, ty1;
      if (rec_tiles(P, rq, tx0, tx1, ty0, ty1)) {
        mine += (tx1 - tx0 + 1) * (ty1 - ty0 + 1);
        for (int ty = ty0; ty <= ty1; ++ty)
          for (int tx = tx0; tx <= tx1; ++tx) {
            const int t = ty * P.TX + tx;
            if (LDS) atomicAdd(&hist[t], 1);
            else atomicAdd(&P.cnt[(int64_t)n * P.T + t], 1);
          }
      }
    }
  }
  block_add_256(mine, &P.vtot[n]);  // also the barrier before the histogram flush
  if (LDS) {
    for (int i = threadIdx.x; i < P.T; i += blockDim.x)
      if (hist[i]) atomicAdd(&P.cnt[(int64_t)n * P.T + i], hist[i]);
  }
}

template <bool LDS>
__global__ void __launch_bounds__(256) k_bin_fill_world(SetupParams P, int64_t F, int fpt, int nviews, ShadeParams S,
                                                        ShadeRec* __restrict__ srec) {
  extern __shared__ __attribute__((aligned(16))) int hist[];
  const int n = blockIdx.y;
  if (n == nviews) {  // extra row: the mesh's per-face ShadeRecs (k_setup_zero wrote the normals)
    for (int k = 0; k < fpt; ++k) {
      const int64_t f = ((int64_t)blockIdx.x * fpt + k) * blockDim.x + threadIdx.x;
      if (f >= F) break;
      ShadeRec R;
      make_shade_rec(S, (uint32_t)f, R);
      srec[f] = R;
    }
    return;
  }
  const int64_t f0 = (int64_t)blockIdx.x * fpt * blockDim.x + threadIdx.x;
  int64_t Fv = F, rbase = (int64_t)n * F;  // view n's records [rbase, rbase + Fv), as k_bin_count_world
  if (P.vff) {
    rbase = P.vff[n];
    Fv = P.vff[n + 1] - rbase;
  }
  // q = 0: the face instance's record; q = 1: the second triangle of a split face (FR_PAIR)
  auto rec_q = [&](int64_t f, int q, FaceRec& r) -> bool {
    const int64_t rid = rbase + f;
    r = P.recs[rid];
    if (q == 0) return true;
    if (!(r.flags & FR_PAIR)) return false;
    r = P.recs[P.NF + rid];
    return true;
  };
  const int nq = P.clipz ? 2 : 1;
  if (LDS) {
    for (int i = threadIdx.x; i < P.T; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int k = 0; k < fpt; ++k) {
      const int64_t f = f0 + (int64_t)k * blockDim.x;
      for (int q = 0; q < nq && f < Fv; ++q) {
        FaceRec r;
        int tx0, tx1, ty0, ty1;
        if (rec_q(f, q, r) && rec_tiles(P, r, tx0, tx1, ty0, ty1))
          for (int ty = ty0; ty <= ty1; ++ty)
            for (int tx = tx0; tx <= tx1; ++tx) atomicAdd(&hist[ty * P.TX + tx], 1);
      }
    }
    __syncthreads();
    const int vb = P.vbase[n];
    for (int i = threadIdx.x; i < P.T; i += blockDim.x)
      if (hist[i]) hist[i] = vb + atomicAdd(&P.cur[(int64_t)n * P.T + i], hist[i]);  // reserve a block
    __syncthreads();
    for (int k = 0; k < fpt; ++k) {
      const int64_t f = f0 + (int64_t)k * blockDim.x;
      for (int q = 0; q < nq && f < Fv; ++q) {
        const int rid = (int)(rbase + f + (q ? P.NF : 0));
        FaceRec r;
        int tx0, tx1, ty0, ty1;
        if (rec_q(f, q, r) && rec_tiles(P, r, tx0, tx1, ty0, ty1))
          for (int ty = ty0; ty <= ty1; ++ty)
            for (int tx = tx0; tx <= tx1; ++tx) {
              const int pos = atomicAdd(&hist[ty * P.TX + tx], 1);
              if (pos < P.list_cap) P.list[pos] = rid;
            }
      }
    }
  } else {
    for (int k = 0; k < fpt; ++k) {
      const int64_t f = f0 + (int64_t)k * blockDim.x;
      for (int q = 0; q < nq && f < Fv; ++q) {
        const int rid = (int)(rbase + f + (q ? P.NF : 0));
        FaceRec r;
        int tx0, tx1, ty0, ty1;
        if (rec_q(f, q, r) && rec_tiles(P, r, tx0, tx1, ty0, ty1))
          for (int ty = ty0; ty <= ty1; ++ty)
            for (int tx = tx0; tx <= tx1; ++tx) {
              const int pos = P.vbase[n] + atomicAdd(&P.cur[(int64_t)n * P.T + ty * P.TX + tx], 1);
              if (pos < P.list_cap) P.list[pos] = rid;
            }
      }
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

// face_verts mode (PyTorch3D _C boundary): rec = packed face id. A workgroup takes a run of
// 256 * MR_FV_FPT consecutive faces: their face_verts (36 B each) are staged in LDS with
// coalesced 16-B loads, the mesh of each face comes from a binary search over the mesh offsets
// cached in LDS (N <= MR_FV_NMAX; else in global memory), and a workgroup whose faces all belong
// to one mesh (the common case: meshes are contiguous runs of faces) counts tiles through an LDS
// histogram, otherwise with global atomics.
#define MR_FV_FPT 2
#define MR_FV_NMAX 2048
struct FvBlock {
  int64_t f0, nf;  // first face, faces of this workgroup
  int n0, n1;      // meshes of the first and last face
};

MR_DEV int mesh_of_face_lds(const int* first32, int64_t N, int64_t f) {
  int lo = 0, hi = (int)N - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (first32[mid] <= f) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Workgroup prologue: cache the mesh offsets in LDS; stage this workgroup's face_verts in LDS.
MR_DEV FvBlock fv_block_setup(const float* __restrict__ fv, int64_t Ftot, const int64_t* __restrict__ first, int64_t N,
                              int* first32, float* sfv, bool stage) {
  FvBlock B;
  B.f0 = (int64_t)blockIdx.x * blockDim.x * MR_FV_FPT;
  B.nf = Ftot - B.f0 < (int64_t)blockDim.x * MR_FV_FPT ? Ftot - B.f0 : (int64_t)blockDim.x * MR_FV_FPT;
  if (N <= MR_FV_NMAX)
    for (int i = threadIdx.x; i < N; i += blockDim.x) first32[i] = (int)first[i];
  if (stage) {
    // 9 floats per face, the workgroup's floats start 16-B aligned (f0 is a multiple of 4)
    const float4* src = (const float4*)(fv + 9 * B.f0);
    const int n4 = ((uintptr_t)src & 15) == 0 ? (int)(9 * B.nf) / 4 : 0;  // else scalar loads below
    for (int i = threadIdx.x; i < n4; i += blockDim.x) ((float4*)sfv)[i] = src[i];
    for (int i = 4 * n4 + threadIdx.x; i < 9 * B.nf; i += blockDim.x) sfv[i] = fv[9 * B.f0 + i];
  }
  __syncthreads();
  B.n0 = N <= MR_FV_NMAX ? mesh_of_face_lds(first32, N, B.f0) : mesh_of_face(first, N, B.f0);
  B.n1 = N <= MR_FV_NMAX ? mesh_of_face_lds(first32, N, B.f0 + B.nf - 1) : mesh_of_face(first, N, B.f0 + B.nf - 1);
  return B;
}

MR_DEV int fv_mesh(const FvBlock& B, const int* first32, const int64_t* first, int64_t N, int64_t f) {
  if (B.n0 == B.n1) return B.n0;
  return N <= MR_FV_NMAX ? mesh_of_face_lds(first32, N, f) : mesh_of_face(first, N, f);
}

template <bool LDS>
__global__ void __launch_bounds__(256) k_bin_count_fv(SetupParams P, const float* __restrict__ fv, int64_t Ftot,
                                                      const int64_t* __restrict__ first, int64_t N) {
  extern __shared__ __attribute__((aligned(16))) int hist[];
  __shared__ __attribute__((aligned(16))) float sfv[9 * 256 * MR_FV_FPT];
  __shared__ int first32[MR_FV_NMAX];
  const FvBlock B = fv_block_setup(fv, Ftot, first, N, first32, sfv, true);
  const bool lds = LDS && B.n0 == B.n1;  // uniform over the workgroup
  if (lds) {
    for (int i = threadIdx.x; i < P.T; i += blockDim.x) hist[i] = 0;
    __syncthreads();
  }
  // entry totals: of the first mesh (mine) and, in a workgroup that straddles meshes, of the
  // last (mine1) — one block-wide sum each; only meshes strictly inside the workgroup's face run
  // (small meshes) take a per-face atomic. (Per-face atomics on the few total counters of a
  // straddling workgroup serialise at the L2: they made this kernel 10x slower.)
  int mine = 0, mine1 = 0;
  for (int k = 0; k < MR_FV_FPT; ++k) {
    const int64_t lf = (int64_t)k * blockDim.x + threadIdx.x;
    if (lf >= B.nf) break;
    const int64_t f = B.f0 + lf;
    const int n = fv_mesh(B, first32, first, N, f);
    float v[3][3];
    for (int c = 0; c < 3; ++c)
      for (int q = 0; q < 3; ++q) v[c][q] = sfv[9 * lf + 3 * c + q];
    FaceRec r2;
    const FaceRec r = build_records(P, f, (uint32_t)f, v, r2);
    P.recs[f] = r;
    int m = 0;
    for (int q = 0; q < 2; ++q) {
      const FaceRec& rq = q == 0 ? r : r2;
      int tx0, tx1, ty0, ty1;
      if (rec_tiles(P, rq, tx0, tx1, ty0, ty1)) {
        m += (tx1 - tx0 + 1) * (ty1 - ty0 + 1);
        for (int ty = ty0; ty <= ty1; ++ty)
          for (int tx = tx0; tx <= tx1; ++tx) {
            if (lds) atomicAdd(&hist[ty * P.TX + tx], 1);
            else atomicAdd(&P.cnt[(int64_t)n * P.T + ty * P.TX + tx], 1);
          }
      }
    }
    if (n == B.n0) mine += m;
    else if (n == B.n1) mine1 += m;
    else if (m) atomicAdd(&P.vtot[n], m);
  }
  block_add_256(mine, &P.vtot[B.n0]);  // also the barrier before the histogram flush
  if (B.n1 != B.n0) {
    __syncthreads();  // block_add_256's partials are reused
    block_add_256(mine1, &P.vtot[B.n1]);
  }
  if (lds) {
    for (int i = threadIdx.x; i < P.T; i += blockDim.x)
      if (hist[i]) atomicAdd(&P.cnt[(int64_t)B.n0 * P.T + i], hist[i]);
  }
}

template <bool LDS>
__global__ void __launch_bounds__(256) k_bin_fill_fv(SetupParams P, int64_t Ftot, const int64_t* __restrict__ first,
                                                     int64_t N) {
  extern __shared__ __attribute__((aligned(16))) int hist[];
  __shared__ int first32[MR_FV_NMAX];
  const FvBlock B = fv_block_setup(nullptr, Ftot, first, N, first32, nullptr, false);
  const bool lds = LDS && B.n0 == B.n1;
  const int nq = P.clipz ? 2 : 1;
  auto rec_q = [&](int64_t f, int q, FaceRec& r) -> bool {
    r = P.recs[f];
    if (q == 0) return true;
    if (!(r.flags & FR_PAIR)) return false;
    r = P.recs[P.NF + f];
    return true;
  };
  if (lds) {
    for (int i = threadIdx.x; i < P.T; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int k = 0; k < MR_FV_FPT; ++k) {
      const int64_t lf = (int64_t)k * blockDim.x + threadIdx.x;
      for (int q = 0; q < nq && lf < B.nf; ++q) {
        FaceRec r;
        int tx0, tx1, ty0, ty1;
        if (rec_q(B.f0 + lf, q, r) && rec_tiles(P, r, tx0, tx1, ty0, ty1))
          for (int ty = ty0; ty <= ty1; ++ty)
            for (int tx = tx0; tx <= tx1; ++tx) atomicAdd(&hist[ty * P.TX + tx], 1);
      }
    }
    __syncthreads();
    const int vb = P.vbase[B.n0];
    for (int i = threadIdx.x; i < P.T; i += blockDim.x)
      if (hist[i]) hist[i] = vb + atomicAdd(&P.cur[(int64_t)B.n0 * P.T + i], hist[i]);  // reserve a block
    __syncthreads();
    for (int k = 0; k < MR_FV_FPT; ++k) {
      const int64_t lf = (int64_t)k * blockDim.x + threadIdx.x;
      for (int q = 0; q < nq && lf < B.nf; ++q) {
        FaceRec r;
        int tx0, tx1, ty0, ty1;
        if (rec_q(B.f0 + lf, q, r) && rec_tiles(P, r, tx0, tx1, ty0, ty1))
          for (int ty = ty0; ty <= ty1; ++ty)
            for (int tx = tx0; tx <= tx1; ++tx) {
              const int pos = atomicAdd(&hist[ty * P.TX + tx], 1);
              if (pos < P.list_cap) P.list[pos] = (int)(B.f0 + lf + (q ? P.NF : 0));
            }
      }
    }
  } else {
    for (int k = 0; k < MR_FV_FPT; ++k) {
      const int64_t lf = (int64_t)k * blockDim.x + threadIdx.x;
      if (lf >= B.nf) break;
      const int64_t f = B.f0 + lf;
      const int n = fv_mesh(B, first32, first, N, f);
      for (int q = 0; q < nq; ++q) {
        FaceRec r;
        int tx0, tx1, ty0, ty1;
        if (rec_q(f, q, r) && rec_tiles(P, r, tx0, tx1, ty0, ty1))
          for (int ty = ty0; ty <= ty1; ++ty)
            for (int tx = tx0; tx <= tx1; ++tx) {
              const int pos = P.vbase[n] + atomicAdd(&P.cur[(int64_t)n * P.T + ty * P.TX + tx], 1);
              if (pos < P.list_cap) P.list[pos] = (int)(f + (q ? P.NF : 0));
            }
      }
    }
  }
}

struct ScanParams {
  int T, mfpb;
  int64_t list_cap;
  const int* cnt;
  const int* vtot;
  int* start;
  int* cur;
  int* vbase;
  int* tdone;
  int* vslot;
  int* stile;
  int4* units;
  int* ctr;
  unsigned long long* tkey;
  const int64_t* view_count;  // NULL: shared mode (count = F)
  int64_t F;
};

// One 1024-thread workgroup per view:
//  * vbase[n] = entries of the views before n (from the per-view totals of k_bin_count);
//  * start/cur = per-tile exclusive scan of the entry counts inside the view's region;
//  * every non-empty tile gets a compact slot and ceil(entries / MR_UE) work units
//    (one unit scanning every face of the view when its list would overflow the pool);
//    view bases for slots and units come from one atomic each (any view order is fine:
//    the raster result does not depend on the order units run in);
//  * the 64 keys of a slot that several units share start at EMPTY (they merge by atomicMin)
//    and its count-down starts at units - 1 (the unit that takes it to -1 appends the pixels).
#define MR_KEY_EMPTY ((0x7f800000ull << 32) | 0x7fffffffull)
#define MR_SCAN_MULTI 4096  // multi-unit slots of one view whose keys the block initialises
__global__ void __launch_bounds__(1024) k_bin_scan(ScanParams P) {
  __shared__ int part[16];
  __shared__ long long red[16];
  __shared__ int base[2];
  __shared__ int nmulti;
  __shared__ int multi_slot[MR_SCAN_MULTI];
  const int n = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // vb = sum of vtot[m < n]
  long long s = 0;
  for (int m = t; m < n; m += 1024) s += P.vtot[m];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  long long vb = 0;
  for (int k = 0; k < 16; ++k) vb += red[k];
  if (t == 0) P.vbase[n] = (int)(vb < 0x7fffffffll ? vb : 0x7fffffffll);
  const int vcount = (int)(P.view_count ? (P.view_count[n] < 0x7fffffffll ? P.view_count[n] : 0x7fffffffll) : P.F);
  const int* c = P.cnt + (int64_t)n * P.T;
  // Each thread owns a run of C consecutive tiles, so the view needs three block-wide scans
  // (entries, units, slots) instead of three per 1024 tiles; slots and units still come out in
  // tile order.
  const int C = (P.T + 1023) / 1024;
  const int t0 = min(t * C, P.T), t1 = min(t0 + C, P.T);
  int le = 0;
  for (int tt = t0; tt < t1; ++tt) le += c[tt];
  int te;
  const int ex0 = block_incl_sum(le, part, te) - le;  // view-local entry offset of tile t0
  // pass 1: entry offsets; unit and slot counts of the run
  int my_u = 0, my_s = 0;
  for (int tt = t0, ex = ex0; tt < t1; ++tt) {
    const int cc = c[tt];
    P.start[(int64_t)n * P.T + tt] = ex;
    P.cur[(int64_t)n * P.T + tt] = ex;
    const bool ovf = cc > 0 && (vb + ex + cc > P.list_cap || (P.mfpb > 0 && cc > P.mfpb));
    my_u += cc == 0 ? 0 : ovf ? 1 : (cc + MR_UE - 1) / MR_UE;
    my_s += cc > 0 ? 1 : 0;
    ex += cc;
  }
  int au, as;
  const int iu = block_incl_sum(my_u, part, au);
  const int is = block_incl_sum(my_s, part, as);
  if (t == 0) {
    base[0] = atomicAdd(&P.ctr[CTR_UNITS], au);
    base[1] = atomicAdd(&P.ctr[CTR_SLOTS], as);
    P.vslot[n] = base[1];
    P.vslot[gridDim.x + n] = as;
    nmulti = 0;
  }
  __syncthreads();
  // pass 2: units, slots, key init for shared slots
  int u0 = base[0] + iu - my_u, slot = base[1] + is - my_s;
  for (int tt = t0, ex = ex0; tt < t1; ++tt) {
    const int cc = c[tt];
    const bool ovf = cc > 0 && (vb + ex + cc > P.list_cap || (P.mfpb > 0 && cc > P.mfpb));
    const int nu = cc == 0 ? 0 : ovf ? 1 : (cc + MR_UE - 1) / MR_UE;
    const int gt = n * P.T + tt;
    if (cc > 0) P.stile[slot] = gt;
    const int multi = nu > 1 ? (int)0x80000000u : 0;
    for (int k = 0; k < nu; ++k) {
      int4 U;
      U.x = gt;
      U.y = ovf ? -1 : (int)(vb + ex) + k * MR_UE;
      U.z = ovf ? vcount : min(MR_UE, cc - k * MR_UE);
      U.w = slot | multi;
      P.units[u0 + k] = U;
    }
    if (nu > 1) {
      P.tdone[slot] = nu - 1;
      const int k = atomicAdd(&nmulti, 1);
      if (k < MR_SCAN_MULTI) multi_slot[k] = slot;
      else
        for (int i = 0; i < 64; ++i) P.tkey[(int64_t)slot * 64 + i] = MR_KEY_EMPTY;
    }
    u0 += nu;
    slot += cc > 0 ? 1 : 0;
    ex += cc;
  }
  // the 64 keys of every multi-unit slot, written by the whole block (a slot's 512 B by 64
  // consecutive threads) instead of 64 serial stores by the tile's thread
  __syncthreads();
  const int nm = min(nmulti, MR_SCAN_MULTI);
  for (int i = t; i < nm * 64; i += 1024) P.tkey[(int64_t)multi_slot[i >> 6] * 64 + (i & 63)] = MR_KEY_EMPTY;
}

// ---------------------------------------------------------------------------
// 1b. per-view binning (the common case: tile grids of <= MR_VIEW_TMAX tiles, <= 256 per side)
// ---------------------------------------------------------------------------
// k_bin_rect_* project the faces and write each record's 8x8-tile rectangle (4 bytes); one
// 1024-thread workgroup per view (k_bin_view) then counts the view's tile lists in an LDS
// histogram, scans them, emits the view's slots and work units, and fills the lists through LDS
// cursors: count -> scan -> fill of one view never leaves the workgroup (no global per-tile
// counters, no per-tile global atomics, one launch instead of two). List, slot and unit space
// come from one atomic each per view; the raster result does not depend on their order.
#define MR_VIEW_TMAX 16384              // LDS histogram: 64 KB
#define MR_VIEW_FMAX 65536              // faces per view (mean) above which the count -> scan path is used
#define MR_RECT_NONE 0x000000ffu        // tx0 = 255 > tx1 = 0: an empty rectangle
#define MR_CURSOR_OFF 0x40000000        // fill cursor of a tile whose list is not filled (list_cap <= it)
#define MR_VIEW_RPT 8                   // rectangles per thread per chunk
MR_DEV uint32_t rec_rect(const SetupParams& P, const FaceRec& r) {
  int tx0, tx1, ty0, ty1;
  if (!rec_tiles(P, r, tx0, tx1, ty0, ty1)) return MR_RECT_NONE;
  return (uint32_t)tx0 | ((uint32_t)tx1 << 8) | ((uint32_t)ty0 << 16) | ((uint32_t)ty1 << 24);
}

MR_DEV void vertex_normal(const float* __restrict__ verts, const int32_t* __restrict__ faces,
                          const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj, int64_t v,
                          float* __restrict__ vn, float* __restrict__ vraw);
// The fused forward's setup, world mode (the first launch of the per-view path): grid rows 1..N
// project (face, view) pairs, one thread each; row 0, dispatched first (the CSR gathers are its
// longest dependent chain), computes the vertex normals when the call asks for them (as
// k_setup_zero does on the count -> scan path) and clears the work counters. The ShadeRecs, which
// read the normals, are packed by extra workgroups of k_bin_view.
// CLIP: near-plane clipping on (its sub-triangle code indexes corners dynamically: scratch);
// the CLIP = false instantiation carries none of it.
struct NormalsArgs {
  int64_t V;
  const int32_t* ptr;
  const int32_t* adj;
  float* vn;    // NULL: no normals to compute
  float* vraw;
  float4* zero4;   // the fused backward's face-gradient rows, cleared here (nzero4 float4s; NULL: none)
  int64_t nzero4;
};
// OpenCV poses converted on the fly (mr_render_forward_opencv): element k of view n's record,
// as k_views_from_opencv writes it (torch_renderer.py:73-80; bitwise the torch conversion).
struct CvPoses {
  const float* R;  // NULL: the view records are given
  int64_t sR;
  const float* t;
  int64_t sT;
  const float* intr;
  int64_t sI;
  float* out;  // (N,16) view records written for the later launches
  int opencv;  // 1: OpenCV R_cv / t_cv (converted); 0: PyTorch3D R / T as given
};
MR_DEV float cv_view_elem(const CvPoses& C, int64_t n, int k) {
  float v;
  if (!C.opencv) {
    v = k < 9 ? C.R[n * C.sR + k] : k < 12 ? C.t[n * C.sT + (k - 9)] : C.intr[n * C.sI + (k - 12)];
  } else if (k < 9) {  // R_p3d[a][b] = R_cv[b][a] * s[b], s = (-1, -1, 1)
    const int a = k / 3, b = k - 3 * a;
    v = C.R[n * C.sR + 3 * b + a];
    if (b < 2) v = -v;
  } else if (k < 12) {
    v = C.t[n * C.sT + (k - 9)];
    if (k < 11) v = -v;
  } else {
    v = C.intr[n * C.sI + (k - 12)];
  }
  return v;
}
template <bool CLIP>
__global__ void __launch_bounds__(256) k_bin_rect_world(SetupParams P, const float* __restrict__ verts,
                                                        const int32_t* __restrict__ faces, int64_t F,
                                                        const ViewRec* __restrict__ views, NormalsArgs NA,
                                                        int* __restrict__ ctr, CvPoses C) {
  const int n = (int)blockIdx.y - 1;
  if (n >= 0 && C.R && blockIdx.x == 0 && threadIdx.x < 16) C.out[(int64_t)n * 16 + threadIdx.x] = cv_view_elem(C, n, threadIdx.x);
  if (n < 0) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < CTR_COUNT) ctr[threadIdx.x] = 0;
    for (int64_t i = v; i < NA.nzero4; i += (int64_t)gridDim.x * blockDim.x) NA.zero4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (NA.vn && v < NA.V) vertex_normal(verts, faces, NA.ptr, NA.adj, v, NA.vn, NA.vraw);
    return;
  }
static_assert(sizeof(FaceRec) == 64, "FaceRec is staged as 4 float4");
  // One face per thread; the workgroup's records (and face_verts rows) are contiguous in HBM, so
  // they are staged through LDS and stored as whole lines (each store instruction writes 1 KB of
  // consecutive bytes instead of 64 lanes' 16-B pieces 64 B apart).
  // s4 element e (record e / 4, quarter e % 4) at e + e / 16: the record-major writes (16-B pieces
  // 64 B apart) then land on distinct bank groups (4-way conflicts without the pad)
  __shared__ float4 s4[4 * 256 + 64];
  __shared__ float s9[9 * 256];
  // view n's faces: mesh faces [fbase, fbase + Fv) -> records [rbase, rbase + Fv)
  int64_t Fv = F, rbase = (int64_t)n * F, fbase = 0;
  if (P.vff) {  // distinct meshes: view n renders mesh n (records = union faces)
    rbase = fbase = P.vff[n];
    Fv = P.vff[n + 1] - rbase;
  }
  const int t = threadIdx.x;
  const int64_t fb = (int64_t)blockIdx.x * 256;
  if (fb >= Fv) return;  // uniform over the workgroup
  const int64_t fl = fb + t;
  const int nf = (int)(Fv - fb < 256 ? Fv - fb : 256);
  const int64_t rid0 = rbase + fb;
  if (fl < Fv) {
    float v[3][3];
    ViewRec V;
    if (C.R) {
      float* e = (float*)&V;
#pragma unroll
      for (int k = 0; k < 16; ++k) e[k] = cv_view_elem(C, n, k);
    } else {
      V = views[n];
    }
    const int64_t f = fbase + fl;
    world_face_verts(verts, faces, f, V, v);
    const int64_t rid = rid0 + t;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int q = 0; q < 3; ++q) s9[9 * t + 3 * c + q] = v[c][q];
    FaceRec r2;
    const FaceRec r = CLIP ? build_records(P, rid, (uint32_t)f, v, r2) : make_rec(P, (uint32_t)f, v);
    float4 q4[4];
    __builtin_memcpy(q4, &r, sizeof(q4));
#pragma unroll
    for (int q = 0; q < 4; ++q) s4[4 * t + q + (t >> 2)] = q4[q];
    P.rects[rid] = rec_rect(P, r);
    if (CLIP) P.rects[P.NF + rid] = (r.flags & FR_PAIR) ? rec_rect(P, r2) : MR_RECT_NONE;
  }
  __syncthreads();
  float4* d4 = (float4*)(P.recs + rid0);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j * 256 + t < 4 * nf) d4[j * 256 + t] = s4[j * 256 + t + ((j * 256 + t) >> 4)];
  if (P.fv_out) {
    float* d9 = P.fv_out + rid0 * 9;
#pragma unroll
    for (int j = 0; j < 9; ++j)
      if (j * 256 + t < 9 * nf) d9[j * 256 + t] = s9[j * 256 + t];
  }
}

// face_verts mode (record = packed face id): the workgroup's face_verts staged through LDS
// with 16-B loads.
template <bool CLIP>
__global__ void __launch_bounds__(256) k_bin_rect_fv(SetupParams P, const float* __restrict__ fv, int64_t Ftot,
                                                     int* __restrict__ ctr) {
  __shared__ __attribute__((aligned(16))) float sfv[9 * 256];
  const int64_t f0 = (int64_t)blockIdx.x * blockDim.x;
  if (blockIdx.x == 0 && threadIdx.x < CTR_COUNT) ctr[threadIdx.x] = 0;  // the work counters (k_bin_view)
  const int nf = (int)(Ftot - f0 < (int64_t)blockDim.x ? Ftot - f0 : (int64_t)blockDim.x);
  const float4* src = (const float4*)(fv + 9 * f0);  // f0 % 256 == 0: 16-B aligned if fv is
  const int n4 = ((uintptr_t)src & 15) == 0 ? 9 * nf / 4 : 0;
  for (int i = threadIdx.x; i < n4; i += blockDim.x) ((float4*)sfv)[i] = src[i];
  for (int i = 4 * n4 + threadIdx.x; i < 9 * nf; i += blockDim.x) sfv[i] = fv[9 * f0 + i];
  __syncthreads();
  if ((int)threadIdx.x >= nf) return;
  const int64_t f = f0 + threadIdx.x;
  float v[3][3];
  for (int c = 0; c < 3; ++c)
    for (int q = 0; q < 3; ++q) v[c][q] = sfv[9 * threadIdx.x + 3 * c + q];
  FaceRec r2;
  const FaceRec r = CLIP ? build_records(P, f, (uint32_t)f, v, r2) : make_rec(P, (uint32_t)f, v);
  P.recs[f] = r;
  P.rects[f] = rec_rect(P, r);
  if (CLIP) P.rects[P.NF + f] = (r.flags & FR_PAIR) ? rec_rect(P, r2) : MR_RECT_NONE;
}

struct ViewBinParams {
  int T, TX, mfpb, clipz;
  int nviews;
  int ranges;  // write cnt / start per tile (read by k_raster_k, K > 1)
  int64_t list_cap, NF;
  const uint32_t* rects;
  const int64_t* first;       // NULL: shared mode (view n's records are n*F + f)
  const int64_t* view_count;  // NULL: shared mode (F faces per view)
  int64_t F;
  int* cnt;
  int* start;
  int* vbase;
  int* tdone;
  int* vslot;
  int* stile;
  int4* units;
  int* ctr;
  unsigned long long* tkey;
  int* list;
  // workgroups N.. pack the mesh's ShadeRecs (fused path; srec NULL otherwise)
  ShadeParams S;
  ShadeRec* srec;
  int64_t Fs;
  int nsrec_wg;  // ShadeRec workgroups (N .. N + nsrec_wg - 1); the background ones follow (k_bin_view<MODE, CH>)
  int stage_cap;  // list entries of a view staged in LDS (after the histogram)
};

template <typename Fn>
MR_DEV void rect_tiles(uint32_t r, int TX, Fn&& fn) {
  const int tx0 = r & 255, tx1 = (r >> 8) & 255, ty0 = (r >> 16) & 255, ty1 = r >> 24;
  for (int ty = ty0; ty <= ty1; ++ty)
    for (int tx = tx0; tx <= tx1; ++tx) fn(ty * TX + tx);
}

MR_DEV void bin_view_body(const ViewBinParams& P) {
  extern __shared__ __attribute__((aligned(16))) int hist[];  // T (+ T/64 pad): counts, then fill cursors
  __shared__ int part[16];
  __shared__ long long base[3];
  __shared__ int nmulti;
  __shared__ int multi_slot[MR_SCAN_MULTI];
  const int n = blockIdx.x, t = threadIdx.x;
  if (n >= (int)P.nviews) {  // ShadeRec workgroups (they run on the CUs the views leave idle)
    const int64_t f = (int64_t)(n - P.nviews) * 1024 + t;
    if (f < P.Fs) {
      ShadeRec R;
      make_shade_rec(P.S, (uint32_t)f, R);
      P.srec[f] = R;
    }
    return;
  }
  // tile tt lives at hist[tt + tt / 64] (the scan's per-thread runs of C tiles spread over the
  // banks); a view's rectangles are read in chunks of MR_VIEW_RPT per thread, all loads of a
  // chunk in flight together, and a view of one chunk keeps them in registers for the fill.
  const int j = t;
  const int64_t f0 = P.first ? P.first[n] : (int64_t)n * P.F;
  const int vcount = (int)(P.view_count ? (P.view_count[n] < 0x7fffffffll ? P.view_count[n] : 0x7fffffffll) : P.F);
  for (int i = t; i < P.T + (P.T >> 6); i += 1024) hist[i] = 0;
  if (t == 0) nmulti = 0;
  lds_barrier();
  const int nq = P.clipz ? 2 : 1;
  uint32_t rr[MR_VIEW_RPT][2];
  auto load_chunk = [&](int i0) {
#pragma unroll
    for (int k = 0; k < MR_VIEW_RPT; ++k)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = i0 + k * 1024 + j;
        rr[k][q] = (q < nq && i < vcount) ? P.rects[(q ? P.NF : 0) + f0 + i] : MR_RECT_NONE;
      }
  };
  // count
#pragma unroll 1
  for (int i0 = 0; i0 < vcount; i0 += 1024 * MR_VIEW_RPT) {
    load_chunk(i0);
#pragma unroll
    for (int k = 0; k < MR_VIEW_RPT; ++k)
#pragma unroll
      for (int q = 0; q < 2; ++q) rect_tiles(rr[k][q], P.TX, [&](int tt) { atomicAdd(&hist[tt + (tt >> 6)], 1); });
  }
  lds_barrier();
  // scan: each thread owns a run of C consecutive tiles (entries, units, slots in tile order)
  const int C = (P.T + 1023) / 1024;
  const int t0 = min(t * C, P.T), t1 = min(t0 + C, P.T);
  int le = 0, my_u = 0, my_s = 0;
  for (int tt = t0; tt < t1; ++tt) {
    const int cc = hist[tt + (tt >> 6)];
    le += cc;
    const bool mo = P.mfpb > 0 && cc > P.mfpb;  // PyTorch3D's per-bin cap: the whole-view path
    my_u += cc == 0 ? 0 : mo ? 1 : (cc + MR_UE - 1) / MR_UE;
    my_s += cc > 0 ? 1 : 0;
  }
  int te, au, as;
  const int ex0 = block_incl_sum<true>(le, part, te) - le;
  const int iu = block_incl_sum<true>(my_u, part, au);
  const int is = block_incl_sum<true>(my_s, part, as);
  // the three allocations from three waves: their round trips overlap instead of queueing
  if (t == 0) {
    base[0] = atomicAdd(&P.ctr[CTR_UNITS], au);
  } else if (t == 64) {
    const int b1 = atomicAdd(&P.ctr[CTR_SLOTS], as);
    base[1] = b1;
    P.vslot[n] = b1;
    P.vslot[P.nviews + n] = as;
  } else if (t == 128) {
    base[2] = (long long)atomicAdd((unsigned long long*)(P.ctr + CTR_ENTRIES64), (unsigned long long)te);
  }
  lds_barrier();
  const long long vb = base[2];
  if (t == 0) P.vbase[n] = (int)(vb < 0x7fffffffll ? vb : 0x7fffffffll);
  int u0 = (int)base[0] + iu - my_u, slot = (int)base[1] + is - my_s;
  for (int tt = t0, ex = ex0; tt < t1; ++tt) {
    const int cc = hist[tt + (tt >> 6)];
    const int gt = n * P.T + tt;
    if (P.ranges) {
      P.cnt[gt] = cc;
      P.start[gt] = ex;
    }
    const bool mo = P.mfpb > 0 && cc > P.mfpb;
    const int nu = cc == 0 ? 0 : mo ? 1 : (cc + MR_UE - 1) / MR_UE;
    // a list that would overflow the pool: its first unit scans every face of the view, the
    // others (reserved before the pool base was known) are empty
    const bool ovf = cc > 0 && (mo || vb + ex + cc > P.list_cap);
    if (cc > 0) P.stile[slot] = gt;
    const int multi = nu > 1 ? (int)0x80000000u : 0;
    for (int k = 0; k < nu; ++k) {
      int4 U;
      U.x = gt;
      U.y = ovf ? -1 : (int)(vb + ex) + k * MR_UE;
      U.z = ovf ? (k == 0 ? vcount : 0) : min(MR_UE, cc - k * MR_UE);
      U.w = slot | multi;
      P.units[u0 + k] = U;
    }
    if (nu > 1) {
      P.tdone[slot] = nu - 1;
      const int k = atomicAdd(&nmulti, 1);
      if (k < MR_SCAN_MULTI) multi_slot[k] = slot;
      else
        for (int i = 0; i < 64; ++i) P.tkey[(int64_t)slot * 64 + i] = MR_KEY_EMPTY;
    }
    hist[tt + (tt >> 6)] = ovf ? MR_CURSOR_OFF : (int)(vb + ex);  // fill cursor (overflowing lists are not filled)
    u0 += nu;
    slot += cc > 0 ? 1 : 0;
    ex += cc;
  }
  lds_barrier();
  const int nm = min(nmulti, MR_SCAN_MULTI);
  for (int i = t; i < nm * 64; i += 1024) P.tkey[(int64_t)multi_slot[i >> 6] * 64 + (i & 63)] = MR_KEY_EMPTY;
  // fill: the view's entries occupy [vb, vb + te) of the pool; the first stage_cap of them are
  // staged in LDS and stored as consecutive lines afterwards (scattered 4-B stores issue one
  // lane per cycle), the rest (a view larger than the stage) go straight to the pool
  int* stage = hist + ((P.T + (P.T >> 6) + 3) & ~3);
  const int lst = min(te, P.stage_cap);
  const bool one = vcount <= 1024 * MR_VIEW_RPT;  // the rectangles are still in registers
#pragma unroll 1
  for (int i0 = 0; i0 < vcount; i0 += 1024 * MR_VIEW_RPT) {
    if (!one) load_chunk(i0);
#pragma unroll
    for (int k = 0; k < MR_VIEW_RPT; ++k)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int rid = (int)((q ? P.NF : 0) + f0 + i0 + k * 1024 + j);
        rect_tiles(rr[k][q], P.TX, [&](int tt) {
          // an overflowing tile's cursor starts at MR_CURSOR_OFF >= list_cap: no store, and no
          // read of the cursor before the atomic
          const int pos = atomicAdd(&hist[tt + (tt >> 6)], 1);
          if (pos < P.list_cap) {
            const int rel = (int)(pos - vb);
            if (rel < lst) stage[rel] = rid;
            else P.list[pos] = rid;
          }
        });
      }
  }
  lds_barrier();
  for (int i = t; i < lst; i += 1024)
    if (vb + i < P.list_cap) P.list[vb + i] = stage[i];
}
__global__ void __launch_bounds__(1024) k_bin_view(ViewBinParams P) { bin_view_body(P); }

// ---------------------------------------------------------------------------
// 2. raster: per-tile depth keys (k_tile_raster), then a streaming resolve (k_resolve)
// ---------------------------------------------------------------------------
// Exact per-(pixel, face) decision and depth: eval_face's return value and pz, without
// the point-triangle distance unless blur > 0 and the pixel is outside. On the fast path
// (blur == 0, FR_FAST) the edge signs reject before any division: a pixel whose edge
// functions do not all carry the area's strict sign has some w_i <= 0, hence c_i <= 0
// (all z > 0), hence is not inside, hence eval_face rejects it too.
// Candidate pixels of one face in one 8x8 tile, as a 64-bit coverage mask (bit 8 * row + col,
// tile-local): the rectangle [rx0, rx1] x [ry0, ry1] (the face's padded bbox clipped to the
// tile), narrowed on the fast path to the columns of each row whose centre can pass the
// edge-sign test. Every pixel frag_keep keeps is in the mask; a few columns within 0.02 px of an
// edge are extra (frag_keep rejects them exactly).
// Edge E_i(p) = (px - ax)(by - ay) - (py - ay)(bx - ax), kept iff s E_i > 0 (s = sign of the
// area). On row py this is linear in px: A (px - ax) > g with A = s dy, g = s dx (py - ay), i.e.
// px > T (A > 0) or px < T (A < 0), T = ax + g / A. Columns run right to left in NDC (tile column
// c of NDC x: c = C0 - x C1), so px > T is c < c(T) and px < T is c > c(T). g is lowered by a
// slack of 2 tol, tol bounding the float rounding of the edge function evaluated in frag_keep
// and of this threshold; a horizontal edge (A = 0) is the limit A -> +0 (all or no columns).
struct TileCols {
  float C0, C1;  // tile column of an NDC x: c = C0 - x * C1
  float omax;    // bound on |NDC| of any pixel centre
};
MR_DEV TileCols tile_cols(int x0, int H, int W) {
  TileCols t;
  t.C1 = W > H ? 0.5f * (float)H : 0.5f * (float)W;
  t.C0 = 0.5f * (float)W - 0.5f - (float)x0;
  t.omax = (float)max(W, H) / (float)min(W, H);
  return t;
}
MR_DEV unsigned long long rect_mask(int rx0, int rx1, int ry0, int ry1) {
  const unsigned long long row = (2ull << rx1) - (1ull << rx0);
  const unsigned long long rows = (0x0101010101010101ull >> (8 * (7 - ry1))) & (~0ull << (8 * ry0));
  return row * rows;
}
MR_DEV unsigned long long tri_mask(const FaceRec& r, const float* ys, int rx0, int rx1, int ry0, int ry1,
                                   const TileCols& tc) {
  const float s = r.area > 0.0f ? 1.0f : -1.0f;
  float Gx[3], K[3], rA[3], ax[3], sC1[3], sC0[3];
  bool up[3];  // A > 0 (or = 0): the edge bounds the columns from above
  const float vx[3] = {r.x0, r.x1, r.x2}, vy[3] = {r.y0, r.y1, r.y2};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int a = (i + 1) % 3, b = (i + 2) % 3;  // E_0 = E(p, v1, v2), E_1 = E(p, v2, v0), E_2 = E(p, v0, v1)
    const float dx = vx[b] - vx[a], dy = vy[b] - vy[a];
    const float A = s * dy;
    const float tol = 1e-6f * (fabsf(dx) + fabsf(dy)) * (tc.omax + fabsf(vx[a]) + fabsf(vy[a]));
    Gx[i] = s * dx;
    K[i] = Gx[i] * vy[a] + 2.0f * tol;  // g - 2 tol = Gx py - K
    up[i] = A >= 0.0f;
    rA[i] = A != 0.0f ? __builtin_amdgcn_rcpf(A) : 1e30f;
    ax[i] = vx[a];
    // sigma c(T) + eps, sigma = +1 (up) / -1: floor of it bounds hi (up) or -lo
    sC1[i] = up[i] ? -tc.C1 : tc.C1;
    sC0[i] = (up[i] ? tc.C0 : -tc.C0) + 0.02f;
  }
  unsigned long long m = 0;
#pragma unroll
  for (int ry = 0; ry < MR_TS; ++ry) {
    if (ry < ry0 || ry > ry1) continue;
    const float py = ys[ry];
    int hi = rx1, lo = rx0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float T = fmaf(fmaf(Gx[i], py, -K[i]), rA[i], ax[i]);
      const float v = __builtin_amdgcn_fmed3f(fmaf(T, sC1[i], sC0[i]), -10.0f, 10.0f);  // NaN -> -10: no column
      const int h = (int)floorf(v);
      if (up[i]) hi = min(hi, h);
      else lo = max(lo, -h);
    }
    if (lo <= hi) m |= ((2ull << hi) - (1ull << lo)) << (8 * ry);
  }
  return m;
}

// The k-th (from 0) set bit of m (k < popcount(m)).
MR_DEV int kth_bit(unsigned long long m, int k) {
  const unsigned lo = (unsigned)m;
  const int clo = __popc(lo);
  const bool hi = k >= clo;
  unsigned x = hi ? (unsigned)(m >> 32) : lo;
  int pos = hi ? 32 : 0;
  k = hi ? k - clo : k;
#pragma unroll
  for (int sh = 16; sh >= 1; sh >>= 1) {
    const int c = __popc(x & ((1u << sh) - 1u));
    const bool go = k >= c;
    x = go ? x >> sh : x;
    k = go ? k - c : k;
    pos = go ? pos + sh : pos;
  }
  return pos;
}

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

#define MR_NONE 0x7fffffff  // "no face" sentinel, larger than any face code

// Sort code of a record id: upstream's clipped packed order puts the two triangles of a split
// face at consecutive ids in place of the face, so the (z, face) tie order is by (face instance,
// triangle): code = 2 * rid (+1 for the second triangle, record NF + rid). Requires NF < 2^30.
MR_DEV unsigned rec_code(int id, int64_t NF) {
  return id < NF ? 2u * (unsigned)id : 2u * (unsigned)(id - NF) + 1u;
}
MR_DEV int code_rec(unsigned code, int64_t NF) {
  return (code & 1u) ? (int)(NF + (code >> 1)) : (int)(code >> 1);
}
// The original face instance (pix_to_face) of a record id.
MR_DEV int rec_orig(int id, int64_t NF) { return id >= NF ? (int)(id - NF) : id; }

// A split face's two triangles at one pixel (upstream clipped_faces_neighbor_idx rule, for the
// pair as one candidate): if both are kept the second replaces the first iff its distance to the
// pixel is smaller than the first's |signed distance|; else whichever is kept. Returns the record
// id and depth of the candidate.
MR_DEV bool pair_keep(const FaceRec* __restrict__ recs, int64_t NF, int id, const FaceRec& r, float x, float y,
                      float pad, float blur, bool persp, bool clipb, int& cid, float& pz);
// The pixels of one lane's tile rectangle for a split face's triangle (k_tile_raster, rare path;
// out of line so that its registers do not weigh on the pixel-pair loop).
MR_DEV void stage_rec_put(float (*rec)[64], int lane, const FaceRec& r) {
  const float* f = (const float*)&r;
#pragma unroll
  for (int i = 0; i < 16; ++i) rec[i][lane] = f[i];
}
MR_DEV FaceRec stage_rec_get(const float (*rec)[64], int m) {
  FaceRec r;
  float* f = (float*)&r;
#pragma unroll
  for (int i = 0; i < 16; ++i) f[i] = rec[i][m];
  return r;
}
__attribute__((noinline)) __device__ void raster_pair_rect(const FaceRec* __restrict__ recs, int64_t NF,
                                                           const float (*srec)[64], const int* sid, const float* xs,
                                                           const float* ys, unsigned long long* key, int lane,
                                                           int prect, float pad, float blur, bool persp, bool clipb);
MR_DEV bool pair_keep(const FaceRec* __restrict__ recs, int64_t NF, int id, const FaceRec& r, float x, float y,
                      float pad, float blur, bool persp, bool clipb, int& cid, float& pz) {
  const bool second = id >= NF;
  const int oid = second ? (int)(id - NF) : (int)(id + NF);
  const FaceRec ro = recs[oid];
  const FaceRec& r1 = second ? ro : r;
  const FaceRec& r2 = second ? r : ro;
  const int id1 = second ? oid : id, id2 = second ? id : oid;
  FragEval e1, e2;
  const bool k1 = (r1.flags & FR_VALID) && eval_face(r1, x, y, pad, blur, persp, clipb, e1);
  const bool k2 = (r2.flags & FR_VALID) && eval_face(r2, x, y, pad, blur, persp, clipb, e2);
  if (k1 && k2) {
    const bool use2 = fabsf(e2.sdist) < fabsf(e1.sdist);
    cid = use2 ? id2 : id1;
    pz = use2 ? e2.pz : e1.pz;
    return true;
  }
  if (k1 || k2) {
    cid = k1 ? id1 : id2;
    pz = k1 ? e1.pz : e2.pz;
    return true;
  }
  return false;
}

// (z, face) packed so that unsigned order == frag_less order on the depths that are ever
// kept (pz >= 0; -0 folds onto +0, which the CPU compares equal). The empty key sorts
// after every kept fragment, +inf depth included.
MR_DEV unsigned long long frag_key(float z, int f) {
  const unsigned zb = z == 0.0f ? 0u : __float_as_uint(z);
  return ((unsigned long long)zb << 32) | (unsigned)f;
}

// Everything the forward kernels read and write (geometry, work lists, outputs).
struct FwdParams {
  int N, H, W, TX, T, K;
  float blur, bbox_pad;
  int persp, clipb;
  const int64_t* view_first;  // NULL: shared mode (overflow units scan faces n*F ..)
  int64_t F;                  // faces per view in shared mode (record id = n*F + face)
  int64_t NF;                 // face instances: the second triangle of a split face is record NF + rid
  const ClipRec* crec;        // conversions of clipped records (flag FR_CLIP)
  const FaceRec* recs;
  const int* list;
  const int4* units;
  const int64_t* view_count;  // modular mode: faces per view (overflow tiles scan them all)
  const int* cnt;             // per-tile entries, start inside the view, view bases (K > 1)
  const int* start;
  const int* vbase;
  int64_t list_cap;
  int mfpb;
  int fill;  // k_tile_raster also writes the background
  int fill_first;  // ... from this chunk on: the chunks before it were written by k_bin_view<MODE, CH>
  int* ctr;
  unsigned long long* tkey;
  int* tdone;
  int* sface;       // (slots, 64) winning face record per tile pixel or -1
  const int* stile; // (slots) view * T + tile
  // MODE 0 outputs (PyTorch3D Fragments, K = 1)
  int64_t* p2f;
  float* zbuf;
  float* bary;
  float* dists;
  // MODE 1 outputs
  ShadeParams S;
  const ShadeRec* srec;
  int out_flags;
  float* depth;
  float* sil;
  float* rgb;
  int32_t* p2f32;  // optional
  float4* frec;    // MODE 1: the winners' fragments for the backward (slot-major, 64 per slot)
};

// One wave's LDS: the batch of up to 64 entries of its unit and the tile's 64 keys (5.4 KB).
// Face records of the unit's entries, structure-of-arrays: field i of entry m at rec[i][m]. The
// pair passes read the records of up to 64 different entries at once; an array of 64-B records
// put entries 4 apart on the same LDS bank (bank conflicts on every record read), the field
// arrays put distinct entries on distinct banks.
struct WaveStage {
  float rec[16][64];
  int id[64];
  int meta[64];  // index of the entry's first candidate pixel
  int mark[64];  // pass-local: candidate slot -> entry lane that starts there
  unsigned long long key[64];
  unsigned long long cmask[64];  // the entry's candidate pixels (bit 8 * row + col)
  float xs[MR_TS], ys[MR_TS];
};

// Background values of every output (view-independent: a pixel without a face has zero
// blend weight, so depth = relu(-1) = 0, silhouette = 0, rgb = background, alpha = 0).
struct Bg {
  float d, s, c[4];
};
template <int MODE>
MR_DEV Bg background(const FwdParams& P) {
  Bg b;
  b.d = b.s = -1.0f;
  b.c[0] = b.c[1] = b.c[2] = b.c[3] = -1.0f;
  if (MODE == 1) {
    PixGeom G;
    ShadeOut o;
    ShadeCache C;
    shade_fwd(P.S, 0, false, G, 0.f, 0.f, 0.f, 0.f, 0.f, o, C);
    b.d = o.depth;
    b.s = o.sil;
    b.c[0] = o.rgb[0]; b.c[1] = o.rgb[1]; b.c[2] = o.rgb[2]; b.c[3] = o.alpha;
  }
  return b;
}

// Background of one 64-lane chunk of view n: 4 pixels per lane and 16-B vector stores when
// W % 4 == 0 (every row then starts 16-B aligned), else one pixel per lane.
template <int MODE, int CH>
MR_DEV void fill_chunk(const FwdParams& P, const Bg& b, int n, int c, bool vec) {
  const int lane = threadIdx.x & 63;
  const int64_t HW = (int64_t)P.H * P.W * (MODE == 0 ? P.K : 1);  // MODE 0: every entry is -1
  if (vec) {
    const int64_t g = (int64_t)c * 64 + lane;
    if (g >= HW / 4) return;
    const int64_t pix = (int64_t)n * HW + 4 * g;
    if (MODE == 0) {
      const float4 m1 = make_float4(-1.f, -1.f, -1.f, -1.f);
      longlong2* q = (longlong2*)(P.p2f + pix);
      q[0] = make_longlong2(-1ll, -1ll);
      q[1] = make_longlong2(-1ll, -1ll);
      *(float4*)(P.zbuf + pix) = m1;
      *(float4*)(P.dists + pix) = m1;
      float4* q3 = (float4*)(P.bary + pix * 3);
      q3[0] = m1; q3[1] = m1; q3[2] = m1;
    } else {
      if (P.out_flags & MR_OUT_DEPTH) *(float4*)(P.depth + pix) = make_float4(b.d, b.d, b.d, b.d);
      if (P.out_flags & MR_OUT_SIL) {
        if (P.out_flags & MR_OUT_SIL_RGBA) {
          float4* q = (float4*)(P.sil + pix * 4);
          const float4 v = make_float4(1.0f, 1.0f, 1.0f, b.s);
          q[0] = v; q[1] = v; q[2] = v; q[3] = v;
        } else {
          *(float4*)(P.sil + pix) = make_float4(b.s, b.s, b.s, b.s);
        }
      }
      if (P.p2f32) *(int4*)(P.p2f32 + pix) = make_int4(-1, -1, -1, -1);
      if (P.out_flags & MR_OUT_RGB) {
        float4* q = (float4*)(P.rgb + pix * CH);
        if (CH == 4) {
          const float4 v = make_float4(b.c[0], b.c[1], b.c[2], b.c[3]);
          q[0] = v; q[1] = v; q[2] = v; q[3] = v;
        } else {
          // 4 pixels x 3 channels = 3 aligned 16-B stores. Opaque copies keep the compiler from
          // re-splitting the period-3 pattern into four unaligned 12-B stores.
          float r0 = b.c[0], g0 = b.c[1], b0 = b.c[2], r1 = r0, g1 = g0, b1 = b0, r2 = r0, g2 = g0, b2 = b0;
          asm volatile("" : "+v"(r1), "+v"(g1), "+v"(b1), "+v"(r2), "+v"(g2), "+v"(b2));
          q[0] = make_float4(r0, g0, b0, r1);
          q[1] = make_float4(g1, b1, r2, g2);
          q[2] = make_float4(b2, r0, g0, b0);
        }
      }
    }
  } else {
    const int64_t i = (int64_t)c * 64 + lane;
    if (i >= HW) return;
    const int64_t q = (int64_t)n * HW + i;
    if (MODE == 0) {
      P.p2f[q] = -1ll;
      P.zbuf[q] = -1.0f;
      P.dists[q] = -1.0f;
      for (int k = 0; k < 3; ++k) P.bary[q * 3 + k] = -1.0f;
    } else {
      if (P.out_flags & MR_OUT_DEPTH) P.depth[q] = b.d;
      if (P.out_flags & MR_OUT_SIL) {
        if (P.out_flags & MR_OUT_SIL_RGBA) *(float4*)(P.sil + q * 4) = make_float4(1.0f, 1.0f, 1.0f, b.s);
        else P.sil[q] = b.s;
      }
      if (P.p2f32) P.p2f32[q] = -1;
      if (P.out_flags & MR_OUT_RGB)
        for (int k = 0; k < CH; ++k) P.rgb[q * CH + k] = b.c[k];
    }
  }
}

// Persistent grid of independent waves (4 per workgroup, no workgroup barriers): wave g
// takes units g, g + G, ... of the list k_bin_scan emitted (G = resident waves). Per unit:
//  (1) one entry per lane: load its face record, clip the face's padded pixel bbox to the
//      tile (<= 64 pixels);
//  (2) a DPP prefix sum over the rectangle sizes numbers the (face, pixel) pairs, and the
//      wave evaluates 64 pairs per pass exactly (frag_keep), one per lane — a ~3-pixel
//      face costs ~3 lanes, not a wave;
//  (3) kept fragments meet in a per-pixel ds_min_u64 on the packed (z, face) key, which is
//      order-independent and equals the CPU's "strictly nearer, earlier face wins";
//  (4) a tile that is a single unit writes its 64 winners (face record or -1) to its slot
//      of sface straight from LDS; units sharing a tile merge their keys with global u64
//      atomicMin, and the last of them to finish (an atomic count-down) reads the merged
//      keys back with returning atomics and writes the slot.
// The background of every pixel (k_shade later overwrites the covered ones) is written by
// the same waves, a share of 64-lane chunks after each unit: the stores stream to HBM while
// the raster work, which is latency-bound, leaves it idle. (Measured: a separate fill kernel
// on a forked stream overlapping binning was slower in the graph-replayed step, and the
// raster's time barely drops without the fill.) k_fill is the stand-alone version, used
// before k_raster_k (K > 1).
template <int MODE, int CH>
__global__ void __launch_bounds__(256) k_fill(FwdParams P) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), G = gridDim.x * 4;
  const bool vec = (P.W & 3) == 0;
  const int64_t HW = (int64_t)P.H * P.W * (MODE == 0 ? P.K : 1);
  const int cpv = (int)(vec ? (HW / 4 + 63) / 64 : (HW + 63) / 64);
  const int nchunks = P.N * cpv;
  const Bg bg = background<MODE>(P);
#pragma unroll 1
  for (int c = gw; c < nchunks; c += G) fill_chunk<MODE, CH>(P, bg, c / cpv, c - (c / cpv) * cpv, vec);
}


// The per-view binning with background workgroups: one 1024-thread workgroup per view leaves
// most CUs idle, so workgroups past the views (and the ShadeRec ones) stream the background of
// the first F.fill_first chunks (view-major) while the views bin; k_tile_raster writes the rest.
// The background does not depend on the raster (k_shade overwrites the covered pixels later).
template <int MODE, int CH>
__global__ void __launch_bounds__(1024) k_bin_view(ViewBinParams P, FwdParams F) {
  const int b = (int)blockIdx.x - P.nviews - P.nsrec_wg;
  if (b < 0) {
    bin_view_body(P);
    return;
  }
  const int nbw = ((int)gridDim.x - P.nviews - P.nsrec_wg) * 16;  // background waves
  const bool vec = (F.W & 3) == 0;
  const int64_t HW = (int64_t)F.H * F.W * (MODE == 0 ? F.K : 1);
  const int cpv = (int)(vec ? (HW / 4 + 63) / 64 : (HW + 63) / 64);
  const Bg bg = background<MODE>(F);
#pragma unroll 1
  for (int c = b * 16 + (int)(threadIdx.x >> 6); c < F.fill_first; c += nbw)
    fill_chunk<MODE, CH>(F, bg, c / cpv, c - (c / cpv) * cpv, vec);
}

__attribute__((noinline)) __device__ void raster_pair_rect(const FaceRec* __restrict__ recs, int64_t NF,
                                                           const float (*srec)[64], const int* sid, const float* xs,
                                                           const float* ys, unsigned long long* key, int lane,
                                                           int prect, float pad, float blur, bool persp, bool clipb) {
  const FaceRec r = stage_rec_get(srec, lane);
  const int id = sid[lane];
  for (int yy = (prect >> 6) & 7; yy <= ((prect >> 9) & 7); ++yy)
    for (int xx = prect & 7; xx <= ((prect >> 3) & 7); ++xx) {
      float pz;
      int cid;
      if (pair_keep(recs, NF, id, r, xs[xx], ys[yy], pad, blur, persp, clipb, cid, pz))
        atomicMin(&key[yy * MR_TS + xx], frag_key(pz, (int)rec_code(cid, NF)));
    }
}

// CLIP: near-plane clipping on (split faces may be present); the CLIP = false instantiation
// carries none of their code, so the common launch keeps its register budget.
#ifndef MR_RASTER_WAVES
#define MR_RASTER_WAVES 4  // waves / SIMD: 5 -> <= 96 VGPRs, 4 -> <= 128
#endif
template <int MODE, int CH, bool CLIP>
__global__ void __launch_bounds__(256, MR_RASTER_WAVES) k_tile_raster(FwdParams P) {
  __shared__ WaveStage stage[4];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  WaveStage& S = stage[wave];
  const int nunits = P.ctr[CTR_UNITS];
  const float pad = P.bbox_pad, blur = P.blur;
  const bool persp = P.persp != 0, clipb = P.clipb != 0;
  const bool fast_ok = !(blur > 0.0f);
  const int H = P.H, W = P.W;
  // background chunks of this wave: c = gw, gw + G, ... < N * cpv, written after its units (the
  // waves that finish their raster work early stream the background while the others still run;
  // chunks interleaved with the units measured 3 us slower, all chunks before them 20 us slower)
  const int gw = blockIdx.x * 4 + wave, G = gridDim.x * 4;
  const bool vec = (W & 3) == 0;
  const int64_t HW = (int64_t)H * W * (MODE == 0 ? P.K : 1);
  const int cpv = (int)(vec ? (HW / 4 + 63) / 64 : (HW + 63) / 64);
  const int nchunks = P.fill ? P.N * cpv : 0;
  // XCD-aware unit partition: workgroups are dispatched round-robin over the 8 XCDs, so
  // blockIdx % 8 names this wave's XCD; each XCD's waves take a contiguous eighth of the
  // (view-major) units, which keeps the face records they gather in that XCD's L2.
  const int parts = (gridDim.x & 7) == 0 ? 8 : 1;
  const int jw = (blockIdx.x / parts) * 4 + wave, Gp = (gridDim.x / parts) * 4;
  const int Cp = (nunits + parts - 1) / parts;
  const int ub = (blockIdx.x % parts) * Cp, ue = ub + Cp < nunits ? ub + Cp : nunits;
  const Bg bg = background<MODE>(P);
  int chunk = P.fill_first + gw;
  // Software pipeline over the wave's units u, u + Gp, u + 2Gp, ...: while unit u is
  // rasterised, the face records of u + Gp, the list entries of u + 2Gp and the unit record of
  // u + 3Gp are in flight (unit records are wave-uniform scalar loads). Each link of the
  // unit -> list entry -> record chain so gets a whole unit of work to land in, and a unit
  // starts with its records in registers. (Overflow units fetch their records in the batch.)
  // The prefetches are unconditional loads of clamped (valid) indices whose results are only
  // used when the unit / entry exists (guarded loads become branches whose phi copies wait on
  // the load at once), and the unit records travel as per-lane copies made uniform where they
  // are consumed (a uniform load is otherwise scalarised: load + readfirstlane + wait at issue).
  const int lz = lane_zero();
  const int ulast = max(ue - 1, 0);
  int4 U1v = P.units[min(ub + jw, ulast) + lz];
  int4 U2v = P.units[min(ub + jw + Gp, ulast) + lz];
  int4 U3v = P.units[min(ub + jw + 2 * Gp, ulast) + lz];
  int id1 = P.list[(ub + jw < ue && U1v.y >= 0 && lane < U1v.z) ? U1v.y + lane : 0];
  int id2 = P.list[(ub + jw + Gp < ue && U2v.y >= 0 && lane < U2v.z) ? U2v.y + lane : 0];
  FaceRec r1 = load_rec(P.recs, (ub + jw < ue && U1v.y >= 0 && lane < U1v.z) ? id1 : 0);
#pragma unroll 1
  for (int u = ub + jw; u < ue; u += Gp) {
    const int4 U = make_int4(__builtin_amdgcn_readfirstlane(U1v.x), __builtin_amdgcn_readfirstlane(U1v.y),
                             __builtin_amdgcn_readfirstlane(U1v.z), __builtin_amdgcn_readfirstlane(U1v.w));
    const int id0 = id1;
    const int n = U.x / P.T, t = U.x - n * P.T;
    const int ty = t / P.TX, tx = t - ty * P.TX;
    const int x0 = tx * MR_TS, y0 = ty * MR_TS;
    const TileCols tc = tile_cols(x0, H, W);
    if (lane < MR_TS) S.xs[lane] = col_ndc(x0 + lane < W ? x0 + lane : W - 1, H, W);
    else if (lane < 2 * MR_TS) S.ys[lane - MR_TS] = row_ndc(y0 + lane - MR_TS < H ? y0 + lane - MR_TS : H - 1, H, W);
    S.key[lane] = MR_KEY_EMPTY;
    S.mark[lane] = -1;
    const bool ovf = U.y < 0;
    wave_lds_sync();
#pragma unroll 1
    for (int eb = 0; eb < U.z; eb += 64) {
      const int e = eb + lane;
      int prect = 0;
      unsigned long long cmask = 0;
      if (e < U.z) {
        int id;
        FaceRec r;
        if (ovf) {  // (the view's first record loaded here: a load hoisted to the unit's start is waited on there)
          const int64_t vfirst = P.view_first ? P.view_first[n] : (int64_t)n * P.F;
          id = (int)(vfirst + e);
          r = P.recs[id];
        } else {  // a listed unit has <= 64 entries: its records are already here
          id = id0;
          r = r1;
        }
        // pixel rectangle: the record's padded bbox; an overflow unit scans only first triangles
        // of split faces, so there it covers both triangles of the pair
        float bx0 = r.xmin, bx1 = r.xmax, by0 = r.ymin, by1 = r.ymax;
        bool bvalid = (r.flags & FR_VALID) != 0;
        if (CLIP && ovf && (r.flags & FR_PAIR)) {
          const FaceRec ro = P.recs[P.NF + id];
          if (ro.flags & FR_VALID) {
            bx0 = bvalid ? smin(bx0, ro.xmin) : ro.xmin;
            bx1 = bvalid ? smax(bx1, ro.xmax) : ro.xmax;
            by0 = bvalid ? smin(by0, ro.ymin) : ro.ymin;
            by1 = bvalid ? smax(by1, ro.ymax) : ro.ymax;
            bvalid = true;
          }
        }
        int cx0, cx1, cy0, cy1;
        ndc_range_to_pix(bx0 - pad, bx1 + pad, W, H, cx0, cx1);
        ndc_range_to_pix(by0 - pad, by1 + pad, H, W, cy0, cy1);
        cx0 = cx0 > x0 ? cx0 : x0;
        cx1 = cx1 < x0 + MR_TS - 1 ? cx1 : x0 + MR_TS - 1;
        cy0 = cy0 > y0 ? cy0 : y0;
        cy1 = cy1 < y0 + MR_TS - 1 ? cy1 : y0 + MR_TS - 1;
        if (bvalid && cx0 <= cx1 && cy0 <= cy1) {
          if (CLIP && (r.flags & FR_PAIR)) {  // a split face's triangle: its own per-lane loop after the passes
            prect = 0x1000 | (cx0 - x0) | ((cx1 - x0) << 3) | ((cy0 - y0) << 6) | ((cy1 - y0) << 9);
          } else {
            const int rx0 = cx0 - x0, rx1 = cx1 - x0, ry0 = cy0 - y0, ry1 = cy1 - y0;
            // coverage rows from the edges (fast path; coordinates small enough that the
            // threshold arithmetic stays finite), else the whole rectangle
            const bool tm = fast_ok && (r.flags & FR_FAST) &&
                            fmaxf(fmaxf(fabsf(r.xmin), fabsf(r.xmax)), fmaxf(fabsf(r.ymin), fabsf(r.ymax))) < 1e12f;
            cmask = tm ? tri_mask(r, S.ys, rx0, rx1, ry0, ry1, tc) : rect_mask(rx0, rx1, ry0, ry1);
          }
        }
        stage_rec_put(S.rec, lane, r);
        S.id[lane] = id;
      }
      if (eb == 0) {  // advance the pipeline (after this unit's records are consumed)
        r1 = load_rec(P.recs, (u + Gp < ue && U2v.y >= 0 && lane < U2v.z) ? id2 : 0);
        id1 = id2;
        U1v = U2v;
        id2 = P.list[(u + 2 * Gp < ue && U3v.y >= 0 && lane < U3v.z) ? U3v.y + lane : 0];
        U2v = U3v;
        U3v = P.units[min(u + 3 * Gp, ulast) + lz];
      }
      // candidate numbering: a DPP prefix sum over the masks' popcounts
      const int np = __popcll(cmask);
      const int pincl = wave_incl_sum(np);
      const int pexcl = pincl - np;
      const int NP = __builtin_amdgcn_readlane(pincl, 63);
      S.meta[lane] = pexcl;
      S.cmask[lane] = cmask;
      // 64 candidates per pass, one per lane, each evaluated exactly (frag_keep: bbox, edge
      // signs, divisions, perspective correction, depth) and merged into the tile's keys
#pragma unroll 1
      for (int pb = 0; pb < NP; pb += 64) {
        wave_lds_sync();
        // the entry starting inside this pass marks its first slot; slot 0 belongs to the
        // entry straddling pb (the last non-empty entry starting at or before it)
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
          const int p = kth_bit(S.cmask[m], q - S.meta[m]);
          const int sx = p & 7, sy = p >> 3;
          const FaceRec r = stage_rec_get(S.rec, m);
          float pz;
          if (frag_keep(r, S.xs[sx], S.ys[sy], pad, blur, persp, clipb, fast_ok && (r.flags & FR_FAST), pz))
            atomicMin(&S.key[p], frag_key(pz, CLIP ? (int)rec_code(S.id[m], P.NF) : 2 * S.id[m]));
        }
      }
      if (CLIP && __builtin_expect(__ballot(prect != 0) != 0ull, 0)) {
        // near-plane split faces (rare): each such lane walks its rectangle, resolving the pair
        if (prect) raster_pair_rect(P.recs, P.NF, S.rec, S.id, S.xs, S.ys, S.key, lane, prect, pad, blur, persp, clipb);
      }
      wave_lds_sync();  // the stage is rewritten by the next batch
    }
    unsigned long long k = S.key[lane];
    const int slot = U.w & 0x7fffffff;
    bool emit = true;
    if (U.w < 0) {  // tile shared by several units
      unsigned long long* dst = P.tkey + (int64_t)slot * 64 + lane;
      // Device-scope atomics are performed at the memory side (never cached in an XCD's L2),
      // so agent atomics on both sides hand the keys over: this wave's 64 atomicMin are
      // acknowledged (vmcnt) before its count-down, and the last unit reads the merged keys
      // with returning atomics issued after it observed the count-down reach it.
      atomicMin(dst, k);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int left = 0;
      if (lane == 0) left = __hip_atomic_fetch_add(&P.tdone[slot], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      left = __builtin_amdgcn_readfirstlane(left);
      emit = left == 0;  // the last unit of the tile
      if (emit) k = atomicMin(dst, MR_KEY_EMPTY);
    }
    if (emit) {
      const unsigned code = (unsigned)(k & 0xffffffffull);
      const int px = x0 + (lane & 7), py = y0 + (lane >> 3);
      const bool hit = code != MR_NONE && px < W && py < H;
      P.sface[(int64_t)slot * 64 + lane] = hit ? (CLIP ? code_rec(code, P.NF) : (int)(code >> 1)) : -1;
    }
    wave_lds_sync();
  }
#pragma unroll 1
  for (; chunk < nchunks; chunk += G) fill_chunk<MODE, CH>(P, bg, chunk / cpv, chunk - (chunk / cpv) * cpv, vec);
}

// Per-face shading records of the shared mesh (one thread per face).
__global__ void __launch_bounds__(256) k_shade_rec(ShadeParams S, int64_t F, ShadeRec* __restrict__ out) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  ShadeRec R;
  make_shade_rec(S, (uint32_t)f, R);
  out[f] = R;
}

MR_DEV void vertex_normal(const float* __restrict__ verts, const int32_t* __restrict__ faces,
                          const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj, int64_t v,
                          float* __restrict__ vn, float* __restrict__ vraw);

// The fused forward's first kernel: blocks [0, vb) compute the vertex normals (one thread per
// vertex, as k_vertex_normals; vb = 0 when the caller passed them), the rest zero `nzero` ints
// (per-tile counts, view totals, work counters) with coalesced stores — one launch instead of a
// normals launch + a memset. The ShadeRecs, which need the normals, are packed by extra blocks
// of the binning fill launch (k_bin_fill_world row N).
__global__ void __launch_bounds__(256) k_setup_zero(const float* __restrict__ verts, int64_t V,
                                                    const int32_t* __restrict__ faces, const int32_t* __restrict__ ptr,
                                                    const int32_t* __restrict__ adj, float* __restrict__ vn,
                                                    float* __restrict__ vraw, int64_t vb, int* __restrict__ zero,
                                                    int64_t nzero) {
  if ((int64_t)blockIdx.x < vb) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V) vertex_normal(verts, faces, ptr, adj, v, vn, vraw);
    return;
  }
  const int64_t base = ((int64_t)blockIdx.x - vb) * 1024;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    if (i < nzero) zero[i] = 0;
  }
}

// XCD-aware slot ranges: workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8
// names the XCD), so each XCD takes a contiguous eighth of the (view-major, tile-ordered) slots
// and its waves stride inside it. Horizontally / vertically adjacent tiles then run on the same
// XCD at about the same time and share that XCD's L2 lines (the 128-B lines of the per-pixel
// upstream gradients and outputs span two 8-pixel tile rows; a face record serves neighbouring
// tiles). Returns the wave's first slot, its stride and the range end.
MR_DEV void xcd_slot_range(int nslots, int wave, int& s0, int& step, int& end) {
  const int parts = (gridDim.x & 7) == 0 ? 8 : 1;
  const int per = (nslots + parts - 1) / parts;
  const int x = blockIdx.x % parts;
  const int b = x * per;
  end = b + per < nslots ? b + per : nslots;
  s0 = b + (int)(blockIdx.x / parts) * 4 + wave;
  step = (int)(gridDim.x / parts) * 4;
}

// Covered pixels: waves stride over the non-empty tiles' slots, one tile pixel per lane:
// recompute the winning fragment exactly, then write PyTorch3D fragments (M = 0) or shade
// (M = 1) over the background k_tile_raster wrote.
template <int MODE, int CH>
__global__ void __launch_bounds__(256) k_shade(FwdParams P) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nslots = P.ctr[CTR_SLOTS];
  const int64_t HW = (int64_t)P.H * P.W;
  int s0, G, send;
  xcd_slot_range(nslots, wave, s0, G, send);
  // Two-deep pipeline: while slot s is processed, the winners' face records of slot s + G and
  // the tile and winners of slot s + 2G are in flight (unconditional loads of clamped indices;
  // the tile id as a per-lane copy made uniform at use — see k_bwd_fused).
  const int lz = lane_zero();
  const int slast = max(nslots - 1, 0);
  int sc = min(s0, slast);
  int gt_c = P.stile[sc + lz], f_c = P.sface[(int64_t)sc * 64 + lane];
  sc = min(s0 + G, slast);
  int gt_n = P.stile[sc + lz], f_n = P.sface[(int64_t)sc * 64 + lane];
  FaceRec r_c = load_rec(P.recs, f_c < 0 ? 0 : f_c);
  for (int s = s0; s < send; s += G) {
    const int gt = __builtin_amdgcn_readfirstlane(gt_c);
    const int f = f_c;
    const FaceRec r = r_c;
    gt_c = gt_n;
    f_c = f_n;
    r_c = load_rec(P.recs, f_c < 0 ? 0 : f_c);
    sc = min(s + 2 * G, slast);
    gt_n = P.stile[sc + lz];
    f_n = P.sface[(int64_t)sc * 64 + lane];
    if (f < 0) continue;
    const int n = gt / P.T, t = gt - n * P.T;
    const int ty = t / P.TX, tx = t - ty * P.TX;
    const int px = tx * MR_TS + (lane & 7), py = ty * MR_TS + (lane >> 3);
    const int64_t q = n * HW + (int64_t)py * P.W + px;
    const int fo = rec_orig(f, P.NF);  // the original face instance
    PixGeom G;
    if (MODE == 1) load_geom(P.srec, (uint32_t)(fo - n * P.F), G);  // in parallel with the record
    FragEval ev;
    const bool hit = eval_face(r, col_ndc(px, P.H, P.W), row_ndc(py, P.H, P.W), P.bbox_pad, P.blur, P.persp,
                               P.clipb, ev);  // true by construction (same test that kept it)
    if (!hit) continue;
    if (r.flags & FR_CLIP) {  // near-plane sub-triangle: barycentrics of the original face
      const ClipRec cr = P.crec[f];
      clip_unconvert(cr, ev.b0, ev.b1, ev.b2, ev.b0, ev.b1, ev.b2);
    }
    if (MODE == 0) {
      P.p2f[q] = (int64_t)fo;
      P.zbuf[q] = ev.pz;
      P.dists[q] = ev.sdist;
      P.bary[3 * q + 0] = ev.b0;
      P.bary[3 * q + 1] = ev.b1;
      P.bary[3 * q + 2] = ev.b2;
    } else {
      // the fragment the backward shades again (its barycentrics must be these bits: they pick the
      // texel cell), so k_bwd_fused does not re-run eval_face's IEEE divisions
      P.frec[(int64_t)s * 64 + lane] = make_float4(ev.b0, ev.b1, ev.b2, ev.sdist);
      ShadeOut o;
      ShadeCache C;
      shade_fwd(P.S, n, true, G, ev.b0, ev.b1, ev.b2, ev.pz, ev.sdist, o, C);
      if (P.out_flags & MR_OUT_DEPTH) P.depth[q] = o.depth;
      if (P.out_flags & MR_OUT_SIL) {
        if (P.out_flags & MR_OUT_SIL_RGBA) *(float4*)(P.sil + q * 4) = make_float4(1.0f, 1.0f, 1.0f, o.sil);
        else P.sil[q] = o.sil;
      }
      if (P.out_flags & MR_OUT_RGB) {
        P.rgb[q * CH + 0] = o.rgb[0];
        P.rgb[q * CH + 1] = o.rgb[1];
        P.rgb[q * CH + 2] = o.rgb[2];
        if (CH == 4) P.rgb[q * CH + 3] = o.alpha;
      }
      if (P.p2f32) P.p2f32[q] = fo;
    }
  }
}

// Resident workgroups of a kernel on the current device (persistent grid size).
template <typename K>
static int resident_grid(K kernel, int threads, int fallback_per_cu) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0) != hipSuccess || per <= 0)
    per = fallback_per_cu;
  return cus * per;
}

// Static forward parameters from the settings; the workspace pointers from the carve.
static FwdParams make_fwd(const mr_raster_settings_t* s, const BinGeom& g, const RasterWS& w, int64_t N,
                          const int64_t* view_first, int64_t F, int64_t NF) {
  FwdParams P;
  memset(&P, 0, sizeof(P));
  P.N = (int)N; P.H = s->H; P.W = s->W; P.TX = g.TX; P.T = g.T; P.K = s->faces_per_pixel;
  P.blur = s->blur_radius;
  P.bbox_pad = sqrtf(s->blur_radius);
  P.persp = s->perspective_correct;
  P.clipb = s->clip_barycentric_coords;
  P.view_first = view_first; P.F = F; P.NF = NF; P.crec = w.crec;
  P.recs = w.recs; P.list = w.list; P.units = w.units; P.ctr = w.ctr; P.tkey = w.tkey;
  P.cnt = w.cnt; P.start = w.start; P.vbase = w.vbase; P.list_cap = g.list_cap; P.mfpb = g.mfpb;
  P.tdone = w.tdone; P.sface = w.sface; P.stile = w.stile;
  P.frec = w.frec;
  return P;
}

// K > 1 (modular path, PyTorch3D faces_per_pixel): one wave per non-empty tile, one pixel per
// lane. The tile's faces are staged 64 at a time in the wave's LDS (one record per lane, then
// read as broadcasts) and each lane keeps the K smallest packed (z, face) keys of its pixel in
// an ascending per-lane LDS list (insertion; lane-strided so the 64 lanes hit 64 banks). The
// K smallest keys are exactly the CPU's K nearest with the earlier face winning depth ties,
// already in output order (RasterizeMeshesNaiveCpu keeps the K smallest, then sorts).
// LDS per wave: K * 512 B of keys + 4.25 KB of staged records.
#define MR_KMAX 128
MR_DEV size_t rk_wave_bytes(int K) { return (size_t)K * 64 * 8 + 64 * sizeof(FaceRec) + 64 * sizeof(int); }
__global__ void __launch_bounds__(256) k_raster_k(FwdParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char rk_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wpg = blockDim.x >> 6;
  const int K = P.K;
  unsigned char* base = rk_lds + (size_t)wave * rk_wave_bytes(K);
  unsigned long long* q = (unsigned long long*)base + lane;  // q[k * 64]
  FaceRec* rs = (FaceRec*)(base + (size_t)K * 64 * 8);
  int* ids = (int*)(rs + 64);
  const int nslots = P.ctr[CTR_SLOTS];
  const float pad = P.bbox_pad, blur = P.blur;
  const bool persp = P.persp != 0, clipb = P.clipb != 0;
  const bool fast_ok = !(blur > 0.0f);
  const int H = P.H, W = P.W;
  const int64_t HW = (int64_t)H * W;
#pragma unroll 1
  for (int s = blockIdx.x * wpg + wave; s < nslots; s += gridDim.x * wpg) {
    const int gt = P.stile[s];
    const int n = gt / P.T, t = gt - n * P.T;
    const int ty = t / P.TX, tx = t - ty * P.TX;
    const int px = tx * MR_TS + (lane & 7), py = ty * MR_TS + (lane >> 3);
    const bool in_img = px < W && py < H;
    const float xf = col_ndc(in_img ? px : 0, H, W), yf = row_ndc(in_img ? py : 0, H, W);
    const int cc = P.cnt[gt], ex = P.start[gt];
    const int64_t vb = P.vbase[n];
    // the scan's overflow rule: scan the whole view
    const bool ovf = vb + ex + cc > P.list_cap || (P.mfpb > 0 && cc > P.mfpb);
    const int64_t vfirst = P.view_first ? P.view_first[n] : (int64_t)n * P.F;
    const int64_t vcnt = P.view_count ? P.view_count[n] : P.F;
    const int count = ovf ? (int)(vcnt < 0x7fffffffll ? vcnt : 0x7fffffffll) : cc;
    int nq = 0;
#pragma unroll 1
    for (int eb = 0; eb < count; eb += 64) {
      const int e = eb + lane;
      if (e < count) {
        const int id = ovf ? (int)(vfirst + e) : P.list[vb + ex + e];
        rs[lane] = P.recs[id];
        ids[lane] = id;
      }
      wave_lds_sync();
      const int m = count - eb < 64 ? count - eb : 64;
#pragma unroll 1
      for (int j = 0; j < m; ++j) {
        const FaceRec r = rs[j];
        const int id = ids[j];
        float pz;
        int cid = id;
        bool keep = false;
        if (in_img && (r.flags & FR_PAIR)) {
          // a split face: the pair's candidate is inserted from its own entry (both entries are
          // listed for every pixel either can keep), or from the first triangle's entry when an
          // overflow unit scans the view's records (second triangles are not scanned there)
          keep = pair_keep(P.recs, P.NF, id, r, xf, yf, pad, blur, persp, clipb, cid, pz) &&
                 (cid == id || (ovf && id < P.NF));
        } else if (in_img && (r.flags & FR_VALID)) {
          keep = frag_keep(r, xf, yf, pad, blur, persp, clipb, fast_ok && (r.flags & FR_FAST), pz);
        }
        if (keep) {
          const unsigned long long key = frag_key(pz, (int)rec_code(cid, P.NF));
          if (key < MR_KEY_EMPTY && (nq < K || key < q[(nq - 1) * 64])) {
            int i = nq < K ? nq : K - 1;
            while (i > 0 && q[(i - 1) * 64] > key) {
              q[i * 64] = q[(i - 1) * 64];
              --i;
            }
            q[i * 64] = key;
            nq += nq < K ? 1 : 0;
          }
        }
      }
      wave_lds_sync();
    }
    if (!in_img) continue;
    const int64_t pix = (n * HW + (int64_t)py * W + px) * K;
#pragma unroll 1
    for (int k = 0; k < K; ++k) {
      int64_t f = -1;
      float z = -1.0f, d = -1.0f, b0 = -1.0f, b1 = -1.0f, b2 = -1.0f;
      if (k < nq) {
        const int id = code_rec((unsigned)(q[k * 64] & 0xffffffffull), P.NF);
        const FaceRec r = P.recs[id];
        FragEval ev;
        eval_face(r, xf, yf, pad, blur, persp, clipb, ev);  // kept by construction
        if (r.flags & FR_CLIP) clip_unconvert(P.crec[id], ev.b0, ev.b1, ev.b2, ev.b0, ev.b1, ev.b2);
        f = rec_orig(id, P.NF); z = ev.pz; d = ev.sdist; b0 = ev.b0; b1 = ev.b1; b2 = ev.b2;
      }
      P.p2f[pix + k] = f;
      P.zbuf[pix + k] = z;
      P.dists[pix + k] = d;
      P.bary[3 * (pix + k) + 0] = b0;
      P.bary[3 * (pix + k) + 1] = b1;
      P.bary[3 * (pix + k) + 2] = b2;
    }
  }
}

// K <= 64 (PyTorch3D faces_per_pixel > 1): one wave per non-empty tile, each lane keeping its pixel's
// K nearest (z, face) keys in REGISTERS (KP >= K slots, ascending; a shift-insert whose KP steps are
// independent selects, shifted out through slot 0 so the array is never dynamically indexed). The
// keys are evaluated over (face, pixel) PAIRS: as in k_tile_raster, each lane clips one list entry's
// padded bbox to the tile, a DPP prefix numbers the pairs and a pass evaluates 64 of them exactly
// (frag_keep / pair_keep, one per lane) — with blur a face of the deform workload covers ~a quarter
// of the tile, and evaluating every listed face at all 64 pixels (the previous kernel) ran 4x the
// exact tests. A kept candidate goes to its PIXEL's LDS bucket; the buckets drain into the register
// lists when the fullest has less than MR_KP_ROOM slots left and at the end of the tile, so a list
// takes one insert per candidate of its pixel (~4 of K = 50 on the deform workload), not one per
// listed face, and a drain whose lists will all hold <= 8 / 16 / 32 keys runs that many shift steps
// instead of KP. A pass is limited to the entries whose candidates the buckets can still take (an
// entry adds at most one candidate per pixel). The K nearest keys do not depend on the insertion
// order: the fragments are bitwise those of the face-at-a-time kernel (deform workload: 2.22 ms
// (two waves per tile, every face at every pixel) -> see DESIGN.md for this kernel's numbers).
#ifndef MR_KP_BC
#define MR_KP_BC 32
#endif
// Shift-insert of key into the first NS positions of the ascending list q (positions >= NS are
// empty for every lane of the wave and stay so: no lane holds more than NS keys).
template <int KP, int NS>
MR_DEV void insert_ns(unsigned long long (&q)[KP], unsigned long long key) {
  if (__ballot(key < q[NS - 1]) != 0ull) {
    bool ltk = key < q[NS - 1];
#pragma unroll
    for (int k = NS - 1; k > 0; --k) {
      const bool ltp = key < q[k - 1];
      q[k] = ltk ? (ltp ? q[k - 1] : key) : q[k];
      ltk = ltp;
    }
    q[0] = ltk ? key : q[0];
  }
}

#ifndef MR_KP_ROOM
#define MR_KP_ROOM 16  // drain the buckets once the fullest one has less room than this
#endif
struct KpStage {
  float rec[16][64];
  int id[64];
  int meta[64];
  int mark[64];
  int bcnt[64];
  unsigned long long cmask[64];
  unsigned long long bucket[MR_KP_BC][64];
};
template <int KP>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_raster_kp(FwdParams P) {
  __shared__ KpStage S;
  const int lane = threadIdx.x;
  const int s = blockIdx.x;
  if (s >= P.ctr[CTR_SLOTS]) return;
  const int K = P.K;
  const float pad = P.bbox_pad, blur = P.blur;
  const bool persp = P.persp != 0, clipb = P.clipb != 0;
  const bool fast_ok = !(blur > 0.0f);
  const int H = P.H, W = P.W;
  const int64_t HW = (int64_t)H * W;
  const int gt = P.stile[s];
  const int n = gt / P.T, t = gt - n * P.T;
  const int ty = t / P.TX, tx = t - ty * P.TX;
  const int x0 = tx * MR_TS, y0 = ty * MR_TS;
  const int px = x0 + (lane & 7), py = y0 + (lane >> 3);
  const bool in_img = px < W && py < H;
  const int cc = P.cnt[gt], ex = P.start[gt];
  const int64_t vb = P.vbase[n];
  const bool ovf = vb + ex + cc > P.list_cap || (P.mfpb > 0 && cc > P.mfpb);
  const int64_t vfirst = P.view_first ? P.view_first[n] : (int64_t)n * P.F;
  const int64_t vcnt = P.view_count ? P.view_count[n] : P.F;
  const int count = ovf ? (int)(vcnt < 0x7fffffffll ? vcnt : 0x7fffffffll) : cc;
  const int xe = min(x0 + MR_TS, W) - 1, ye = min(y0 + MR_TS, H) - 1;  // the tile's last pixels inside the image
  unsigned long long q[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) q[k] = MR_KEY_EMPTY;
  auto insert = [&](unsigned long long key) {
    if (__ballot(key < q[KP - 1]) != 0ull) {
      bool ltk = key < q[KP - 1];
#pragma unroll
      for (int k = KP - 1; k > 0; --k) {
        const bool ltp = key < q[k - 1];
        q[k] = ltk ? (ltp ? q[k - 1] : key) : q[k];
        ltk = ltp;
      }
      q[0] = ltk ? key : q[0];
    }
  };
  S.bcnt[lane] = 0;
  S.mark[lane] = -1;
  int mb = 0;  // the fullest bucket's fill (uniform)
  int lc = 0;  // keys in this lane's list
  // Drain: every bucket's keys into its lane's list. The lists' fill after the drain is known before
  // it (all keys are distinct, so none is dropped until a list holds KP): when no lane will hold more
  // than NS keys, only the first NS positions can change and the shift runs NS steps, not KP
  // (most lists hold a few keys: the full KP-step shift was ~half of the kernel).
  auto drain = [&]() {
    wave_lds_sync();
    const int c = S.bcnt[lane];
    const int mc = __builtin_amdgcn_readlane(wave_incl_max(c), 63);
    lc = min(lc + c, KP);
    const int need = __builtin_amdgcn_readlane(wave_incl_max(lc), 63);
    if (need <= 8 && KP > 8) {
#pragma unroll 1
      for (int i = 0; i < mc; ++i) insert_ns<KP, (KP > 8 ? 8 : KP)>(q, i < c ? S.bucket[i][lane] : MR_KEY_EMPTY);
    } else if (need <= 16 && KP > 16) {
#pragma unroll 1
      for (int i = 0; i < mc; ++i) insert_ns<KP, (KP > 16 ? 16 : KP)>(q, i < c ? S.bucket[i][lane] : MR_KEY_EMPTY);
    } else if (need <= 32 && KP > 32) {
#pragma unroll 1
      for (int i = 0; i < mc; ++i) insert_ns<KP, (KP > 32 ? 32 : KP)>(q, i < c ? S.bucket[i][lane] : MR_KEY_EMPTY);
    } else {
#pragma unroll 1
      for (int i = 0; i < mc; ++i) insert(i < c ? S.bucket[i][lane] : MR_KEY_EMPTY);
    }
    S.bcnt[lane] = 0;
    wave_lds_sync();
    mb = 0;
  };
#pragma unroll 1
  for (int eb = 0; eb < count; eb += 64) {
    const int e = eb + lane;
    unsigned long long cmask = 0;
    if (e < count) {
      const int id = ovf ? (int)(vfirst + e) : P.list[vb + ex + e];
      const FaceRec r = load_rec(P.recs, id);
      // candidate pixels: the record's padded bbox; an overflow unit scans only first triangles of
      // split faces, so there it covers both triangles of the pair (as k_tile_raster)
      float bx0 = r.xmin, bx1 = r.xmax, by0 = r.ymin, by1 = r.ymax;
      bool bvalid = (r.flags & FR_VALID) != 0;
      if (ovf && (r.flags & FR_PAIR) && id < P.NF) {
        const FaceRec ro = load_rec(P.recs, P.NF + id);
        if (ro.flags & FR_VALID) {
          bx0 = bvalid ? smin(bx0, ro.xmin) : ro.xmin;
          bx1 = bvalid ? smax(bx1, ro.xmax) : ro.xmax;
          by0 = bvalid ? smin(by0, ro.ymin) : ro.ymin;
          by1 = bvalid ? smax(by1, ro.ymax) : ro.ymax;
          bvalid = true;
        }
      }
      int cx0, cx1, cy0, cy1;
      ndc_range_to_pix(bx0 - pad, bx1 + pad, W, H, cx0, cx1);
      ndc_range_to_pix(by0 - pad, by1 + pad, H, W, cy0, cy1);
      cx0 = max(cx0, x0);
      cx1 = min(cx1, xe);
      cy0 = max(cy0, y0);
      cy1 = min(cy1, ye);
      if (bvalid && cx0 <= cx1 && cy0 <= cy1) cmask = rect_mask(cx0 - x0, cx1 - x0, cy0 - y0, cy1 - y0);
      stage_rec_put(S.rec, lane, r);
      S.id[lane] = id;
    }
    const int np = __popcll(cmask);
    const int pincl = wave_incl_sum(np);
    const int pexcl = pincl - np;
    const int NP = __builtin_amdgcn_readlane(pincl, 63);
    S.meta[lane] = pexcl;
    S.cmask[lane] = cmask;
#pragma unroll 1
    for (int pb = 0; pb < NP;) {
      if (mb > MR_KP_BC - MR_KP_ROOM) drain();
      // the entry straddling pb, and the first entry past what the buckets can still take
      const int first = 63 - __builtin_clzll(__ballot(np > 0 && pexcl <= pb));
      const int lim = first + (MR_KP_BC - mb);
      const int pend = min(pb + 64, lim < 64 ? __builtin_amdgcn_readlane(pexcl, lim) : NP);
      wave_lds_sync();
      if (np > 0 && pexcl > pb && pexcl < pend) S.mark[pexcl - pb] = lane;
      wave_lds_sync();
      int m = S.mark[lane];
      S.mark[lane] = -1;
      if (lane == 0) m = first;
      m = wave_incl_max(m);
      const int qq = pb + lane;
      if (qq < pend) {
        const int p = kth_bit(S.cmask[m], qq - S.meta[m]);
        const FaceRec r = stage_rec_get(S.rec, m);
        const int id = S.id[m];
        const float xf = col_ndc(x0 + (p & 7), H, W), yf = row_ndc(y0 + (p >> 3), H, W);
        float pz;
        int cid = id;
        bool keep = false;
        if (r.flags & FR_PAIR) {  // the split face's two triangles as one candidate (pair rule)
          keep = pair_keep(P.recs, P.NF, id, r, xf, yf, pad, blur, persp, clipb, cid, pz) &&
                 (cid == id || (ovf && id < P.NF));
        } else if (r.flags & FR_VALID) {
          keep = frag_keep(r, xf, yf, pad, blur, persp, clipb, fast_ok && (r.flags & FR_FAST), pz);
        }
        if (keep) {
          const int pos = atomicAdd(&S.bcnt[p], 1);
          S.bucket[pos][p] = frag_key(pz, (int)rec_code(cid, P.NF));
        }
      }
      pb = pend;
      wave_lds_sync();
      mb = __builtin_amdgcn_readlane(wave_incl_max(S.bcnt[lane]), 63);  // the fullest bucket
    }
    wave_lds_sync();  // the stage is rewritten by the next batch
  }
  drain();
  if (!in_img) return;
  const int64_t pix = (n * HW + (int64_t)py * W + px) * K;
  const float xf = col_ndc(px, H, W), yf = row_ndc(py, H, W);
  // only the filled slots (k_fill wrote the background of every slot); keys shifted out through q[0]
  // (constant indices only: the array stays in registers)
#pragma unroll 1
  for (int k = 0; k < K; ++k) {
    if (__ballot(q[0] < MR_KEY_EMPTY) == 0ull) break;
    const unsigned long long key = q[0];
#pragma unroll
    for (int i = 0; i + 1 < KP; ++i) q[i] = q[i + 1];
    q[KP - 1] = MR_KEY_EMPTY;
    if (!(key < MR_KEY_EMPTY)) continue;
    const int id = code_rec((unsigned)(key & 0xffffffffull), P.NF);
    const FaceRec r = P.recs[id];
    FragEval ev;
    eval_face(r, xf, yf, pad, blur, persp, clipb, ev);  // kept by construction
    if (r.flags & FR_CLIP) clip_unconvert(P.crec[id], ev.b0, ev.b1, ev.b2, ev.b0, ev.b1, ev.b2);
    P.p2f[pix + k] = rec_orig(id, P.NF);
    P.zbuf[pix + k] = ev.pz;
    P.dists[pix + k] = ev.sdist;
    P.bary[3 * (pix + k) + 0] = ev.b0;
    P.bary[3 * (pix + k) + 1] = ev.b1;
    P.bary[3 * (pix + k) + 2] = ev.b2;
  }
}

template <int KP>
static void launch_raster_kr(const FwdParams& P, int64_t slots_cap, hipStream_t st) {
  if (slots_cap >= (1ll << 31)) return;
  MR_TIMED(KID_RASTER_K, st, (k_raster_kp<KP><<<(unsigned)slots_cap, 64, 0, st>>>(P)));  // one wave per tile
}

static int launch_raster_k(const FwdParams& P, const BinGeom& g, int64_t N, hipStream_t st) {
  static int fgrid = 0;
  if (!fgrid) fgrid = resident_grid(k_fill<0, 3>, 256, 8);
  MR_TIMED(KID_FILL_FRAG, st, (k_fill<0, 3><<<fgrid, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_fill");
  const int K = P.K;
  if (K <= 64) {  // keys in registers (k_raster_kr)
    const int64_t sc = N * (int64_t)g.T;
    if (K <= 4) launch_raster_kr<4>(P, sc, st);
    else if (K <= 8) launch_raster_kr<8>(P, sc, st);
    else if (K <= 16) launch_raster_kr<16>(P, sc, st);
    else if (K <= 32) launch_raster_kr<32>(P, sc, st);
    else if (K <= 50) launch_raster_kr<50>(P, sc, st);
    else launch_raster_kr<64>(P, sc, st);
    MR_CHECK_LAUNCH("k_raster_kr");
    return MR_OK;
  }
  const size_t wb = (size_t)K * 64 * 8 + 64 * sizeof(FaceRec) + 64 * sizeof(int);
  const int wpg = wb * 4 <= 65536 ? 4 : wb * 2 <= 65536 ? 2 : 1;
  const int64_t slots_cap = N * (int64_t)g.T;
  const int64_t want = (slots_cap + wpg - 1) / wpg;
  const int grid = (int)(want < 8192 ? want : 8192);
  MR_TIMED(KID_RASTER_K, st, (k_raster_k<<<grid, 64 * wpg, wb * wpg, st>>>(P)));
  MR_CHECK_LAUNCH("k_raster_k");
  return MR_OK;
}

// Raster (+ background) then covered-pixel outputs; grids sized once per kernel instance.
template <int MODE, int CH>
static int launch_raster_and_shade(FwdParams P, const BinGeom& g, int64_t N, hipStream_t st, bool clip) {
  P.fill = 1;
  static int rgrid = 0, rgrid_c = 0, sgrid = 0;
  if (!rgrid) rgrid = resident_grid(k_tile_raster<MODE, CH, false>, 256, 7);
  if (!rgrid_c) rgrid_c = resident_grid(k_tile_raster<MODE, CH, true>, 256, 7);
  if (!sgrid) sgrid = resident_grid(k_shade<MODE, CH>, 256, 6);
  if (clip) MR_TIMED(KID_TILE_RASTER, st, (k_tile_raster<MODE, CH, true><<<rgrid_c, 256, 0, st>>>(P)));
  else MR_TIMED(KID_TILE_RASTER, st, (k_tile_raster<MODE, CH, false><<<rgrid, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_tile_raster");
  const int64_t slots_cap = N * (int64_t)g.T;
  int sg = (int)(slots_cap / 4 + 1 < sgrid ? slots_cap / 4 + 1 : sgrid);
  sg = (sg + 7) / 8 * 8;  // XCD-partitioned slot ranges
  MR_TIMED(MODE == 0 ? KID_SHADE_FRAG : KID_SHADE_RENDER, st, (k_shade<MODE, CH><<<sg, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_shade");
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

// Modular backward (PyTorch3D _C.rasterize_meshes_backward), every one of the K faces per pixel.
struct RasterBwdParams {
  int N, H, W, NBX, K;
  int persp, clipb;
  int cull, clipz;
  float zc, blur, bbox_pad;
  const float* fv;
  const int64_t* p2f;
  const float* gz;
  const float* gb;
  const float* gd;
  float* gfv;
};

// One stored fragment (pixel px, py; slot pix; packed face f) of the modular raster backward:
// the 9 face_verts gradients of face f in g.
MR_DEV void raster_bwd_fragment(const RasterBwdParams& P, int px, int py, int64_t pix, int64_t f, float (&g)[3][3]) {
  FaceRec r;
  const float* v = P.fv + 9 * f;
  r.x0 = v[0]; r.y0 = v[1]; r.z0 = v[2];
  r.x1 = v[3]; r.y1 = v[4]; r.z1 = v[5];
  r.x2 = v[6]; r.y2 = v[7]; r.z2 = v[8];
  r.area = (float)((double)edge_fn(r.x2, r.y2, r.x0, r.y0, r.x1, r.y1) + MR_KEPS_D);
  // an upstream gradient PyTorch passed as None arrives as NULL: zero
  const float gb[3] = {P.gb ? P.gb[3 * pix] : 0.0f, P.gb ? P.gb[3 * pix + 1] : 0.0f, P.gb ? P.gb[3 * pix + 2] : 0.0f};
  const float gzp = P.gz ? P.gz[pix] : 0.0f, gdp = P.gd ? P.gd[pix] : 0.0f;
  const float xf = col_ndc(px, P.H, P.W), yf = row_ndc(py, P.H, P.W);
  int ci = 0;
  const float vv[3][3] = {{r.x0, r.y0, r.z0}, {r.x1, r.y1, r.z1}, {r.x2, r.y2, r.z2}};
  const int nb = P.clipz ? clip_class(vv, P.zc, ci) : 0;
  if (nb == 1 || nb == 2) {
    // the face was split at the near plane: rebuild its sub-triangle(s) exactly as the forward
    // binning did, pick the one that produced this fragment (the forward's pair rule), and chain
    for (int c = 0; c < 3; ++c)
      for (int q = 0; q < 3; ++q) g[c][q] = 0.0f;
    float sv[3][3];
    ClipRec cr0, cr1;
    clip_sub(vv, nb, ci, 0, P.zc, P.persp != 0, sv, cr0);
    FaceRec r0 = make_rec_core(P.cull, P.persp, 0u, sv);
    int use = 0;
    FaceRec r1;
    if (nb == 1) {
      clip_sub(vv, nb, ci, 1, P.zc, P.persp != 0, sv, cr1);
      r1 = make_rec_core(P.cull, P.persp, 0u, sv);
      FragEval e0, e1;
      const bool k0 = (r0.flags & FR_VALID) && eval_face(r0, xf, yf, P.bbox_pad, P.blur, P.persp, P.clipb, e0);
      const bool k1 = (r1.flags & FR_VALID) && eval_face(r1, xf, yf, P.bbox_pad, P.blur, P.persp, P.clipb, e1);
      use = (k0 && k1) ? (fabsf(e1.sdist) < fabsf(e0.sdist) ? 1 : 0) : (k1 ? 1 : 0);
    }
    const FaceRec& rs = use ? r1 : r0;
    const ClipRec& cr = use ? cr1 : cr0;
    FragEval es;
    eval_face(rs, xf, yf, P.bbox_pad, P.blur, P.persp, P.clipb, es);
    const float bs[3] = {es.b0, es.b1, es.b2};
    float gs[3], gsub[3][3];
    clip_gb_sub(cr, gb, gs);
    raster_bwd_pixel<false>(rs, xf, yf, P.persp, P.clipb, gzp, gs, gdp, gsub);
    clip_bwd_chain(cr, vv, P.zc, P.persp != 0, bs, gb, gsub, g);
  } else {
    raster_bwd_pixel<false>(r, xf, yf, P.persp, P.clipb, gzp, gb, gdp, g);
  }
}

// One thread per stored fragment slot (n, y, x, k) in memory order: the loads of pix_to_face and
// of the upstream gradients are coalesced (one lane per pixel walking its K slots strided them by
// K elements), and a block whose 256 slots hold no fragment (most of them when K is large: the
// K-nearest lists are short) returns before touching its LDS accumulator.
__global__ void __launch_bounds__(256) k_raster_bwd_slots(RasterBwdParams P, int64_t nslots) {
  __shared__ LdsAcc<9> L;
  const int64_t pix = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t f = pix < nslots ? P.p2f[pix] : -1;
  if (!__syncthreads_or(f >= 0)) return;
  acc_init(L);
  __syncthreads();
  if (f >= 0) {
    const int64_t p = pix / P.K;
    const int64_t hw = (int64_t)P.H * P.W;
    const int rem = (int)(p % hw);
    const int py = rem / P.W, px = rem - py * P.W;
    float g[3][3];
    raster_bwd_fragment(P, px, py, pix, f, g);
    acc_add<9>(L, P.gfv, (int)f, &g[0][0]);
  }
  __syncthreads();
  acc_flush(L, P.gfv);
}

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
    const int64_t pix0 = (((int64_t)n * P.H + py) * P.W + px) * P.K;
    for (int kk = 0; kk < P.K; ++kk) {
      const int64_t pix = pix0 + kk;
      const int64_t f = P.p2f[pix];
      if (f < 0) continue;
      float g[3][3];
      raster_bwd_fragment(P, px, py, pix, f, g);
      acc_add<9>(L, P.gfv, (int)f, &g[0][0]);
    }
  }
  __syncthreads();
  acc_flush(L, P.gfv);
}

// DPP lane moves (GFX9 / CDNA): no LDS round trip (a __shfl is a ds_bpermute_b32 with LDS
// latency; the backward issued ~180 of them per tile in dependent chains).
MR_DEV int dpp_wave_shr1(int v, int old) { return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xf, 0xf, false); }  // wave_shr:1
MR_DEV int dpp_wave_shl1(int v, int old) { return __builtin_amdgcn_update_dpp(old, v, 0x130, 0xf, 0xf, false); }  // wave_shl:1
template <int CTRL, int ROW_MASK>
MR_DEV float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf, false));
}
// Segmented inclusive sum over lanes: d = distance from the lane to the first lane of its run.
// row_shr 1/2/4/8 inside each 16-lane row, then row_bcast:15 / :31 carry a run across rows
// (the structure of wave_incl_sum, each step gated on the run reaching that far back).
// Each step is written as select(gate, x + shifted, x) so the DPP move folds into the add
// (v_add_f32 with a DPP operand + v_cndmask: two VALU ops per step instead of three).
MR_DEV float seg_incl_sum(float x, int d, int lane) {
  const int r = lane & 15;
  float s;
  s = x + dppf<0x111, 0xf>(x); x = (d >= 1) ? s : x;
  s = x + dppf<0x112, 0xf>(x); x = (d >= 2) ? s : x;
  s = x + dppf<0x114, 0xf>(x); x = (d >= 4) ? s : x;
  s = x + dppf<0x118, 0xf>(x); x = (d >= 8) ? s : x;
  s = x + dppf<0x142, 0xa>(x); x = (d > r) ? s : x;            // rows 1, 3 <- lanes 15, 47
  s = x + dppf<0x143, 0xc>(x); x = (d > lane - 32) ? s : x;    // rows 2, 3 <- lane 31
  return x;
}
// Full-wave sum, result in lane 63.
MR_DEV float wave_sum_f_dpp(float x) {
  x += dppf<0x111, 0xf>(x);
  x += dppf<0x112, 0xf>(x);
  x += dppf<0x114, 0xf>(x);
  x += dppf<0x118, 0xf>(x);
  x += dppf<0x142, 0xa>(x);
  x += dppf<0x143, 0xc>(x);
  return x;
}

// Sum ACC-float rows over runs of equal `key` in lane order (segmented DPP scan; the
// covered-pixel list is row-major, so a face's pixels along a row are consecutive lanes).
// seg_stage leaves the run totals in the wave's LDS rows and returns their count; seg_flush
// adds them with float atomics whose lanes cover consecutive components of consecutive runs
// (contiguous 4*ACC-byte rows per run instead of one scattered dword per lane and instruction).
// Lanes with key < 0 carry zero rows. Uniform calls (full EXEC). (Measured alternative: one LDS
// row per distinct face filled with LDS float atomics — slower, 124 vs 102 us, the same-address
// LDS atomics serialise.)
template <int ACC>
MR_DEV int seg_stage(int key, float (&v)[ACC], float* lrow, int* lkey) {
  const int lane = threadIdx.x & 63;
  const int prev = dpp_wave_shr1(key, -2);  // lane 0: no predecessor
  const bool head = lane == 0 || key != prev;
  const int d = lane - wave_incl_max(head ? lane : 0);  // distance to the run's first lane
#pragma unroll
  for (int i = 0; i < ACC; ++i) v[i] = seg_incl_sum(v[i], d, lane);
  const int next = dpp_wave_shl1(key, -2);  // lane 63: no successor
  const bool emit = (lane == 63 || key != next) && key >= 0;
  const unsigned long long m = __ballot(emit);
  if (emit) {
    const int slot = __popcll(m & ((1ull << lane) - 1ull));
    lkey[slot] = key;
#pragma unroll
    for (int i = 0; i < ACC; ++i) lrow[slot * ACC + i] = v[i];
  }
  wave_lds_sync();
  return __popcll(m);
}
// Straight-line (unrolled, uniform skips): as a loop, the waitcnt pass drains every pending load
// (s_waitcnt vmcnt(0)) in the loop preheader, i.e. waits on the prefetches issued just before.
template <int ACC>
MR_DEV void seg_flush(int nt, float* __restrict__ dst, const float* lrow, const int* lkey) {
  // lane id through an opaque copy: the unrolled blocks' row/column indices are invariant in the
  // caller's slot loop, and hoisted out of it they would stay live across the whole loop
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int tot = nt * ACC;  // <= 64 * ACC
#pragma unroll
  for (int i = 0; i < ACC; ++i) {
    if (64 * i < tot) {
      const int j = 64 * i + lane;
      if (j < tot) {
        const int r = j / ACC;
        const float x = lrow[j];
        if (x != 0.0f) atomicAdd(&dst[(int64_t)lkey[r] * ACC + (j - r * ACC)], x);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // one row block at a time (no hoisting: register peak)
  }
  wave_lds_sync();
}
template <int ACC>
MR_DEV void seg_scatter(int key, float (&v)[ACC], float* __restrict__ dst, float* lrow, int* lkey) {
  seg_flush<ACC>(seg_stage<ACC>(key, v, lrow, lkey), dst, lrow, lkey);
}

// The slot's 12 R/T partial sums (wave-wide DPP sums, fixed order: deterministic), lane i
// holding sum i (lanes 0..11); stored later by one store instruction. Uniform call (full EXEC).
MR_DEV float rt_partial(const float (&gR)[9], const float (&gT)[3], int lane) {
  float o = 0.0f;
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const float t = wave_sum_f_dpp(i < 9 ? gR[i] : gT[i - 9]);
    const float s = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, t), 63));
    o = lane == i ? s : o;
  }
  return o;
}

// Fused render backward over the slots of the non-empty tiles (k_tile_raster's sface: per
// tile pixel the winning face record or -1; the pixel is implied by slot and lane). Per covered
// pixel: half 1 recomputes fragment + shading and differentiates the blends / Phong / texture ->
// a 20-float record (grads of z, signed dist, barycentrics, interpolated point / normal / texel,
// and the barycentrics) handed to half 2 through the wave's LDS; half 2 runs the rasterizer
// backward (edge functions, perspective correction, distances; the near-plane clip's chain rule
// for split faces) + projection backward -> per-face rows summed over runs of equal faces
// (seg_scatter), and the slot's R/T partial sums. (Measured: the same two halves as two kernels
// with the record in HBM took 123 us against 102 for the fused kernel.)
// Waves stride over XCD-contiguous slot ranges (one 8x8 tile, one view each).
#define MR_BWD_REC 5  // float4s per pixel record
struct RenderBwdParams {
  int N, H, W, TX, T;
  float blur, bbox_pad;
  int persp, clipb;
  const FaceRec* recs;
  const int* ctr;
  const int* sface;
  const int* stile;
  const int* vslot;
  const float* gD;
  const float* gS;
  const float* gRGB;
  int rgb_ch;
  int sil_rgba;  // gS is the (N,H,W,4) gradient of an RGBA silhouette (MR_OUT_SIL_RGBA)
  ShadeParams S;
  const ShadeRec* srec;
  int64_t F;     // faces of the shared mesh: record id rid = n*F + face
  int64_t NF;    // N * F: the second triangle of a split face is record NF + rid
  const ClipRec* crec;
  float zc;      // z_clip_value (clipped records only)
  const ViewRec* views;
  float* gface;  // (F, ACC): 9 position rows, 9 normal rows [, 9 vertex-colour rows]
  float* rt_part;  // (slots, 12) per-slot R/T partial sums
  const float4* frec;  // (slots, 64) the forward's fragments (k_shade<1>): b0, b1, b2, signed dist
};

MR_DEV void slot_pixel(const RenderBwdParams& P, int gt, int lane, int& n, int& px, int& py) {
  n = gt / P.T;
  const int t = gt - n * P.T;
  const int ty = t / P.TX, tx = t - ty * P.TX;
  px = tx * MR_TS + (lane & 7);
  py = ty * MR_TS + (lane >> 3);
}

// Both halves in one kernel (the default): the shade backward's 20-float record goes through
// the wave's LDS instead of HBM (80 B written + 80 B read per covered pixel), and the slot,
// winners and face record are fetched once. Peak VGPRs stay those of the larger half: the
// LDS hand-off ends the first half's live ranges.
// Face record and upstream gradients (depth, silhouette, RGB) of one slot pixel. The loads are
// unconditional (record 0 / a zero buffer when the lane has no fragment or an output has no
// gradient; such values are never used): written as guarded loads they become branches whose
// phi copies wait on the load right away, which defeats the prefetch.
__device__ float g_zero4[4];
MR_DEV void bwd_slot_inputs(const RenderBwdParams& P, int slot, int gt, int f, int lane, FaceRec& r, float g[5],
                             float4& fr) {
  int n, px, py;
  slot_pixel(P, gt, lane, n, px, py);
  const int64_t pix = n * (int64_t)P.H * P.W + (int64_t)py * P.W + px;
  r = load_rec(P.recs, f < 0 ? 0 : f);
  fr = P.frec[(int64_t)slot * 64 + lane];
  const float* pD = P.gD ? P.gD + pix : g_zero4;
  const float* pS = P.gS ? P.gS + (P.sil_rgba ? 4 * pix + 3 : pix) : g_zero4;
  const float* pC = P.gRGB ? P.gRGB + pix * P.rgb_ch : g_zero4;
  g[0] = *pD;
  g[1] = *pS;
  g[2] = pC[0];
  g[3] = pC[1];
  g[4] = pC[2];
}

// Near-plane sub-triangle (record f, flag FR_CLIP): gfv holds the raster backward w.r.t. the
// sub-triangle's corners (run with C g_orig); map it to the ORIGINAL face's projected corners
// through the clip's chain rule (sub-corners and the conversion weights), the original corners
// re-projected from the world corners. g_orig: gradient w.r.t. the original-face barycentrics.
MR_DEV void clipped_chain(const RenderBwdParams& P, const FaceRec& r, int f, const ViewRec& V, const float X[3][3],
                          float px, float py, const float g_orig[3], float gfv[3][3]) {
  const ClipRec cr = P.crec[f];
  FragEval e;
  eval_face(r, px, py, P.bbox_pad, P.blur, P.persp, P.clipb, e);
  const float bs[3] = {e.b0, e.b1, e.b2};
  float v[3][3], gsub[3][3];
  for (int c = 0; c < 3; ++c) {
    float vx, vy, vz, nx, ny;
    project_point(V, X[c], vx, vy, vz, nx, ny);
    v[c][0] = nx;
    v[c][1] = ny;
    v[c][2] = vz;
    for (int q = 0; q < 3; ++q) {
      gsub[c][q] = gfv[c][q];
      gfv[c][q] = 0.0f;
    }
  }
  clip_bwd_chain(cr, v, P.zc, P.persp != 0, bs, g_orig, gsub, gfv);
}

// Alpha-channel upstream gradient (RGBA outputs only; the drop-in frame has rgb_ch = 3).
MR_DEV float g_alpha(const RenderBwdParams& P, int gt, int lane) {
  int n, px, py;
  slot_pixel(P, gt, lane, n, px, py);
  const int64_t pix = n * (int64_t)P.H * P.W + (int64_t)py * P.W + px;
  return P.gRGB[pix * P.rgb_ch + 3];
}

// CLIP: near-plane clipping on (clipped sub-triangles may be present); the CLIP = false
// instantiation carries none of the clip chain rule (fewer registers, no dynamic corner indexing).
#define MR_BWD_ATTR
// The kernel's parameters re-read from the kernarg segment through a pointer the compiler cannot see
// through: uniform values used across a long loop body are otherwise hoisted into SGPRs for the whole
// loop, overflow the SGPR file and are spilled into VGPR lanes (one v_readlane per use; k_bwd_fused had
// 70 spilled SGPRs and ~400 readlanes per slot iteration). Re-read per iteration, each is a scalar
// load from the (cached) kernarg segment, live only where it is used.
template <typename T>
MR_DEV const T& kernarg_params() {
  typedef const char __attribute__((address_space(4))) * cptr;
  cptr p = (cptr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const T*)(const char*)p;
}

template <int ACC, bool CLIP>
__global__ void __launch_bounds__(256) MR_BWD_ATTR k_bwd_fused(RenderBwdParams P0) {
  const RenderBwdParams& P = P0;
  __shared__ float lrow[4][64 * ACC];
  __shared__ int lkey[4][64];
  __shared__ float4 lrec[4][MR_BWD_REC][64];
  const bool lut = stage_tex_lut(P.S);  // the u8 texture table in LDS
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nslots = P.ctr[CTR_SLOTS];
  int s, G, send;
  xcd_slot_range(nslots, wave, s, G, send);
  // Three-deep software pipeline (the kernel runs at 2 waves/SIMD, so a wave must hide its own
  // latency): while slot s is processed, the face record and upstream gradients of slot s + G
  // and the tile id and winner of slot s + 2G are in flight.
  // gt_* are per-lane copies of the (uniform) tile id, made uniform where they are consumed
  // Prefetches past the wave's last slot read a clamped (valid) slot and are never consumed.
  const int lz = lane_zero();
  const int slast = max(nslots - 1, 0);
  int sc = min(s, slast);
  int sl_c = sc;  // slot of gt_c / f_c (clamped)
  int gt_c = P.stile[sc + lz], f_c = P.sface[(int64_t)sc * 64 + lane];
  sc = min(s + G, slast);
  int sl_n = sc;
  int gt_n = P.stile[sc + lz], f_n = P.sface[(int64_t)sc * 64 + lane];
  FaceRec r_c;
  float g_c[5];
  float4 fr_c;
  bwd_slot_inputs(P, sl_c, __builtin_amdgcn_readfirstlane(gt_c), f_c, lane, r_c, g_c, fr_c);
  int nt_prev = -1, s_prev = 0;  // the previous slot's staged runs (-1: none yet)
  float rt_prev = 0.0f;
  for (; s < send; s += G) {
    const RenderBwdParams& P = kernarg_params<RenderBwdParams>();  // see kernarg_params
    const int gt = __builtin_amdgcn_readfirstlane(gt_c), f = f_c;
    const FaceRec r = r_c;
    const float4 frag = fr_c;
    float gin[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) gin[i] = g_c[i];
    gt_c = gt_n;
    f_c = f_n;
    sl_c = sl_n;
    bwd_slot_inputs(P, sl_c, __builtin_amdgcn_readfirstlane(gt_c), f_c, lane, r_c, g_c, fr_c);
    sc = min(s + 2 * G, slast);
    sl_n = sc;
    gt_n = P.stile[sc + lz];
    f_n = P.sface[(int64_t)sc * 64 + lane];
    int n, px, py;
    slot_pixel(P, gt, lane, n, px, py);
    // ---- half 1: blends / Phong / texture backward -> lrec
    if (f >= 0) {
      PixGeom Gm;
      load_geom(P.srec, (uint32_t)(rec_orig(f, P.NF) - n * P.F), Gm);
      const float gD = gin[0], gS = gin[1];
      float gC[3] = {gin[2], gin[3], gin[4]};
      const float gA = (P.gRGB && P.rgb_ch == 4) ? g_alpha(P, gt, lane) : 0.0f;
      FragEval e;
      float4 o[MR_BWD_REC];
      // the forward's fragment (k_shade<1> wrote the winner's barycentrics, original-face ones for a
      // near-plane sub-triangle, and signed distance); the depth from the record's corners in
      // eval_face's operation order, or, for a sub-triangle (whose corners are not the original
      // face's), from eval_face itself
      e.b0 = frag.x;
      e.b1 = frag.y;
      e.b2 = frag.z;
      e.sdist = frag.w;
      e.pz = (e.b0 * r.z0 + e.b1 * r.z1) + e.b2 * r.z2;
      if (CLIP && (r.flags & FR_CLIP)) {
        FragEval es;
        eval_face(r, col_ndc(px, P.H, P.W), row_ndc(py, P.H, P.W), P.bbox_pad, P.blur, P.persp, P.clipb, es);
        e.pz = es.pz;
      }
      {
        ShadeOut so;
        ShadeCache C;
        shade_fwd(P.S, n, true, Gm, e.b0, e.b1, e.b2, e.pz, e.sdist, so, C, lut);
        ShadeGrad SG;
        shade_bwd(P.S, Gm, e.b0, e.b1, e.b2, e.pz, C, gD, gS, gC, gA, SG, lut);
        o[0] = make_float4(SG.gz, SG.gsd, SG.gb[0], SG.gb[1]);
        o[1] = make_float4(SG.gb[2], SG.gP[0], SG.gP[1], SG.gP[2]);
        o[2] = make_float4(SG.gNn[0], SG.gNn[1], SG.gNn[2], e.b0);
        o[3] = make_float4(e.b1, e.b2, SG.gtex[0], SG.gtex[1]);
        o[4] = make_float4(SG.gtex[2], 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < MR_BWD_REC; ++k) lrec[wave][k][lane] = o[k];
    }
    wave_lds_sync();
    __builtin_amdgcn_sched_barrier(0);  // keep half 2's loads out of half 1's register peak
    // ---- half 2: raster + projection backward, per-face runs, R/T partials
    const ViewRec V = P.views[n];
    // world corners (first 36 B of the ShadeRec), issued BEFORE the previous slot's deferred
    // atomics: vmcnt retires in issue order, so a load issued after them would wait the
    // atomics' ~3k-cycle completion; issued before, its wait is a precise count
    // (unconditional: face 0 for lanes without a fragment, see bwd_slot_inputs)
    const int face = f >= 0 ? (int)(rec_orig(f, P.NF) - n * P.F) : 0;
    const float4* x4 = (const float4*)(P.srec + face);
    const float4 w0 = x4[0], w1 = x4[1], w2 = x4[2];
    __builtin_amdgcn_sched_barrier(0);
    // previous slot's face rows and R/T partials, deferred to here (see above): the loads of
    // half 1 and the corners above are already in flight or consumed
    if (nt_prev >= 0) {
      seg_flush<ACC>(nt_prev, P.gface, lrow[wave], lkey[wave]);
      if (lane < 12) P.rt_part[(int64_t)s_prev * 12 + lane] = rt_prev;
    }
    __builtin_amdgcn_sched_barrier(0);
    float gR[9], gT[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) gR[i] = 0.0f;
#pragma unroll
    for (int i = 0; i < 3; ++i) gT[i] = 0.0f;
    float row[ACC];
#pragma unroll
    for (int k = 0; k < ACC; ++k) row[k] = 0.0f;
    int key = -1;
    if (f >= 0) {
      const float4 a0 = lrec[wave][0][lane], a1 = lrec[wave][1][lane], a2 = lrec[wave][2][lane];
      const float4 a3 = lrec[wave][3][lane];
      const float4 a4 = ACC == 27 ? lrec[wave][4][lane] : make_float4(0.f, 0.f, 0.f, 0.f);
      const float X[3][3] = {{w0.x, w0.y, w0.z}, {w0.w, w1.x, w1.y}, {w1.z, w1.w, w2.x}};
      const float gb[3] = {a0.z, a0.w, a1.x};
      const float gP[3] = {a1.y, a1.z, a1.w};
      const float gNn[3] = {a2.x, a2.y, a2.z};
      const float b[3] = {a2.w, a3.x, a3.y};
      const float gt3[3] = {a3.z, a3.w, a4.x};
      float gfv[3][3];
      const bool clipped = CLIP && (r.flags & FR_CLIP) != 0;
      const float pxf = col_ndc(px, P.H, P.W), pyf = row_ndc(py, P.H, P.W);
      float gbr[3] = {gb[0], gb[1], gb[2]};
      if (clipped) clip_gb_sub(P.crec[f], gb, gbr);  // near-plane sub-triangle: C g_orig
      raster_bwd_pixel<true>(r, pxf, pyf, P.persp, P.clipb, a0.x, gbr, a0.y, gfv);
      if (__builtin_expect(clipped, 0)) clipped_chain(P, r, f, V, X, pxf, pyf, gb, gfv);
      key = face;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        float gX[3];
        project_bwd(V, X[c], gfv[c], gX, gR, gT);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          row[3 * c + k] = b[c] * gP[k] + gX[k];
          row[9 + 3 * c + k] = b[c] * gNn[k];
          if (ACC == 27) row[18 + 3 * c + k] = b[c] * gt3[k];
        }
      }
    }
    nt_prev = seg_stage<ACC>(key, row, lrow[wave], lkey[wave]);
    rt_prev = rt_partial(gR, gT, lane);
    s_prev = s;
  }
  if (nt_prev >= 0) {
    seg_flush<ACC>(nt_prev, P.gface, lrow[wave], lkey[wave]);
    if (lane < 12) P.rt_part[(int64_t)s_prev * 12 + lane] = rt_prev;
  }
}

// grad_views[n] = sum of the partial rows of view n's slots (fixed order: deterministic).
// out (N,12) PyTorch3D-frame R/T grads, or (gRcv, gtcv) non-null: the same grads written
// straight in the OpenCV frame (k_view_grads_to_opencv's chain rule, saving its launch).
MR_DEV void rt_reduce_view(const float* __restrict__ part, const int* __restrict__ vslot, int N,
                           float* __restrict__ out, float* __restrict__ gRcv, float* __restrict__ gtcv, int n) {
  __shared__ float sm[12][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int s0 = vslot[n], ns = vslot[N + n];
  // each thread sums whole 48-B partial rows (three 16-B loads in flight together instead of 12
  // dependent passes over the rows); per component the order is the same as a per-component loop
  float acc[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) acc[i] = 0.0f;
  for (int t = threadIdx.x; t < ns; t += 256) {
    const float4* q = (const float4*)(part + ((int64_t)s0 + t) * 12);
    const float4 a = q[0], b = q[1], c = q[2];
    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
    acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
    acc[8] += c.x; acc[9] += c.y; acc[10] += c.z; acc[11] += c.w;
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    for (int o = 32; o > 0; o >>= 1) acc[i] += __shfl_xor(acc[i], o, 64);
    if (lane == 0) sm[i][wave] = acc[i];
  }
  __syncthreads();
  const int i = threadIdx.x;
  if (i >= 12) return;
  const float v = ((sm[i][0] + sm[i][1]) + sm[i][2]) + sm[i][3];
  if (!gRcv) {
    out[n * 12 + i] = v;
  } else if (i < 9) {  // dL/dR_cv[b][a] = dL/dR_p3d[a][b] * s[b]
    const int a = i / 3, b = i - 3 * a;
    gRcv[(int64_t)n * 9 + 3 * b + a] = b < 2 ? -v : v;
  } else {
    gtcv[(int64_t)n * 3 + (i - 9)] = i < 11 ? -v : v;
  }
}

__global__ void __launch_bounds__(256) k_rt_reduce(const float* __restrict__ part, const int* __restrict__ vslot,
                                                   int N, float* __restrict__ out, float* __restrict__ gRcv,
                                                   float* __restrict__ gtcv) {
  rt_reduce_view(part, vslot, N, out, gRcv, gtcv, blockIdx.x);
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
  if (v < V) vertex_normal(verts, faces, ptr, adj, v, vn, vraw);
}
// verts_normals_packed for vertex v: the sum of its faces' (unnormalised) normals in CSR order
// (the reference's index_add order), then F.normalize.
MR_DEV void vertex_normal(const float* __restrict__ verts, const int32_t* __restrict__ faces,
                          const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj, int64_t v,
                          float* __restrict__ vn, float* __restrict__ vraw) {
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
#define MR_VL 8  // lanes per vertex in the CSR gathers of the vertex-gradient kernels
template <int ACC>
MR_DEV void vgrad_a_block(int64_t V, const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj,
                          const float* __restrict__ gface, const float* __restrict__ vraw, float* __restrict__ gnu,
                          int64_t blk) {
  // MR_VL lanes per vertex split its CSR entries, then a fixed xor-tree sums them (deterministic)
  const int64_t gid = blk * blockDim.x + threadIdx.x;
  const int64_t v = gid / MR_VL;
  const int j = (int)(gid % MR_VL);
  const bool act = v < V;
  float g[3] = {0.f, 0.f, 0.f};
  if (act) {
    for (int e = ptr[v] + j; e < ptr[v + 1]; e += MR_VL) {
      const int f = adj[e] >> 2, c = adj[e] & 3;
      for (int k = 0; k < 3; ++k) g[k] += gface[(int64_t)f * ACC + 9 + 3 * c + k];
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k)
    for (int o = MR_VL / 2; o > 0; o >>= 1) g[k] += __shfl_xor(g[k], o, 64);
  if (!act || j != 0) return;
  const float x[3] = {vraw[3 * v], vraw[3 * v + 1], vraw[3 * v + 2]};
  const float nrm = sqrtf(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  const float den = smax(nrm, 1e-6f);
  float gx[3];
  normalize3_bwd(x, nrm, den, g, gx);
  for (int k = 0; k < 3; ++k) gnu[3 * v + k] = gx[k];
}

// The per-view R/T reduction and the vertex-normal gradient read disjoint inputs written by
// k_bwd_fused, so one launch does both: blocks [0, N) reduce views, the rest run k_vgrad_a
// (saves a dependent launch of two tiny kernels per step).
template <int ACC>
__global__ void __launch_bounds__(256) k_rt_vgrad_a(const float* __restrict__ part, const int* __restrict__ vslot,
                                                    int N, float* __restrict__ gviews, float* __restrict__ gRcv,
                                                    float* __restrict__ gtcv, int64_t V,
                                                    const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj,
                                                    const float* __restrict__ gface, const float* __restrict__ vraw,
                                                    float* __restrict__ gnu) {
  if ((int)blockIdx.x < N) rt_reduce_view(part, vslot, N, gviews, gRcv, gtcv, blockIdx.x);
  else vgrad_a_block<ACC>(V, ptr, adj, gface, vraw, gnu, (int64_t)blockIdx.x - N);
}

// B: grad_verts[v] = sum over incident (f, c) of position rows + cross-product backward of the face normal.
template <int ACC>
__global__ void __launch_bounds__(256) k_vgrad_b(int64_t V, const float* __restrict__ verts,
                                                 const int32_t* __restrict__ faces, const int32_t* __restrict__ ptr,
                                                 const int32_t* __restrict__ adj, const float* __restrict__ gface,
                                                 const float* __restrict__ gnu, int use_normals,
                                                 float* __restrict__ gverts, float* __restrict__ gcol) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t v = gid / MR_VL;
  const int j = (int)(gid % MR_VL);
  const bool act = v < V;
  float g[3] = {0.f, 0.f, 0.f}, gc[3] = {0.f, 0.f, 0.f};
  const int e0 = act ? ptr[v] + j : 0, e1 = act ? ptr[v + 1] : 0;
  for (int e = e0; e < e1; e += MR_VL) {
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
#pragma unroll
  for (int k = 0; k < 3; ++k)
    for (int o = MR_VL / 2; o > 0; o >>= 1) {
      g[k] += __shfl_xor(g[k], o, 64);
      if (ACC == 27) gc[k] += __shfl_xor(gc[k], o, 64);
    }
  if (!act || j != 0) return;
  for (int k = 0; k < 3; ++k) gverts[3 * v + k] = g[k];
  if (ACC == 27 && gcol)
    for (int k = 0; k < 3; ++k) gcol[3 * v + k] = gc[k];
}

// projection: face_verts[n*F+f][c] = ndc(view n, X); distinct meshes (ff = first union face of
// each view, N+1): face_verts[f] for the faces f of view n's mesh
__global__ void __launch_bounds__(256) k_project_faces(const float* __restrict__ verts, const int32_t* __restrict__ faces,
                                                       int64_t F, const ViewRec* __restrict__ views, float* __restrict__ fv,
                                                       const int64_t* __restrict__ ff) {
  int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = blockIdx.y;
  int64_t o0;  // face_verts row
  if (ff) {
    f += ff[n];
    if (f >= ff[n + 1]) return;
    o0 = f;
  } else {
    if (f >= F) return;
    o0 = (int64_t)n * F + f;
  }
  const ViewRec V = views[n];
  for (int c = 0; c < 3; ++c) {
    const int32_t vi = faces[3 * f + c];
    const float X[3] = {verts[3 * (int64_t)vi], verts[3 * (int64_t)vi + 1], verts[3 * (int64_t)vi + 2]};
    float vx, vy, vz, nx, ny;
    project_point(V, X, vx, vy, vz, nx, ny);
    float* o = fv + (o0 * 3 + c) * 3;
    o[0] = nx;
    o[1] = ny;
    o[2] = vz;
  }
}

// projection backward: thread per (n, v); grads summed over incident faces (CSR order).
// Distinct meshes (vf = first union vertex of each view's mesh, N+1): view n's own vertices, whose
// faces' rows are face_verts[f].
__global__ void __launch_bounds__(256) k_project_faces_bwd(const float* __restrict__ verts, int64_t V, int64_t F,
                                                           const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj,
                                                           const ViewRec* __restrict__ views,
                                                           const float* __restrict__ gfv, float* __restrict__ gverts,
                                                           float* __restrict__ gviews, const int64_t* __restrict__ vf) {
  __shared__ float red[4][12];
  int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = blockIdx.y;
  const ViewRec Vw = views[n];
  const int64_t rb = vf ? 0 : (int64_t)n * F;  // face_verts row of face f: rb + f
  int64_t vend = V;
  if (vf) {
    v += vf[n];
    vend = vf[n + 1];
  }
  float gR[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, gT[3] = {0, 0, 0};
  if (v < vend) {
    float gn[3] = {0.f, 0.f, 0.f};
    for (int e = ptr[v]; e < ptr[v + 1]; ++e) {
      const int f = adj[e] >> 2, c = adj[e] & 3;
      const float* q = gfv + ((rb + f) * 3 + c) * 3;
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
// 5. K-deep soft shading over stored fragments (SoftPhongShader / SoftSilhouetteShader on the
//    output of mr_rasterize_meshes with faces_per_pixel = K; SURVEY §8f rank 1:
//    deform_mesh_with_color.py:153-159 K = 50, renderer_comparison_with_pyrender.py:174-179).
//    One thread per pixel walks its K fragments: Phong colour per fragment (interpolation,
//    texture, lighting) and upstream's softmax_rgb_blend / sigmoid_alpha_blend across them.
//    The backward returns the fragments' gradients (zbuf, bary, dists: into the rasterizer's
//    backward) and the attribute gradients: per-face rows (world position, normal, vertex colour;
//    summed over runs of equal faces per wave and fragment layer), texture-map texels and uvs.
// ---------------------------------------------------------------------------
struct FragShadeParams {
  int N, H, W, K;
  int64_t F;   // faces of the shared mesh; p2f holds packed ids n*F + f
  int sil;     // 1: sigmoid_alpha_blend (rgb = 1); 0: Phong + softmax_rgb_blend
  int hard;    // 1 (with sil = 0): Phong + hard_rgb_blend (HardPhongShader)
  const int64_t* p2f;
  const float* zbuf;
  const float* bary;
  const float* dists;
  ShadeParams S;
  const ShadeRec* srec;
  float* rgba;          // (N,H,W,4)
  const float* g_rgba;  // backward
  float* g_zbuf;
  float* g_bary;
  float* g_dists;
  float* gface;         // (F, ACC)
  float* gmap;          // (Ht, Wt, 4) or null
  float* guv;           // (Vt, 2) or null
};

// z_inv and the softmax weights exp((z_inv - zmax) / gamma) use IEEE division and expf here: with
// gamma = 1e-4 the weights amplify z_inv's rounding 10^4-fold (K > 1 has z_inv < zmax).
// Pass over the pixel's K fragments: z_inv max (masked entries count as 0, as upstream's
// `z_inv * mask`), its first index, and (Phong) the blend sums; alpha product split into the
// product of the non-zero factors and the count / index of zero factors (for the backward's
// product-of-the-others).
struct FragSums {
  float zmax_raw, zmax;  // max_k z_inv (with masked zeros), clamped at 1e-10
  int kmax;
  float alpha_nz;        // product of the non-zero (1 - prob) factors
  int nzero, kzero;
  float numw[3], denw;   // sum_k w_k c_k, sum_k w_k
};

MR_DEV float frag_prob(float d, float inv_sigma) { return sigmoidf_((-d) * inv_sigma); }

MR_DEV void frag_sums(const FragShadeParams& P, int64_t pix, int n, FragSums& R, bool colours) {
  const ShadeParams& S = P.S;
  const int64_t base = pix * P.K;
  R.zmax_raw = 0.0f;
  R.kmax = 0;
  if (!P.sil) {
    for (int k = 0; k < P.K; ++k) {
      const bool m = P.p2f[base + k] >= 0;
      const float zi = ((S.zfar - P.zbuf[base + k]) / (S.zfar - S.znear)) * (m ? 1.0f : 0.0f);
      if (k == 0 || zi > R.zmax_raw) {
        R.zmax_raw = zi;
        R.kmax = k;
      }
    }
  }
  R.zmax = smax(R.zmax_raw, 1e-10f);
  R.alpha_nz = 1.0f;
  R.nzero = 0;
  R.kzero = -1;
  R.denw = 0.0f;
  R.numw[0] = R.numw[1] = R.numw[2] = 0.0f;
  const float isig = P.sil ? S.inv_sigma_sil : S.inv_sigma_rgb;
  for (int k = 0; k < P.K; ++k) {
    const int64_t f = P.p2f[base + k];
    if (f < 0) continue;  // masked: prob 0, factor 1, weight 0
    const float prob = frag_prob(P.dists[base + k], isig);
    const float one_m = 1.0f - prob;
    if (one_m == 0.0f) {
      ++R.nzero;
      R.kzero = k;
    } else {
      R.alpha_nz *= one_m;
    }
    if (P.sil || !colours) continue;
    const float zi = (S.zfar - P.zbuf[base + k]) / (S.zfar - S.znear);
    const float w = prob * expf((zi - R.zmax) / S.gamma);
    PixGeom G;
    load_geom(P.srec, (uint32_t)(f - (int64_t)n * P.F), G);
    const float* b = P.bary + 3 * (base + k);
    float col[3];
    PhongCache C;
    phong_fwd(S, n, G, b[0], b[1], b[2], col, C);
    for (int c = 0; c < 3; ++c) R.numw[c] += w * col[c];
    R.denw += w;
  }
}

__global__ void __launch_bounds__(256) k_frag_shade_fwd(FragShadeParams P) {
  const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t HW = (int64_t)P.H * P.W;
  if (pix >= (int64_t)P.N * HW) return;
  const int n = (int)(pix / HW);
  if (P.hard) {  // hard_rgb_blend: the nearest fragment (k = 0) or the background
    const int64_t f = P.p2f[pix * P.K];
    float4 o = make_float4(P.S.bg[0], P.S.bg[1], P.S.bg[2], 0.0f);
    if (f >= 0) {
      PixGeom G;
      load_geom(P.srec, (uint32_t)(f - (int64_t)n * P.F), G);
      const float* b = P.bary + 3 * (pix * P.K);
      float col[3];
      PhongCache C;
      phong_fwd(P.S, n, G, b[0], b[1], b[2], col, C);
      o = make_float4(col[0], col[1], col[2], 1.0f);
    }
    ((float4*)P.rgba)[pix] = o;
    return;
  }
  FragSums R;
  frag_sums(P, pix, n, R, true);
  const float alpha = R.nzero ? 0.0f : R.alpha_nz;
  float4 o;
  if (P.sil) {
    o = make_float4(1.0f, 1.0f, 1.0f, 1.0f - alpha);
  } else {
    const ShadeParams& S = P.S;
    const float delta = smax(expf((1e-10f - R.zmax) / S.gamma), 1e-10f);
    const float rden = frcp(R.denw + delta);
    o = make_float4((R.numw[0] + delta * S.bg[0]) * rden, (R.numw[1] + delta * S.bg[1]) * rden,
                    (R.numw[2] + delta * S.bg[2]) * rden, 1.0f - alpha);
  }
  ((float4*)P.rgba)[pix] = o;
}

template <int ACC>
__global__ void __launch_bounds__(256) k_frag_shade_bwd(FragShadeParams P) {
  __shared__ float lrow[4][64 * ACC];
  __shared__ int lkey[4][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t HW = (int64_t)P.H * P.W;
  const bool act = pix < (int64_t)P.N * HW;  // inactive lanes still join the uniform scatters
  const int n = act ? (int)(pix / HW) : 0;
  const ShadeParams& S = P.S;
  FragSums R;
  float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float g_num[3] = {0.f, 0.f, 0.f}, g_den = 0.0f, g_zmax = 0.0f, g_alpha = 0.0f;
  if (act && P.hard) {
    g4 = ((const float4*)P.g_rgba)[pix];  // alpha (coverage) has no gradient
  } else if (act) {
    frag_sums(P, pix, n, R, true);
    g4 = ((const float4*)P.g_rgba)[pix];
    g_alpha = -g4.w;  // A = 1 - alpha
    if (!P.sil) {
      const float ex = expf((1e-10f - R.zmax) / S.gamma);
      const float delta = smax(ex, 1e-10f);
      const float den = R.denw + delta;
      const float rden = frcp(den);
      const float gr[3] = {g4.x, g4.y, g4.z};
      float g_delta = 0.0f;
      for (int c = 0; c < 3; ++c) {
        const float num = R.numw[c] + delta * S.bg[c];
        g_num[c] = gr[c] * rden;
        g_den += -gr[c] * num * (rden * rden);
        g_delta += g_num[c] * S.bg[c];
      }
      g_delta += g_den;
      // through the weights' exp((z_inv - zmax) / gamma): sum_k g_w_k w_k, with
      // g_w_k = g_num . c_k + g_den, is g_num . numw + g_den * denw
      const float gwe = ((g_num[0] * R.numw[0] + g_num[1] * R.numw[1]) + g_num[2] * R.numw[2]) + g_den * R.denw;
      g_zmax = -(gwe * S.inv_gamma);
      if (ex >= 1e-10f) g_zmax += -((g_delta * ex) * S.inv_gamma);
      if (!(R.zmax_raw >= 1e-10f)) g_zmax = 0.0f;  // clamp(min=eps) blocks it
    }
  }
  const int64_t base = pix * P.K;
  const float isig = P.sil ? S.inv_sigma_sil : S.inv_sigma_rgb;
#pragma unroll 1
  for (int k = 0; k < P.K; ++k) {  // uniform over the wave (seg_scatter inside)
    const int64_t f = act ? P.p2f[base + k] : -1;
    float row[ACC];
#pragma unroll
    for (int q = 0; q < ACC; ++q) row[q] = 0.0f;
    int key = -1;
    if (f >= 0 && P.hard) {
      // hard_rgb_blend: only the nearest fragment's colour carries a gradient; no depth / dists
      float gb[3] = {0.f, 0.f, 0.f};
      if (k == 0) {
        const int face = (int)(f - (int64_t)n * P.F);
        PixGeom G;
        load_geom(P.srec, (uint32_t)face, G);
        const float* b = P.bary + 3 * base;
        float col[3];
        PhongCache C;
        phong_fwd(S, n, G, b[0], b[1], b[2], col, C);
        const float gcol[3] = {g4.x, g4.y, g4.z};
        float gP[3], gNn[3], gtex[3], guv[2];
        phong_bwd(S, G, C, gcol, gb, gP, gNn, gtex, guv);
        key = face;
        for (int c = 0; c < 3; ++c)
          for (int q = 0; q < 3; ++q) {
            row[3 * c + q] = b[c] * gP[q];
            row[9 + 3 * c + q] = b[c] * gNn[q];
            if (ACC == 27) row[18 + 3 * c + q] = b[c] * gtex[q];
          }
        if (S.tex_kind == 2) {
          if (P.gmap) tex_map_bwd(S, C.tap, gtex, P.gmap);
          if (P.guv) {
            const int32_t* fu = S.faces_uvs + 3 * (int64_t)face;
            for (int c = 0; c < 3; ++c) {
              if (guv[0] != 0.0f) atomicAdd(&P.guv[2 * (int64_t)fu[c]], b[c] * guv[0]);
              if (guv[1] != 0.0f) atomicAdd(&P.guv[2 * (int64_t)fu[c] + 1], b[c] * guv[1]);
            }
          }
        }
      }
      P.g_zbuf[base + k] = 0.0f;
      P.g_dists[base + k] = 0.0f;
      P.g_bary[3 * (base + k)] = gb[0];
      P.g_bary[3 * (base + k) + 1] = gb[1];
      P.g_bary[3 * (base + k) + 2] = gb[2];
    } else if (f >= 0) {
      const float d = P.dists[base + k];
      const float prob = frag_prob(d, isig);
      const float one_m = 1.0f - prob;
      const float others = R.nzero == 0 ? R.alpha_nz * frcp(one_m) : (R.nzero == 1 && R.kzero == k ? R.alpha_nz : 0.0f);
      float g_prob = g_alpha * (-others);
      float gz = 0.0f;
      float gb[3] = {0.f, 0.f, 0.f};
      if (!P.sil) {
        const int face = (int)(f - (int64_t)n * P.F);
        const float zi = (S.zfar - P.zbuf[base + k]) / (S.zfar - S.znear);
        const float E = expf((zi - R.zmax) / S.gamma);
        const float w = prob * E;
        PixGeom G;
        load_geom(P.srec, (uint32_t)face, G);
        const float* b = P.bary + 3 * (base + k);
        float col[3];
        PhongCache C;
        phong_fwd(S, n, G, b[0], b[1], b[2], col, C);
        const float g_w = ((g_num[0] * col[0] + g_num[1] * col[1]) + g_num[2] * col[2]) + g_den;
        const float gcol[3] = {g_num[0] * w, g_num[1] * w, g_num[2] * w};
        g_prob += g_w * E;
        float g_zi = (g_w * prob) * E * S.inv_gamma;
        if (k == R.kmax) g_zi += g_zmax;
        gz = -(g_zi * S.inv_zrange);
        float gP[3], gNn[3], gtex[3], guv[2];
        phong_bwd(S, G, C, gcol, gb, gP, gNn, gtex, guv);
        key = face;
        for (int c = 0; c < 3; ++c)
          for (int q = 0; q < 3; ++q) {
            row[3 * c + q] = b[c] * gP[q];
            row[9 + 3 * c + q] = b[c] * gNn[q];
            if (ACC == 27) row[18 + 3 * c + q] = b[c] * gtex[q];
          }
        if (S.tex_kind == 2) {
          if (P.gmap) tex_map_bwd(S, C.tap, gtex, P.gmap);
          if (P.guv) {
            const int32_t* fu = S.faces_uvs + 3 * (int64_t)face;
            for (int c = 0; c < 3; ++c) {
              if (guv[0] != 0.0f) atomicAdd(&P.guv[2 * (int64_t)fu[c]], b[c] * guv[0]);
              if (guv[1] != 0.0f) atomicAdd(&P.guv[2 * (int64_t)fu[c] + 1], b[c] * guv[1]);
            }
          }
        }
      } else if (k == R.kmax) {
        // silhouette: no depth dependence
      }
      float sp_, sq_;  // prob and 1 - prob, each accurate (sigmoid2): the derivative's factor
      sigmoid2((-d) * isig, sp_, sq_);
      const float gd = -((g_prob * (sp_ * sq_)) * isig);
      P.g_zbuf[base + k] = gz;
      P.g_dists[base + k] = gd;
      P.g_bary[3 * (base + k)] = gb[0];
      P.g_bary[3 * (base + k) + 1] = gb[1];
      P.g_bary[3 * (base + k) + 2] = gb[2];
    }
    // (empty slots: their zero gradients were written by coalesced fills before the launch; written
    // here one lane per pixel they were K-strided 4-B stores, most of this kernel's time at large K)
    if (!P.sil && S.light_kind == 0) seg_scatter<ACC>(key, row, P.gface, lrow[wave], lkey[wave]);
    else if (ACC == 27 && !P.sil) seg_scatter<ACC>(key, row, P.gface, lrow[wave], lkey[wave]);
  }
}

// ---------------------------------------------------------------------------
// Fused pose-optimiser loss (camera_pose_optimizer.py:257-276 Model.calc_loss):
//   sil_loss   = L1Loss()(silhouette, mask)               mean over all pixels
//   hloss      = HuberLoss(delta)(depth[mask], depth_ref[mask])   mean over the masked pixels
//   color_loss = MSELoss()(color, rgb_ref)                mean over all pixels x 3
//   total      = sil_loss + hloss + w_color * color_loss
// Forward: per-block partial sums (fixed-order wave / block reductions), then one block sums the
// partials in block order (deterministic). Backward: the elementwise gradients of the three
// means, scaled by the device scalar dL/dtotal (no host read).
// ---------------------------------------------------------------------------
struct PoseLossParams {
  const float* depth;
  const float* sil;
  const float* rgb;
  int64_t rgb_stride;  // floats between consecutive pixels' colours (3, or 4 for an RGBA view)
  const uint8_t* mask;
  const float* depth_ref;
  const float* rgb_ref;  // (npix, 3)
  int64_t npix;
  float delta, w_color;
};
#define MR_LOSS_BLOCKS 512

MR_DEV float huber_val(float d, float delta) {
  const float a = fabsf(d);
  return a < delta ? 0.5f * d * d : delta * (a - 0.5f * delta);
}
MR_DEV float huber_grad(float d, float delta) {
  return fabsf(d) < delta ? d : (d > 0.0f ? delta : (d < 0.0f ? -delta : 0.0f));
}
MR_DEV float block_sum_256(float v, float* sm) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  __syncthreads();
  const float t = ((sm[0] + sm[1]) + sm[2]) + sm[3];
  __syncthreads();
  return t;
}

__global__ void __launch_bounds__(256) k_pose_loss_partial(PoseLossParams P, float* __restrict__ part,
                                                           int* __restrict__ pcnt) {
  __shared__ float sm[4];
  float s_l1 = 0.0f, s_h = 0.0f, s_mse = 0.0f;
  int cnt = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < P.npix; i += (int64_t)gridDim.x * 256) {
    const bool m = P.mask[i] != 0;
    s_l1 += fabsf(P.sil[i] - (m ? 1.0f : 0.0f));
    if (m) {
      s_h += huber_val(P.depth[i] - P.depth_ref[i], P.delta);
      ++cnt;
    }
    const float* c = P.rgb + i * P.rgb_stride;
    const float* r = P.rgb_ref + 3 * i;
    const float d0 = c[0] - r[0], d1 = c[1] - r[1], d2 = c[2] - r[2];
    s_mse += (d0 * d0 + d1 * d1) + d2 * d2;
  }
  const float a = block_sum_256(s_l1, sm), b = block_sum_256(s_h, sm), c = block_sum_256(s_mse, sm);
  const float n = block_sum_256((float)cnt, sm);  // exact: <= 2^24 pixels per block
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x] = a;
    part[3 * blockIdx.x + 1] = b;
    part[3 * blockIdx.x + 2] = c;
    pcnt[blockIdx.x] = (int)n;
  }
}

// out: {total, sil_loss, hloss, color_loss}; count: the number of masked pixels (backward)
__global__ void __launch_bounds__(256) k_pose_loss_final(PoseLossParams P, const float* __restrict__ part,
                                                         const int* __restrict__ pcnt, int nb, float* __restrict__ out,
                                                         int64_t* __restrict__ count) {
  __shared__ float sm[4];
  float a = 0.0f, b = 0.0f, c = 0.0f;
  long long n = 0;
  for (int i = threadIdx.x; i < nb; i += 256) {
    a += part[3 * i];
    b += part[3 * i + 1];
    c += part[3 * i + 2];
    n += pcnt[i];
  }
  a = block_sum_256(a, sm);
  b = block_sum_256(b, sm);
  c = block_sum_256(c, sm);
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
  __shared__ long long sn[4];
  if ((threadIdx.x & 63) == 0) sn[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    const long long tn = ((sn[0] + sn[1]) + sn[2]) + sn[3];
    const float l1 = a / (float)P.npix;
    const float hl = b / (float)tn;  // an empty mask gives NaN, as torch's mean of nothing
    const float ms = c / (float)(3 * P.npix);
    out[0] = (l1 + hl) + P.w_color * ms;
    out[1] = l1;
    out[2] = hl;
    out[3] = ms;
    *count = tn;
  }
}

__global__ void __launch_bounds__(256) k_pose_loss_bwd(PoseLossParams P, const float* __restrict__ g_total,
                                                       const int64_t* __restrict__ count, float* __restrict__ g_depth,
                                                       float* __restrict__ g_sil, float* __restrict__ g_rgb) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= P.npix) return;
  const float g = *g_total;
  const bool m = P.mask[i] != 0;
  const float e = P.sil[i] - (m ? 1.0f : 0.0f);
  g_sil[i] = g * ((e > 0.0f ? 1.0f : (e < 0.0f ? -1.0f : 0.0f)) / (float)P.npix);
  g_depth[i] = m ? g * (huber_grad(P.depth[i] - P.depth_ref[i], P.delta) / (float)*count) : 0.0f;
  const float s = g * P.w_color * (2.0f / (float)(3 * P.npix));
  const float* c = P.rgb + i * P.rgb_stride;
  const float* r = P.rgb_ref + 3 * i;
  g_rgb[3 * i] = s * (c[0] - r[0]);
  g_rgb[3 * i + 1] = s * (c[1] - r[1]);
  g_rgb[3 * i + 2] = s * (c[2] - r[2]);
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* mr_last_error(void) { return g_err; }


int32_t mr_version(void) { return 3; }

int32_t mr_struct_size(int32_t which) {
  switch (which) {
    case 0: return (int32_t)sizeof(mr_view_t);
    case 1: return (int32_t)sizeof(mr_raster_settings_t);
    case 2: return (int32_t)sizeof(mr_shade_params_t);
    case 3: return (int32_t)sizeof(mr_mesh_t);
    default: return -1;
  }
}

static int check_settings(const mr_raster_settings_t* s) {
  if (!s) return set_err(MR_EINVAL, "settings is NULL");
  if (s->H <= 0 || s->W <= 0) return set_err(MR_EINVAL, "image size must be positive (got %d x %d)", s->H, s->W);
  if (s->H > 8192 || s->W > 8192) return set_err(MR_EUNSUPPORTED, "image size above 8192");
  if (s->faces_per_pixel < 1 || s->faces_per_pixel > MR_KMAX)
    return set_err(MR_EUNSUPPORTED, "faces_per_pixel=%d: supported range is [1, %d]", s->faces_per_pixel, MR_KMAX);
  if (!(s->blur_radius >= 0.0f) || !__builtin_isfinite(s->blur_radius))
    return set_err(MR_EINVAL, "blur_radius must be finite and >= 0");
  return MR_OK;
}

size_t mr_rasterize_meshes_workspace(int64_t num_meshes, int64_t total_faces, int32_t H, int32_t W,
                                     int32_t max_faces_per_bin) {
  const int64_t Ftot = total_faces > 0 ? total_faces : 1;
  BinGeom g = bin_geom(H, W, num_meshes, Ftot, max_faces_per_bin);
  return carve_raster_ws(nullptr, num_meshes, Ftot, H, W, g).bytes;
}

static SetupParams make_setup(const mr_raster_settings_t* s, const BinGeom& g, const RasterWS& w) {
  SetupParams P;
  P.H = s->H; P.W = s->W; P.TX = g.TX; P.TY = g.TY; P.T = g.T;
  P.bbox_pad = sqrtf(s->blur_radius);
  P.persp = s->perspective_correct;
  P.cull = s->cull_backfaces;
  P.clipz = s->clip_z != 0;
  P.zc = s->z_clip_value;
  P.NF = 0;  // set by the caller
  P.crec = w.crec;
  P.list_cap = g.list_cap;
  P.recs = w.recs;
  P.cnt = w.cnt;
  P.cur = w.cur;
  P.list = w.list;
  P.vtot = w.vtot;
  P.vbase = w.vbase;
  P.rects = w.rects;
  P.fv_out = nullptr;
  P.vff = nullptr;
  return P;
}

static int launch_scan(const RasterWS& w, int64_t N, const BinGeom& g, const int64_t* view_count, int64_t F,
                       hipStream_t st) {
  ScanParams P;
  P.T = g.T; P.mfpb = g.mfpb; P.list_cap = g.list_cap;
  P.cnt = w.cnt; P.vtot = w.vtot; P.start = w.start; P.cur = w.cur; P.vbase = w.vbase;
  P.tdone = w.tdone; P.vslot = w.vslot; P.stile = w.stile; P.units = w.units; P.ctr = w.ctr; P.tkey = w.tkey;
  P.view_count = view_count; P.F = F;
  MR_TIMED(KID_BIN_SCAN, st, (k_bin_scan<<<(unsigned)N, 1024, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_bin_scan");
  return MR_OK;
}

// The per-view binning applies to tile grids of <= MR_VIEW_TMAX tiles (<= 256 a side) and
// meshes of <= MR_VIEW_FMAX faces per view on average; else count -> scan -> fill.
static bool view_binning(const BinGeom& g, int64_t N, int64_t Ftot) {
  return g.T <= MR_VIEW_TMAX && g.TX <= 256 && g.TY <= 256 && Ftot <= (int64_t)MR_VIEW_FMAX * N;
}
extern "C++" {
// Background chunks per wave of k_bin_view's background workgroups (measured on the bench
// workloads, profiles/r2e_bg_ab.txt): beyond these the stores slow the view workgroups' binning
// more than they shorten the raster.
#ifndef MR_BG_CPW_RENDER
#define MR_BG_CPW_RENDER 8  // 5 KB chunks (depth, silhouette, RGB)
#endif
#ifndef MR_BG_CPW_FRAG
#define MR_BG_CPW_FRAG 4    // 7 KB chunks (PyTorch3D fragments)
#endif
#ifndef MR_VIEW_LDS
#define MR_VIEW_LDS 98304  // k_bin_view's LDS: the tile histogram + the list stage
#endif
static size_t view_lds_bytes() {
  static size_t b = 0;
  if (!b) {
    int dev = 0, mx = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&mx, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || mx <= 0) mx = 65536;
    b = std::min<size_t>((size_t)mx, MR_VIEW_LDS);
  }
  return b;
}
static int num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}
// Background chunks the k_bin_view launch takes over (chunks of 64 lanes x 4 pixels when W % 4 == 0,
// else 64 pixels); 0 when the views leave no CU idle.
static int64_t bg_chunks(int64_t N, int64_t sb, int H, int W, int mode) {
  const int64_t nbg = (int64_t)num_cus() - N - sb;
  if (nbg <= 0) return 0;
  const int64_t HW = (int64_t)H * W;
  const int64_t nchunks = N * ((W & 3) == 0 ? (HW / 4 + 63) / 64 : (HW + 63) / 64);
  return std::min<int64_t>(nchunks, nbg * 16 * (mode == 0 ? MR_BG_CPW_FRAG : MR_BG_CPW_RENDER));
}
// MODE >= 0 with Pf: the fused K = 1 raster follows, and the CUs the views leave idle stream the
// first chunks of its background (Pf->fill_first).
template <int MODE = -1, int CH = 3>
static int launch_bin_view(const SetupParams& SP, const RasterWS& w, const BinGeom& g, int64_t N, const int64_t* first,
                           const int64_t* view_count, int64_t F, bool ranges, hipStream_t st,
                           const ShadeParams* S = nullptr, FwdParams* Pf = nullptr) {
  ViewBinParams V;
  memset(&V, 0, sizeof(V));
  V.ranges = ranges ? 1 : 0;
  V.nviews = (int)N;
  int64_t sb = 0;
  if (S) {
    V.S = *S;
    V.srec = w.srec;
    V.Fs = F;
    sb = ceil_div(F, 1024);
  }
  V.nsrec_wg = (int)sb;
  V.T = g.T; V.TX = g.TX; V.mfpb = g.mfpb; V.clipz = SP.clipz;
  V.list_cap = g.list_cap; V.NF = SP.NF;
  V.rects = w.rects; V.first = first; V.view_count = view_count; V.F = F;
  V.cnt = w.cnt; V.start = w.start; V.vbase = w.vbase; V.tdone = w.tdone; V.vslot = w.vslot; V.stile = w.stile;
  V.units = w.units; V.ctr = w.ctr; V.tkey = w.tkey; V.list = w.list;
  const size_t hist_b = sizeof(int) * (size_t)((g.T + (g.T >> 6) + 3) & ~3);
  const size_t shm = std::max(hist_b, view_lds_bytes());
  V.stage_cap = (int)((shm - hist_b) / sizeof(int));
  if constexpr (MODE >= 0) {
    const int64_t nbg = (int64_t)num_cus() - N - sb;
    if (Pf && nbg > 0 && (MODE != 0 || Pf->K == 1)) {
      Pf->fill_first = (int)bg_chunks(N, sb, Pf->H, Pf->W, MODE);
      MR_TIMED(KID_BIN_VIEW, st, (k_bin_view<MODE, CH><<<(unsigned)(N + sb + nbg), 1024, shm, st>>>(V, *Pf)));
      MR_CHECK_LAUNCH("k_bin_view");
      return MR_OK;
    }
  }
  MR_TIMED(KID_BIN_VIEW, st, (k_bin_view<<<(unsigned)(N + sb), 1024, shm, st>>>(V)));
  MR_CHECK_LAUNCH("k_bin_view");
  return MR_OK;
}
}  // extern "C++"

int64_t mr_binning_background_pixels(int64_t N, int64_t F, int32_t H, int32_t W, int32_t mode) {
  if (N <= 0 || H <= 0 || W <= 0) return 0;
  BinGeom g = bin_geom(H, W, N, N * (F > 0 ? F : 1), 0);
  if (!view_binning(g, N, N * (F > 0 ? F : 1))) return 0;
  const int64_t sb = mode == 1 ? ceil_div(F, 1024) : 0;
  const int64_t px = bg_chunks(N, sb, H, W, mode) * ((W & 3) == 0 ? 256 : 64);
  return std::min<int64_t>(px, N * (int64_t)H * W);
}

int32_t mr_rasterize_meshes(const float* face_verts, const int64_t* first, const int64_t* count, int64_t N,
                            int64_t Ftot, const mr_raster_settings_t* s, int64_t* p2f, float* zbuf, float* bary,
                            float* dists, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "num_meshes must be in [1, 65535] (got %lld)", (long long)N);
  if (Ftot < 0 || Ftot >= (1ll << 31)) return set_err(MR_EINVAL, "total_faces out of range");
  if ((int64_t)N * s->H * s->W >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "N*H*W >= 2^31");
  if (!p2f || !zbuf || !bary || !dists || !first || !count || (Ftot > 0 && !face_verts))
    return set_err(MR_EINVAL, "NULL tensor argument");
  hipStream_t st = (hipStream_t)stream;
  const int64_t Fb = Ftot > 0 ? Ftot : 1;
  BinGeom g = bin_geom(s->H, s->W, N, Fb, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws(ws, N, Fb, s->H, s->W, g);
  if (ws_bytes < w.bytes) return set_err(MR_EWORKSPACE, "workspace too small: %zu < %zu", ws_bytes, w.bytes);
  const bool vpath = view_binning(g, N, Fb);
  // per-view path: k_bin_rect_fv clears the counters
  if ((!vpath || Ftot == 0) && hipMemsetAsync(w.ctr, 0, zero_bytes(N, g, vpath), st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  SetupParams SP = make_setup(s, g, w);
  FwdParams P = make_fwd(s, g, w, N, first, 0, Fb);
  P.p2f = p2f; P.zbuf = zbuf; P.bary = bary; P.dists = dists;
  P.view_count = count;
  const bool lds = g.T <= MR_LDS_HIST;
  const size_t shm = lds ? sizeof(int) * (size_t)g.T : 0;
  SP.NF = Fb;
  if (vpath) {
    if (Ftot > 0) {
      if (SP.clipz) MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_fv<true><<<ceil_div(Ftot, 256), 256, 0, st>>>(SP, face_verts, Ftot, w.ctr)));
      else MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_fv<false><<<ceil_div(Ftot, 256), 256, 0, st>>>(SP, face_verts, Ftot, w.ctr)));
      MR_CHECK_LAUNCH("k_bin_rect_fv");
    }
    if (s->faces_per_pixel > 1) {
      if ((rc = launch_bin_view(SP, w, g, N, first, count, 0, true, st))) return rc;
      return launch_raster_k(P, g, N, st);
    }
    if ((rc = launch_bin_view<0, 3>(SP, w, g, N, first, count, 0, false, st, nullptr, &P))) return rc;
    return launch_raster_and_shade<0, 3>(P, g, N, st, s->clip_z != 0);
  }
  const int fvb = ceil_div(Ftot, 256 * MR_FV_FPT);
  if (Ftot > 0) {
    if (lds) MR_TIMED(KID_BIN_COUNT, st, (k_bin_count_fv<true><<<fvb, 256, shm, st>>>(SP, face_verts, Ftot, first, N)));
    else MR_TIMED(KID_BIN_COUNT, st, (k_bin_count_fv<false><<<fvb, 256, 0, st>>>(SP, face_verts, Ftot, first, N)));
    MR_CHECK_LAUNCH("k_bin_count_fv");
  }
  if ((rc = launch_scan(w, N, g, count, 0, st))) return rc;
  if (Ftot > 0) {
    if (lds) MR_TIMED(KID_BIN_FILL, st, (k_bin_fill_fv<true><<<fvb, 256, shm, st>>>(SP, Ftot, first, N)));
    else MR_TIMED(KID_BIN_FILL, st, (k_bin_fill_fv<false><<<fvb, 256, 0, st>>>(SP, Ftot, first, N)));
    MR_CHECK_LAUNCH("k_bin_fill_fv");
  }
  if (s->faces_per_pixel > 1) return launch_raster_k(P, g, N, st);
  return launch_raster_and_shade<0, 3>(P, g, N, st, s->clip_z != 0);
}

// View records from PyTorch3D poses, and the shared-mesh face ranges (first[n] = n F, count F)
// the count -> scan fallback of mr_rasterize_meshes_world reads.
__global__ void __launch_bounds__(256) k_views_from_poses(CvPoses C, int64_t N, int64_t F, int64_t* __restrict__ first,
                                                          int64_t* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < N * 16) C.out[i] = cv_view_elem(C, i >> 4, (int)(i & 15));
  if (i < N) {
    first[i] = i * F;
    count[i] = F;
  }
}

size_t mr_rasterize_meshes_world_workspace(int64_t N, int64_t F, int32_t H, int32_t W, int32_t max_faces_per_bin) {
  return align_up(mr_rasterize_meshes_workspace(N, N * F, H, W, max_faces_per_bin), 256) +
         align_up(sizeof(int64_t) * 2 * (size_t)(N > 0 ? N : 1), 256);
}

// MeshRasterizer.forward of one mesh shared by N views: transform + rasterize. On the per-view
// binning path the projection happens in k_bin_rect_world (record, tile rectangle and face_verts
// row of each (view, face) from one thread; the counters cleared by its row 0), so the step is
// k_bin_rect_world -> k_bin_view -> k_tile_raster -> k_shade<0> with no projection launch, memset
// or host-side view packing. Else: view records, mr_project_faces, mr_rasterize_meshes.
int32_t mr_rasterize_meshes_world(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                                  const mr_poses_t* poses, int64_t N, const mr_raster_settings_t* s,
                                  mr_view_t* views_out, float* face_verts, int64_t* p2f, float* zbuf, float* bary,
                                  float* dists, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "N must be in [1, 65535] (got %lld)", (long long)N);
  if (F < 0 || V < 0 || N * F >= (1ll << 30)) return set_err(MR_EINVAL, "F / V out of range");
  if ((int64_t)N * s->H * s->W >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "N*H*W >= 2^31");
  if (!poses || !poses->R || !poses->T || !poses->intr || !views_out || !p2f || !zbuf || !bary || !dists ||
      (F > 0 && (!verts || !faces || !face_verts)))
    return set_err(MR_EINVAL, "NULL argument");
  if (poses->R_stride < 0 || poses->T_stride < 0 || poses->intr_stride < 0) return set_err(MR_EINVAL, "negative stride");
  const size_t need = mr_rasterize_meshes_world_workspace(N, F, s->H, s->W, s->max_faces_per_bin);
  if (ws_bytes < need) return set_err(MR_EWORKSPACE, "workspace too small: %zu < %zu", ws_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  CvPoses C;
  C.R = poses->R; C.sR = poses->R_stride; C.t = poses->T; C.sT = poses->T_stride;
  C.intr = poses->intr; C.sI = poses->intr_stride; C.out = (float*)views_out; C.opencv = 0;
  const int64_t Fb = N * F > 0 ? N * F : 1;
  BinGeom g = bin_geom(s->H, s->W, N, Fb, s->max_faces_per_bin);
  if (F == 0 || !view_binning(g, N, Fb)) {
    const size_t rws = align_up(mr_rasterize_meshes_workspace(N, N * F, s->H, s->W, s->max_faces_per_bin), 256);
    int64_t* first = (int64_t*)((char*)ws + rws);
    k_views_from_poses<<<ceil_div(N * 16, 256), 256, 0, st>>>(C, N, F, first, first + N);
    MR_CHECK_LAUNCH("k_views_from_poses");
    if ((rc = mr_project_faces(verts, V, faces, F, views_out, N, face_verts, stream))) return rc;
    return mr_rasterize_meshes(face_verts, first, first + N, N, N * F, s, p2f, zbuf, bary, dists, ws, rws, stream);
  }
  RasterWS w = carve_raster_ws(ws, N, Fb, s->H, s->W, g);
  SetupParams SP = make_setup(s, g, w);
  SP.NF = Fb;
  SP.fv_out = face_verts;
  FwdParams P = make_fwd(s, g, w, N, nullptr, F, Fb);
  P.p2f = p2f; P.zbuf = zbuf; P.bary = bary; P.dists = dists;
  NormalsArgs NA;
  memset(&NA, 0, sizeof(NA));
  dim3 rgrid((unsigned)ceil_div(F, 256), (unsigned)N + 1);  // row 0: counter clear
  if (SP.clipz) MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_world<true><<<rgrid, 256, 0, st>>>(SP, verts, faces, F, (const ViewRec*)views_out, NA, w.ctr, C)));
  else MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_world<false><<<rgrid, 256, 0, st>>>(SP, verts, faces, F, (const ViewRec*)views_out, NA, w.ctr, C)));
  MR_CHECK_LAUNCH("k_bin_rect_world");
  if (s->faces_per_pixel > 1) {
    if ((rc = launch_bin_view(SP, w, g, N, nullptr, nullptr, F, true, st))) return rc;
    return launch_raster_k(P, g, N, st);
  }
  if ((rc = launch_bin_view<0, 3>(SP, w, g, N, nullptr, nullptr, F, false, st, nullptr, &P))) return rc;
  return launch_raster_and_shade<0, 3>(P, g, N, st, s->clip_z != 0);
}

int32_t mr_rasterize_meshes_backward(const float* fv, const int64_t* p2f, const float* gz, const float* gb,
                                     const float* gd, int64_t N, int64_t Ftot, const mr_raster_settings_t* s,
                                     float* gfv, void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "num_meshes out of range");
  if (!p2f || !gfv) return set_err(MR_EINVAL, "NULL tensor argument");
  hipStream_t st = (hipStream_t)stream;
  if (Ftot > 0 && hipMemsetAsync(gfv, 0, sizeof(float) * 9 * (size_t)Ftot, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  if (Ftot == 0 || (!gz && !gb && !gd)) return MR_OK;  // NULL gradients are zero
  RasterBwdParams P;
  P.N = (int)N; P.H = s->H; P.W = s->W; P.NBX = ceil_div(s->W, MR_BT); P.K = s->faces_per_pixel;
  P.persp = s->perspective_correct; P.clipb = s->clip_barycentric_coords;
  P.cull = s->cull_backfaces; P.clipz = s->clip_z != 0; P.zc = s->z_clip_value;
  P.blur = s->blur_radius; P.bbox_pad = sqrtf(s->blur_radius);
  P.fv = fv; P.p2f = p2f; P.gz = gz; P.gb = gb; P.gd = gd; P.gfv = gfv;
  const int64_t nslots = N * (int64_t)s->H * s->W * s->faces_per_pixel;
  MR_TIMED(KID_RASTER_BWD, st, (k_raster_bwd_slots<<<(unsigned)((nslots + 255) / 256), 256, 0, st>>>(P, nslots)));
  MR_CHECK_LAUNCH("k_raster_bwd");
  return MR_OK;
}

int32_t mr_project_faces(const float* verts, int64_t V, const int32_t* faces, int64_t F, const mr_view_t* views,
                         int64_t N, float* fv, void* stream) {
  if (N <= 0 || N > 65535 || F < 0 || V < 0) return set_err(MR_EINVAL, "bad sizes");
  if (F == 0) return MR_OK;
  if (!verts || !faces || !views || !fv) return set_err(MR_EINVAL, "NULL argument");
  dim3 grid(ceil_div(F, 256), (unsigned)N);
  MR_TIMED(KID_PROJECT, (hipStream_t)stream, (k_project_faces<<<grid, 256, 0, (hipStream_t)stream>>>(verts, faces, F, (const ViewRec*)views, fv, nullptr)));
  MR_CHECK_LAUNCH("k_project_faces");
  return MR_OK;
}

int32_t mr_project_faces_meshes(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                                const int64_t* view_face_first, int64_t max_view_faces, const mr_view_t* views,
                                int64_t N, float* fv, void* stream) {
  if (N <= 0 || N > 65535 || F < 0 || V < 0 || max_view_faces < 0) return set_err(MR_EINVAL, "bad sizes");
  if (F == 0 || max_view_faces == 0) return MR_OK;
  if (!verts || !faces || !views || !fv || !view_face_first) return set_err(MR_EINVAL, "NULL argument");
  dim3 grid(ceil_div(max_view_faces, 256), (unsigned)N);
  MR_TIMED(KID_PROJECT, (hipStream_t)stream, (k_project_faces<<<grid, 256, 0, (hipStream_t)stream>>>(verts, faces, F, (const ViewRec*)views, fv, view_face_first)));
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
  MR_TIMED(KID_PROJECT_BWD, st, (k_project_faces_bwd<<<grid, 256, 0, st>>>(verts, V, F, ptr, adj, (const ViewRec*)views, gfv, gverts, gviews, nullptr)));
  MR_CHECK_LAUNCH("k_project_faces_bwd");
  return MR_OK;
}

int32_t mr_project_faces_meshes_backward(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                                         const int32_t* ptr, const int32_t* adj, const int64_t* view_vert_first,
                                         int64_t max_view_verts, const mr_view_t* views, int64_t N, const float* gfv,
                                         float* gverts, float* gviews, void* stream) {
  (void)faces;
  if (N <= 0 || N > 65535 || F < 0 || V < 0 || max_view_verts < 0) return set_err(MR_EINVAL, "bad sizes");
  if (!view_vert_first) return set_err(MR_EINVAL, "NULL argument");
  hipStream_t st = (hipStream_t)stream;
  if (V > 0 && hipMemsetAsync(gverts, 0, sizeof(float) * 3 * (size_t)V, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  if (hipMemsetAsync(gviews, 0, sizeof(float) * 12 * (size_t)N, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  if (V == 0 || max_view_verts == 0) return MR_OK;
  dim3 grid(ceil_div(max_view_verts, 256), (unsigned)N);
  MR_TIMED(KID_PROJECT_BWD, st, (k_project_faces_bwd<<<grid, 256, 0, st>>>(verts, V, F, ptr, adj, (const ViewRec*)views, gfv, gverts, gviews, view_vert_first)));
  MR_CHECK_LAUNCH("k_project_faces_bwd");
  return MR_OK;
}

// OpenCV pose -> view records, and the conversion's chain rule (one thread per output float).
__global__ void __launch_bounds__(256) k_views_from_opencv(const float* __restrict__ R, int64_t sR,
                                                           const float* __restrict__ t, int64_t sT,
                                                           const float* __restrict__ intr, int64_t sI, int64_t N,
                                                           float* __restrict__ views) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * 16) return;
  const int64_t n = i >> 4;
  const int k = (int)(i & 15);
  float v;
  if (k < 9) {  // R_p3d[a][b] = R_cv[b][a] * s[b], s = (-1, -1, 1)
    const int a = k / 3, b = k - 3 * a;
    v = R[n * sR + 3 * b + a];
    if (b < 2) v = -v;
  } else if (k < 12) {
    v = t[n * sT + (k - 9)];
    if (k < 11) v = -v;
  } else {
    v = intr[n * sI + (k - 12)];
  }
  views[i] = v;
}

__global__ void __launch_bounds__(256) k_view_grads_to_opencv(const float* __restrict__ g, int64_t N,
                                                              float* __restrict__ gR, float* __restrict__ gt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * 12) return;
  const int64_t n = i / 12;
  const int k = (int)(i - n * 12);
  if (k < 9) {  // dL/dR_cv[b][a] = dL/dR_p3d[a][b] * s[b]
    const int b = k / 3, a = k - 3 * b;
    const float v = g[n * 12 + 3 * a + b];
    gR[n * 9 + k] = b < 2 ? -v : v;
  } else {
    const float v = g[n * 12 + k];
    gt[n * 3 + (k - 9)] = k < 11 ? -v : v;
  }
}

int32_t mr_views_from_opencv(const float* R_cv, int64_t R_stride, const float* t_cv, int64_t t_stride,
                             const float* intr, int64_t intr_stride, int64_t N, mr_view_t* views, void* stream) {
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "N out of range");
  if (!R_cv || !t_cv || !intr || !views) return set_err(MR_EINVAL, "NULL argument");
  if (R_stride < 0 || t_stride < 0 || intr_stride < 0) return set_err(MR_EINVAL, "negative stride");
  hipStream_t st = (hipStream_t)stream;
  k_views_from_opencv<<<ceil_div(N * 16, 256), 256, 0, st>>>(R_cv, R_stride, t_cv, t_stride, intr, intr_stride, N,
                                                            (float*)views);
  MR_CHECK_LAUNCH("k_views_from_opencv");
  return MR_OK;
}

int32_t mr_view_grads_to_opencv(const float* grad_views, int64_t N, float* grad_R_cv, float* grad_t_cv,
                                void* stream) {
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "N out of range");
  if (!grad_views || !grad_R_cv || !grad_t_cv) return set_err(MR_EINVAL, "NULL argument");
  hipStream_t st = (hipStream_t)stream;
  k_view_grads_to_opencv<<<ceil_div(N * 12, 256), 256, 0, st>>>(grad_views, N, grad_R_cv, grad_t_cv);
  MR_CHECK_LAUNCH("k_view_grads_to_opencv");
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
  S.tex8 = (m->tex_u8 && m->tex_lut) ? (const uchar4*)m->tex_u8 : nullptr;
  S.tex_lut = m->tex_lut;
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
  S.inv_sigma_rgb = 1.0f / sp->sigma_rgb;
  S.inv_gamma = 1.0f / sp->gamma;
  S.inv_zrange = 1.0f / (sp->zfar - sp->znear);
  S.inv_sigma_sil = 1.0f / sp->sigma_sil;
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
  return carve_raster_ws(nullptr, N, N * F, H, W, g, F).bytes;
}
size_t mr_render_workspace_meshes(int64_t N, int64_t F, int32_t H, int32_t W, int32_t max_faces_per_bin) {
  BinGeom g = bin_geom(H, W, N, F, max_faces_per_bin);
  return carve_raster_ws(nullptr, N, F, H, W, g, F).bytes;
}

static int32_t render_forward(const mr_mesh_t* m, const mr_view_t* views, int64_t N, const float* cc, int64_t ncc,
                              const mr_raster_settings_t* s, const mr_shade_params_t* sp, float* depth, float* sil,
                              float* rgb, int32_t* p2f32, void* ws, size_t ws_bytes, void* stream, const CvPoses& C);
int32_t mr_render_forward(const mr_mesh_t* m, const mr_view_t* views, int64_t N, const float* cc, int64_t ncc,
                          const mr_raster_settings_t* s, const mr_shade_params_t* sp, float* depth, float* sil,
                          float* rgb, int32_t* p2f32, void* ws, size_t ws_bytes, void* stream) {
  CvPoses C;
  memset(&C, 0, sizeof(C));
  return render_forward(m, views, N, cc, ncc, s, sp, depth, sil, rgb, p2f32, ws, ws_bytes, stream, C);
}
int32_t mr_render_forward_opencv(const mr_mesh_t* m, const mr_opencv_poses_t* poses, mr_view_t* views_out, int64_t N,
                                 const float* cc, int64_t ncc, const mr_raster_settings_t* s,
                                 const mr_shade_params_t* sp, float* depth, float* sil, float* rgb, int32_t* p2f32,
                                 void* ws, size_t ws_bytes, void* stream) {
  if (!poses || !poses->R || !poses->t || !poses->intr || !views_out) return set_err(MR_EINVAL, "NULL pose argument");
  if (poses->R_stride < 0 || poses->t_stride < 0 || poses->intr_stride < 0) return set_err(MR_EINVAL, "negative stride");
  CvPoses C;
  C.R = poses->R; C.sR = poses->R_stride; C.t = poses->t; C.sT = poses->t_stride;
  C.intr = poses->intr; C.sI = poses->intr_stride; C.out = (float*)views_out;
  C.opencv = 1;
  return render_forward(m, views_out, N, cc, ncc, s, sp, depth, sil, rgb, p2f32, ws, ws_bytes, stream, C);
}
static int32_t render_forward(const mr_mesh_t* m, const mr_view_t* views, int64_t N, const float* cc, int64_t ncc,
                              const mr_raster_settings_t* s, const mr_shade_params_t* sp, float* depth, float* sil,
                              float* rgb, int32_t* p2f32, void* ws, size_t ws_bytes, void* stream, const CvPoses& C) {
  int rc = check_settings(s);
  if (rc) return rc;
  rc = check_mesh(m, sp);
  if (rc) return rc;
  if (s->faces_per_pixel != 1) return set_err(MR_EUNSUPPORTED, "the fused render path is K = 1 (faces_per_pixel=%d)", s->faces_per_pixel);
  if (sp->out_flags & MR_OUT_HARD) return set_err(MR_EUNSUPPORTED, "hard_rgb_blend runs on the fragment-shader path (mr_shade_fragments_*)");
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "N out of range");
  // record ids: n*F + f for one shared mesh; the union face id for distinct meshes
  const bool multi = m->view_face_first != nullptr;
  const int64_t NF = multi ? m->F : N * m->F, maxvf = multi ? m->max_view_faces : m->F;
  if (multi && (!m->view_face_count || maxvf <= 0)) return set_err(MR_EINVAL, "distinct meshes: face ranges missing");
  if (NF >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "N*F >= 2^31");
  if ((int64_t)N * s->H * s->W >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "N*H*W >= 2^31");
  if (!views) return set_err(MR_EINVAL, "NULL views");
  if ((sp->out_flags & MR_OUT_DEPTH) && !depth) return set_err(MR_EINVAL, "depth output NULL");
  if ((sp->out_flags & MR_OUT_SIL) && !sil) return set_err(MR_EINVAL, "silhouette output NULL");
  if ((sp->out_flags & MR_OUT_RGB) && !rgb) return set_err(MR_EINVAL, "rgb output NULL");
  if (sp->light_kind == 0 && (!cc || (ncc != 1 && ncc != N))) return set_err(MR_EINVAL, "camera centres");
  hipStream_t st = (hipStream_t)stream;
  BinGeom g = bin_geom(s->H, s->W, N, NF, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws(ws, N, NF, s->H, s->W, g, m->F);
  if (ws_bytes < w.bytes) return set_err(MR_EWORKSPACE, "workspace too small: %zu < %zu", ws_bytes, w.bytes);
  SetupParams SP = make_setup(s, g, w);
  SP.NF = NF;
  SP.vff = m->view_face_first;
  FwdParams P = make_fwd(s, g, w, N, m->view_face_first, multi ? 0 : m->F, NF);
  P.view_count = m->view_face_count;
  P.S = make_shade(m, sp, cc, ncc);
  P.srec = w.srec;
  P.out_flags = sp->out_flags;
  P.depth = depth;
  P.sil = sil;
  P.rgb = rgb;
  P.p2f32 = p2f32;
  const bool vpath = view_binning(g, N, NF);
  const int64_t nzero = (int64_t)(zero_bytes(N, g, vpath) / sizeof(int));
  // normals computed here (the mesh's vnormals_out) or passed in (vnormals)
  const int64_t vb = (sp->light_kind == 0 && m->vnormals_out) ? ceil_div(m->V, 256) : 0;
  if (vb) {
    if (!m->vraw_out) return set_err(MR_EINVAL, "vnormals_out without vraw_out");
    P.S.vnormals = m->vnormals_out;
  }
  if (vpath) {
    NormalsArgs NA;
    NA.V = m->V; NA.ptr = m->vadj_ptr; NA.adj = m->vadj;
    NA.vn = vb ? m->vnormals_out : nullptr;
    NA.vraw = m->vraw_out;
    NA.zero4 = (float4*)w.grows;
    NA.nzero4 = (27 * m->F + 3) / 4;
    const int64_t bx = std::max<int64_t>(ceil_div(maxvf, 256), ceil_div(m->V, 256));
    dim3 rgrid((unsigned)(bx > 0 ? bx : 1), (unsigned)N + 1);  // row 0: normals + counter clear
    if (SP.clipz) MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_world<true><<<rgrid, 256, 0, st>>>(SP, m->verts, m->faces, m->F, (const ViewRec*)views, NA, w.ctr, C)));
    else MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_world<false><<<rgrid, 256, 0, st>>>(SP, m->verts, m->faces, m->F, (const ViewRec*)views, NA, w.ctr, C)));
    MR_CHECK_LAUNCH("k_bin_rect_world");
    if (sp->rgb_channels == 4) {
      if ((rc = launch_bin_view<1, 4>(SP, w, g, N, m->view_face_first, m->view_face_count, m->F, false, st, &P.S, &P))) return rc;
      return launch_raster_and_shade<1, 4>(P, g, N, st, s->clip_z != 0);
    }
    if ((rc = launch_bin_view<1, 3>(SP, w, g, N, m->view_face_first, m->view_face_count, m->F, false, st, &P.S, &P))) return rc;
    return launch_raster_and_shade<1, 3>(P, g, N, st, s->clip_z != 0);
  }
  if (hipMemsetAsync(w.grows, 0, sizeof(float) * 27 * (size_t)m->F, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  if (C.R) {  // count -> scan path: the view records first
    k_views_from_opencv<<<ceil_div(N * 16, 256), 256, 0, st>>>(C.R, C.sR, C.t, C.sT, C.intr, C.sI, N, C.out);
    MR_CHECK_LAUNCH("k_views_from_opencv");
  }
  MR_TIMED(KID_SETUP, st, (k_setup_zero<<<(unsigned)(vb + ceil_div(nzero, 1024)), 256, 0, st>>>(m->verts, m->V, m->faces, m->vadj_ptr, m->vadj, m->vnormals_out, m->vraw_out, vb, w.ctr, nzero)));
  MR_CHECK_LAUNCH("k_setup_zero");
  const int fpt = MR_BIN_FPT;
  dim3 sgrid(ceil_div(maxvf, 256 * fpt), (unsigned)N);
  dim3 fgrid(ceil_div(m->F, 256 * fpt), (unsigned)N + 1);  // + the ShadeRec row (every face of the mesh(es))
  const bool lds = g.T <= MR_LDS_HIST;
  const size_t shm = lds ? sizeof(int) * (size_t)g.T : 0;
  if (lds)
    MR_TIMED(KID_BIN_COUNT, st, (k_bin_count_world<true><<<sgrid, 256, shm, st>>>(SP, m->verts, m->faces, m->F, (const ViewRec*)views, fpt)));
  else
    MR_TIMED(KID_BIN_COUNT, st, (k_bin_count_world<false><<<sgrid, 256, 0, st>>>(SP, m->verts, m->faces, m->F, (const ViewRec*)views, fpt)));
  MR_CHECK_LAUNCH("k_bin_count_world");
  if ((rc = launch_scan(w, N, g, m->view_face_count, m->F, st))) return rc;
  if (lds)
    MR_TIMED(KID_BIN_FILL, st, (k_bin_fill_world<true><<<fgrid, 256, shm, st>>>(SP, m->F, fpt, (int)N, P.S, w.srec)));
  else
    MR_TIMED(KID_BIN_FILL, st, (k_bin_fill_world<false><<<fgrid, 256, 0, st>>>(SP, m->F, fpt, (int)N, P.S, w.srec)));
  MR_CHECK_LAUNCH("k_bin_fill_world");
  if (sp->rgb_channels == 4) return launch_raster_and_shade<1, 4>(P, g, N, st, s->clip_z != 0);
  return launch_raster_and_shade<1, 3>(P, g, N, st, s->clip_z != 0);
}

size_t mr_render_backward_workspace(int64_t N, int64_t V, int64_t F, int32_t H, int32_t W) {
  const int64_t NT = N * (int64_t)ceil_div(W, MR_TS) * ceil_div(H, MR_TS);
  (void)F;  // the face-gradient rows are in the forward's workspace
  size_t off = align_up(sizeof(float) * 3 * (size_t)V, 256);                   // gnu
  off = align_up(off + sizeof(float) * 12 * (size_t)NT, 256);                  // rt_part
  return off;
}

static int32_t render_backward(const mr_mesh_t* m, const float* vraw, const mr_view_t* views, int64_t N,
                               const float* cc, int64_t ncc, const mr_raster_settings_t* s,
                               const mr_shade_params_t* sp, const float* gD, const float* gS, const float* gRGB,
                               const void* fws, void* bws, size_t bws_bytes, float* gverts, float* gviews,
                               float* gRcv, float* gtcv, float* gcol, void* stream);

int32_t mr_render_backward(const mr_mesh_t* m, const float* vraw, const mr_view_t* views, int64_t N, const float* cc,
                           int64_t ncc, const mr_raster_settings_t* s, const mr_shade_params_t* sp,
                           const float* gD, const float* gS, const float* gRGB, const void* fws, void* bws,
                           size_t bws_bytes, float* gverts, float* gviews, float* gcol, void* stream) {
  if (!gviews) return set_err(MR_EINVAL, "NULL argument");
  return render_backward(m, vraw, views, N, cc, ncc, s, sp, gD, gS, gRGB, fws, bws, bws_bytes, gverts, gviews,
                         nullptr, nullptr, gcol, stream);
}

int32_t mr_render_backward_opencv(const mr_mesh_t* m, const float* vraw, const mr_view_t* views, int64_t N,
                                  const float* cc, int64_t ncc, const mr_raster_settings_t* s,
                                  const mr_shade_params_t* sp, const float* gD, const float* gS, const float* gRGB,
                                  const void* fws, void* bws, size_t bws_bytes, float* gverts, float* grad_R_cv,
                                  float* grad_t_cv, float* gcol, void* stream) {
  if (!grad_R_cv || !grad_t_cv) return set_err(MR_EINVAL, "NULL argument");
  return render_backward(m, vraw, views, N, cc, ncc, s, sp, gD, gS, gRGB, fws, bws, bws_bytes, gverts, nullptr,
                         grad_R_cv, grad_t_cv, gcol, stream);
}

static int32_t render_backward(const mr_mesh_t* m, const float* vraw, const mr_view_t* views, int64_t N,
                               const float* cc, int64_t ncc, const mr_raster_settings_t* s,
                               const mr_shade_params_t* sp, const float* gD, const float* gS, const float* gRGB,
                               const void* fws, void* bws, size_t bws_bytes, float* gverts, float* gviews,
                               float* gRcv, float* gtcv, float* gcol, void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  rc = check_mesh(m, sp);
  if (rc) return rc;
  if (s->faces_per_pixel != 1) return set_err(MR_EUNSUPPORTED, "the fused render path is K = 1 (faces_per_pixel=%d)", s->faces_per_pixel);
  if (sp->out_flags & MR_OUT_HARD) return set_err(MR_EUNSUPPORTED, "hard_rgb_blend runs on the fragment-shader path (mr_shade_fragments_*)");
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "N out of range");
  if (!fws || !bws || !gverts || (!gviews && !(gRcv && gtcv))) return set_err(MR_EINVAL, "NULL argument");
  if (sp->light_kind == 0 && !vraw) return set_err(MR_EINVAL, "raw vertex normals required");
  const size_t need = mr_render_backward_workspace(N, m->V, m->F, s->H, s->W);
  if (bws_bytes < need) return set_err(MR_EWORKSPACE, "backward workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const bool multi = m->view_face_first != nullptr;  // distinct meshes: record id = union face id
  const int64_t NF = multi ? m->F : N * m->F;
  BinGeom g = bin_geom(s->H, s->W, N, NF, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws((void*)fws, N, NF, s->H, s->W, g, m->F);
  const bool vcol = m->tex_kind == 1;
  const int ACC = vcol ? 27 : 18;
  const int64_t NT = N * (int64_t)g.T;
  char* b = (char*)bws;
  size_t off = 0;
  float* gnu = (float*)(b + off);
  off = align_up(off + sizeof(float) * 3 * (size_t)m->V, 256);
  float* rt_part = (float*)(b + off);
  // the per-face gradient rows live in the forward's workspace, which the forward cleared; a
  // second backward over the same forward (MR_GRAD_ROWS_CLEARED not set) clears them again
  float* gface = w.grows;
  if (!(sp->out_flags & MR_GRAD_ROWS_CLEARED) &&
      hipMemsetAsync(gface, 0, sizeof(float) * ACC * (size_t)m->F, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  RenderBwdParams P;
  memset(&P, 0, sizeof(P));
  P.N = (int)N; P.H = s->H; P.W = s->W; P.TX = g.TX; P.T = g.T;
  P.blur = s->blur_radius; P.bbox_pad = sqrtf(s->blur_radius);
  P.persp = s->perspective_correct; P.clipb = s->clip_barycentric_coords;
  P.recs = w.recs;
  P.ctr = w.ctr;
  P.sface = w.sface;
  P.stile = w.stile;
  P.vslot = w.vslot;
  P.gD = (sp->out_flags & MR_OUT_DEPTH) ? gD : nullptr;
  P.gS = (sp->out_flags & MR_OUT_SIL) ? gS : nullptr;
  P.gRGB = (sp->out_flags & MR_OUT_RGB) ? gRGB : nullptr;
  P.rgb_ch = sp->rgb_channels;
  P.sil_rgba = (sp->out_flags & MR_OUT_SIL_RGBA) ? 1 : 0;
  P.S = make_shade(m, sp, cc, ncc);
  P.srec = w.srec;
  P.F = multi ? 0 : m->F;
  P.NF = NF;
  P.crec = w.crec;
  P.zc = s->z_clip_value;
  P.views = (const ViewRec*)views;
  P.gface = gface;
  P.rt_part = rt_part;
  P.frec = w.frec;
  auto cap = [&](int gr) {  // enough waves for every tile, a multiple of 8 (XCD-partitioned slot ranges)
    const int c = (int)(NT / 4 + 1 < gr ? NT / 4 + 1 : gr);
    return (c + 7) / 8 * 8;
  };
  static int f18 = 0, f27 = 0, f18c = 0, f27c = 0;
  if (!f18) f18 = resident_grid(k_bwd_fused<18, false>, 256, 3);
  if (!f27) f27 = resident_grid(k_bwd_fused<27, false>, 256, 2);
  if (!f18c) f18c = resident_grid(k_bwd_fused<18, true>, 256, 3);
  if (!f27c) f27c = resident_grid(k_bwd_fused<27, true>, 256, 2);
  if (s->clip_z) {
    if (vcol) MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<27, true><<<cap(f27c), 256, 0, st>>>(P)));
    else MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<18, true><<<cap(f18c), 256, 0, st>>>(P)));
  } else {
    if (vcol) MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<27, false><<<cap(f27), 256, 0, st>>>(P)));
    else MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<18, false><<<cap(f18), 256, 0, st>>>(P)));
  }
  MR_CHECK_LAUNCH("k_bwd_fused");
  const int use_n = sp->light_kind == 0;
  const int vb = ceil_div(m->V * MR_VL, 256);
  if (!use_n) MR_TIMED(KID_RT_REDUCE, st, (k_rt_reduce<<<(unsigned)N, 256, 0, st>>>(rt_part, w.vslot, (int)N, gviews, gRcv, gtcv)));
  else if (vcol) MR_TIMED(KID_RT_VGRAD_A, st, (k_rt_vgrad_a<27><<<(unsigned)(N + vb), 256, 0, st>>>(rt_part, w.vslot, (int)N, gviews, gRcv, gtcv, m->V, m->vadj_ptr, m->vadj, gface, vraw, gnu)));
  else MR_TIMED(KID_RT_VGRAD_A, st, (k_rt_vgrad_a<18><<<(unsigned)(N + vb), 256, 0, st>>>(rt_part, w.vslot, (int)N, gviews, gRcv, gtcv, m->V, m->vadj_ptr, m->vadj, gface, vraw, gnu)));
  MR_CHECK_LAUNCH("k_rt_vgrad_a");
  if (vcol) {
    MR_TIMED(KID_VGRAD_B, st, (k_vgrad_b<27><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, gface, gnu, use_n, gverts, gcol)));
  } else {
    MR_TIMED(KID_VGRAD_B, st, (k_vgrad_b<18><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, gface, gnu, use_n, gverts, gcol)));
  }
  MR_CHECK_LAUNCH("k_vgrad");
  return MR_OK;
}

// ---------------- K-deep soft shading over stored fragments ----------------
static int check_frags(const mr_mesh_t* m, const mr_shade_params_t* sp, const int64_t* p2f, const float* zbuf,
                       const float* bary, const float* dists, int64_t N, int32_t H, int32_t W, int32_t K) {
  int rc = check_mesh(m, sp);
  if (rc) return rc;
  if (N <= 0 || N > 65535 || H <= 0 || W <= 0 || K < 1 || K > MR_KMAX) return set_err(MR_EINVAL, "bad fragment sizes");
  if (N * (int64_t)H * W * K >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "N*H*W*K >= 2^31");
  if (!p2f || !zbuf || !bary || !dists) return set_err(MR_EINVAL, "NULL fragment tensor");
  const int of = sp->out_flags & (MR_OUT_SIL | MR_OUT_RGB);
  if (of != MR_OUT_SIL && of != MR_OUT_RGB) return set_err(MR_EINVAL, "out_flags: exactly one of MR_OUT_SIL, MR_OUT_RGB");
  return MR_OK;
}

static FragShadeParams make_frag(const mr_mesh_t* m, const mr_shade_params_t* sp, const float* cc, int64_t ncc,
                                 const int64_t* p2f, const float* zbuf, const float* bary, const float* dists,
                                 int64_t N, int32_t H, int32_t W, int32_t K, const void* ws) {
  FragShadeParams P;
  memset(&P, 0, sizeof(P));
  P.N = (int)N; P.H = H; P.W = W; P.K = K;
  P.F = m->view_face_first ? 0 : m->F;  // face of packed id p: p - n*F (distinct meshes: p itself)
  P.sil = (sp->out_flags & MR_OUT_SIL) ? 1 : 0;
  P.hard = (!P.sil && (sp->out_flags & MR_OUT_HARD)) ? 1 : 0;
  P.p2f = p2f; P.zbuf = zbuf; P.bary = bary; P.dists = dists;
  P.S = make_shade(m, sp, cc, ncc);
  P.srec = (const ShadeRec*)ws;
  return P;
}

size_t mr_shade_fragments_workspace(int64_t F) { return align_up(sizeof(ShadeRec) * (size_t)(F > 0 ? F : 1), 256); }

int32_t mr_shade_fragments_forward(const mr_mesh_t* m, const int64_t* p2f, const float* zbuf, const float* bary,
                                   const float* dists, int64_t N, int32_t H, int32_t W, int32_t K,
                                   const float* cc, int64_t ncc, const mr_shade_params_t* sp, float* rgba,
                                   void* ws, size_t ws_bytes, void* stream) {
  int rc = check_frags(m, sp, p2f, zbuf, bary, dists, N, H, W, K);
  if (rc) return rc;
  if (!rgba || !ws) return set_err(MR_EINVAL, "NULL output / workspace");
  if (ws_bytes < mr_shade_fragments_workspace(m->F)) return set_err(MR_EWORKSPACE, "workspace too small");
  if (sp->light_kind == 0 && (!cc || (ncc != 1 && ncc != N))) return set_err(MR_EINVAL, "camera centres");
  hipStream_t st = (hipStream_t)stream;
  FragShadeParams P = make_frag(m, sp, cc, ncc, p2f, zbuf, bary, dists, N, H, W, K, ws);
  P.rgba = rgba;
  MR_TIMED(KID_SHADE_REC, st, (k_shade_rec<<<ceil_div(m->F, 256), 256, 0, st>>>(P.S, m->F, (ShadeRec*)ws)));
  MR_CHECK_LAUNCH("k_shade_rec");
  MR_TIMED(KID_FRAG_SHADE, st, (k_frag_shade_fwd<<<ceil_div(N * (int64_t)H * W, 256), 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_frag_shade_fwd");
  return MR_OK;
}

size_t mr_shade_fragments_backward_workspace(int64_t V, int64_t F) {
  size_t off = align_up(sizeof(float) * 27 * (size_t)(F > 0 ? F : 1), 256);  // gface
  return align_up(off + sizeof(float) * 3 * (size_t)(V > 0 ? V : 1), 256);    // gnu
}

int32_t mr_shade_fragments_backward(const mr_mesh_t* m, const float* vraw, const int64_t* p2f, const float* zbuf,
                                    const float* bary, const float* dists, int64_t N, int32_t H, int32_t W,
                                    int32_t K, const float* cc, int64_t ncc, const mr_shade_params_t* sp,
                                    const float* grad_rgba, const void* fwd_ws, void* bws, size_t bws_bytes,
                                    float* g_zbuf, float* g_bary, float* g_dists, float* g_verts, float* g_vcolors,
                                    float* g_tex_rgba, float* g_verts_uvs, int64_t num_verts_uvs, void* stream) {
  int rc = check_frags(m, sp, p2f, zbuf, bary, dists, N, H, W, K);
  if (rc) return rc;
  if (!grad_rgba || !fwd_ws || !bws || !g_zbuf || !g_bary || !g_dists || !g_verts)
    return set_err(MR_EINVAL, "NULL argument");
  if (bws_bytes < mr_shade_fragments_backward_workspace(m->V, m->F)) return set_err(MR_EWORKSPACE, "backward workspace too small");
  if (sp->light_kind == 0 && !vraw) return set_err(MR_EINVAL, "raw vertex normals required");
  hipStream_t st = (hipStream_t)stream;
  const bool vcol = m->tex_kind == 1;
  const int ACC = vcol ? 27 : 18;
  float* gface = (float*)bws;
  float* gnu = (float*)((char*)bws + align_up(sizeof(float) * 27 * (size_t)m->F, 256));
  if (hipMemsetAsync(gface, 0, sizeof(float) * ACC * (size_t)m->F, st) != hipSuccess) return set_err(MR_ELAUNCH, "memset failed");
  if (g_tex_rgba && m->tex_kind == 2 &&
      hipMemsetAsync(g_tex_rgba, 0, sizeof(float) * 4 * (size_t)m->tex_h * m->tex_w, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  if (g_verts_uvs && m->tex_kind == 2 && num_verts_uvs > 0 &&
      hipMemsetAsync(g_verts_uvs, 0, sizeof(float) * 2 * (size_t)num_verts_uvs, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  FragShadeParams P = make_frag(m, sp, cc, ncc, p2f, zbuf, bary, dists, N, H, W, K, fwd_ws);
  P.g_rgba = grad_rgba;
  P.g_zbuf = g_zbuf; P.g_bary = g_bary; P.g_dists = g_dists;
  P.gface = gface;
  P.gmap = m->tex_kind == 2 ? g_tex_rgba : nullptr;
  P.guv = m->tex_kind == 2 ? g_verts_uvs : nullptr;
  const int grid = ceil_div(N * (int64_t)H * W, 256);
  {  // the fragment gradients of empty slots are zero: cleared here with coalesced fills
    const size_t slots = (size_t)N * H * W * K;
    if (hipMemsetAsync(g_zbuf, 0, sizeof(float) * slots, st) != hipSuccess ||
        hipMemsetAsync(g_dists, 0, sizeof(float) * slots, st) != hipSuccess ||
        hipMemsetAsync(g_bary, 0, sizeof(float) * 3 * slots, st) != hipSuccess)
      return set_err(MR_ELAUNCH, "memset failed");
  }
  if (vcol) MR_TIMED(KID_FRAG_SHADE_BWD, st, (k_frag_shade_bwd<27><<<grid, 256, 0, st>>>(P)));
  else MR_TIMED(KID_FRAG_SHADE_BWD, st, (k_frag_shade_bwd<18><<<grid, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_frag_shade_bwd");
  // vertex gradients of the attribute rows (interpolated positions and normals, vertex colours)
  const int use_n = sp->light_kind == 0 && !P.sil;
  const int vb = ceil_div(m->V * MR_VL, 256);
  if (use_n) {
    if (vcol) k_rt_vgrad_a<27><<<(unsigned)vb, 256, 0, st>>>(nullptr, nullptr, 0, nullptr, nullptr, nullptr, m->V, m->vadj_ptr, m->vadj, gface, vraw, gnu);
    else k_rt_vgrad_a<18><<<(unsigned)vb, 256, 0, st>>>(nullptr, nullptr, 0, nullptr, nullptr, nullptr, m->V, m->vadj_ptr, m->vadj, gface, vraw, gnu);
    MR_CHECK_LAUNCH("k_rt_vgrad_a");
  }
  if (vcol) k_vgrad_b<27><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, gface, gnu, use_n, g_verts, g_vcolors);
  else k_vgrad_b<18><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, gface, gnu, use_n, g_verts, g_vcolors);
  MR_CHECK_LAUNCH("k_vgrad_b");
  return MR_OK;
}

// Covered pixels of a forward (stats only; a same-address counter in the raster serialises).
__global__ void __launch_bounds__(256) k_count_covered(const int* __restrict__ sface, const int* __restrict__ ctr,
                                                       int* __restrict__ out) {
  const int64_t n = (int64_t)ctr[CTR_SLOTS] * 64;
  int c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += sface[i] >= 0 ? 1 : 0;
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

int32_t mr_workspace_stats(const void* ws, int64_t N, int64_t Ftot, int32_t H, int32_t W, int32_t mfpb, int64_t* out,
                           void* stream) {
  if (!ws || !out || N <= 0 || N > 65535) return set_err(MR_EINVAL, "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  BinGeom g = bin_geom(H, W, N, Ftot > 0 ? Ftot : 1, mfpb);
  RasterWS w = carve_raster_ws((void*)ws, N, Ftot > 0 ? Ftot : 1, H, W, g);
  const size_t n = (size_t)N + CTR_COUNT + (size_t)N * g.T;  // ctr, cnt and vtot are contiguous
  if (hipMemsetAsync(w.ctr + CTR_COVERED, 0, sizeof(int), st) != hipSuccess) return set_err(MR_ELAUNCH, "memset failed");
  k_count_covered<<<1024, 256, 0, st>>>(w.sface, w.ctr, w.ctr + CTR_COVERED);
  MR_CHECK_LAUNCH("k_count_covered");
  int* h = (int*)malloc(sizeof(int) * n);
  if (!h) return set_err(MR_EINVAL, "out of host memory");
  if (hipMemcpyAsync(h, w.ctr, sizeof(int) * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    free(h);
    return set_err(MR_ELAUNCH, "stats copy failed");
  }
  // entries: the per-view binning's u64 counter, else the per-view totals of the count pass
  unsigned long long e64;
  memcpy(&e64, h + CTR_ENTRIES64, sizeof(e64));
  int64_t ent = (int64_t)e64;
  if (!view_binning(g, N, Ftot > 0 ? Ftot : 1))
    for (int64_t i = 0; i < N; ++i) ent += h[CTR_COUNT + (size_t)N * g.T + i];
  out[0] = ent;
  out[1] = h[CTR_UNITS];
  out[2] = h[CTR_SLOTS];
  out[3] = h[CTR_COVERED];
  free(h);
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

static int pose_loss_params(PoseLossParams& P, const float* depth, const float* sil, const float* rgb,
                            int64_t rgb_stride, const uint8_t* mask, const float* depth_ref, const float* rgb_ref,
                            int64_t npix, float delta, float w_color) {
  if (npix <= 0) return set_err(MR_EINVAL, "npix must be > 0");
  if (!depth || !sil || !rgb || !mask || !depth_ref || !rgb_ref) return set_err(MR_EINVAL, "NULL loss input");
  if (rgb_stride < 3) return set_err(MR_EINVAL, "rgb_stride must be >= 3");
  if (!(delta > 0.0f)) return set_err(MR_EINVAL, "huber delta must be > 0");
  P.depth = depth; P.sil = sil; P.rgb = rgb; P.rgb_stride = rgb_stride; P.mask = mask;
  P.depth_ref = depth_ref; P.rgb_ref = rgb_ref; P.npix = npix; P.delta = delta; P.w_color = w_color;
  return MR_OK;
}

size_t mr_pose_loss_workspace(int64_t npix) {
  (void)npix;
  return align_up(sizeof(float) * 3 * MR_LOSS_BLOCKS, 256) + align_up(sizeof(int) * MR_LOSS_BLOCKS, 256) + 256;
}

int32_t mr_pose_loss_forward(const float* depth, const float* sil, const float* rgb, int64_t rgb_stride,
                             const uint8_t* mask, const float* depth_ref, const float* rgb_ref, int64_t npix,
                             float delta, float w_color, float* out, void* ws, size_t ws_bytes, void* stream) {
  PoseLossParams P;
  int rc = pose_loss_params(P, depth, sil, rgb, rgb_stride, mask, depth_ref, rgb_ref, npix, delta, w_color);
  if (rc) return rc;
  if (!out || !ws) return set_err(MR_EINVAL, "NULL output / workspace");
  if (ws_bytes < mr_pose_loss_workspace(npix)) return set_err(MR_EWORKSPACE, "loss workspace too small");
  char* w = (char*)ws;
  float* part = (float*)w;
  int* pcnt = (int*)(w + align_up(sizeof(float) * 3 * MR_LOSS_BLOCKS, 256));
  int64_t* count = (int64_t*)(w + align_up(sizeof(float) * 3 * MR_LOSS_BLOCKS, 256) + align_up(sizeof(int) * MR_LOSS_BLOCKS, 256));
  const int nb = (int)std::min<int64_t>(MR_LOSS_BLOCKS, ceil_div(npix, 256));
  hipStream_t st = (hipStream_t)stream;
  k_pose_loss_partial<<<nb, 256, 0, st>>>(P, part, pcnt);
  MR_CHECK_LAUNCH("k_pose_loss_partial");
  k_pose_loss_final<<<1, 256, 0, st>>>(P, part, pcnt, nb, out, count);
  MR_CHECK_LAUNCH("k_pose_loss_final");
  return MR_OK;
}

int32_t mr_pose_loss_backward(const float* depth, const float* sil, const float* rgb, int64_t rgb_stride,
                              const uint8_t* mask, const float* depth_ref, const float* rgb_ref, int64_t npix,
                              float delta, float w_color, const float* g_total, const void* fwd_ws,
                              float* g_depth, float* g_sil, float* g_rgb, void* stream) {
  PoseLossParams P;
  int rc = pose_loss_params(P, depth, sil, rgb, rgb_stride, mask, depth_ref, rgb_ref, npix, delta, w_color);
  if (rc) return rc;
  if (!g_total || !fwd_ws || !g_depth || !g_sil || !g_rgb) return set_err(MR_EINVAL, "NULL gradient argument");
  const char* w = (const char*)fwd_ws;
  const int64_t* count = (const int64_t*)(w + align_up(sizeof(float) * 3 * MR_LOSS_BLOCKS, 256) +
                                          align_up(sizeof(int) * MR_LOSS_BLOCKS, 256));
  k_pose_loss_bwd<<<(unsigned)ceil_div(npix, 256), 256, 0, (hipStream_t)stream>>>(P, g_total, count, g_depth, g_sil, g_rgb);
  MR_CHECK_LAUNCH("k_pose_loss_bwd");
  return MR_OK;
}

}  // extern "C"
