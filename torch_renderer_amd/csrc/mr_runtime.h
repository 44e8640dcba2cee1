// mi355r — Host-side runtime of the library: error state, per-kernel timing events, the workspace
// carve (face records, tile lists, work units, per-slot winners) and its counters.
// Part of the single translation unit mr_raster.hip (included there, in this order).
#pragma once

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
enum KernelId { KID_BIN_COUNT, KID_BIN_SCAN, KID_BIN_FILL, KID_TILE_RASTER, KID_SHADE_FRAG, KID_SHADE_RENDER, KID_RASTER_BWD, KID_RT_VGRAD_B, KID_BWD_GEOM, KID_RT_REDUCE,
                KID_VGRAD_A, KID_VGRAD_B,
                KID_VNORMALS, KID_PROJECT, KID_PROJECT_BWD, KID_SHADE_REC, KID_FILL_FRAG,
                KID_RASTER_K, KID_BWD_FUSED, KID_RT_VGRAD_A, KID_FRAG_SHADE, KID_FRAG_SHADE_BWD, KID_SETUP, KID_BIN_RECT, KID_BIN_VIEW,
                KID_FACE_REDUCE, KID_BAND_BUCKET, KID_POSE_LOSS, KID_POSE_LOSS_SCALE, KID_UNIT_ORDER, KID_COUNT };
static const char* kKernelNames[KID_COUNT] = {"k_bin_count", "k_bin_scan", "k_bin_fill", "k_tile_raster",
                                              "k_shade<0>", "k_shade<1>",
                                              "k_raster_bwd", "k_rt_vgrad_b", "k_bwd_geom(unused)", "k_rt_reduce",
                                              "k_vgrad_a", "k_vgrad_b",
                                              "k_vertex_normals", "k_project_faces", "k_project_faces_bwd",
                                              "k_shade_rec", "k_fill<0>", "k_raster_k", "k_bwd_fused",
                                              "k_rt_vgrad_a", "k_frag_shade_fwd", "k_frag_shade_bwd", "k_setup_zero",
                                              "k_bin_rect", "k_bin_view", "k_face_reduce(unused)", "k_band_bucket",
                                              "k_pose_loss_fused", "k_pose_loss_scale", "k_unit_order"};
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
#ifndef MR_BANDS_MAX
#define MR_BANDS_MAX 64  // per-view binning: workgroups (bands of tile rows) per view (32 -> 64: C5 k_bin_view 24.6 -> 18.8 us, r6n)
#endif
#define MR_SREC_SLOTS 4  // ShadeRec sets per fused-forward workspace (out_flags bits 8-9 pick one)
#define MR_UE 64  // (tile, face) entries per raster work unit (one wave, one entry per lane)
// ctr[CTR_ENTRIES64 .. +2) is a u64: list entries allocated by the per-view binning (k_bin_view)
// ctr[CTR_SENT]: fragments kept by the fused soft silhouette's raster (mr_soft_silhouette_forward)
// ctr[CTR_ZWALK]: tiles the K-deep raster walked near-to-far (its depth-ordered list walk)
// ctr[CTR_FLT]: non-zero once k_bwd_fused wrote a float remainder (a total component >= MR_FIX_MAX): the
// vertex-gradient gathers read the remainder rows only then (they are all zero otherwise)
enum { CTR_UNITS = 0, CTR_SLOTS = 1, CTR_COVERED = 2, CTR_SENT = 3, CTR_ENTRIES64 = 4, CTR_ZWALK = 6,
       CTR_FLT = 7, CTR_COUNT = 8 };

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

static int num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}
// Workgroups (bands of tile rows) per view of the per-view binning: enough for the views to cover
// 1 / MR_BAND_CU_DIV of the CUs (1 view -> 64 bands, 16 views -> 4, 64 views -> 1 on 256 CUs), at
// most MR_BANDS_MAX and one tile row per band. The CUs left over stream the background beside the
// binning: banding 64 views 4 ways starved that share (fragment pass 421k -> 363k frames/s, render
// 240k -> 223k, profiles/r4f_bands_ab.txt). A pure function of the batch geometry: the backward's
// R/T reduction walks the same (view, band) ranges.
#ifndef MR_BAND_CU_DIV
#define MR_BAND_CU_DIV 4
#endif
static int bin_bands(int64_t N, const BinGeom& g) {
  int64_t b = (int64_t)num_cus() / ((N > 0 ? N : 1) * MR_BAND_CU_DIV);
  if (b > MR_BANDS_MAX) b = MR_BANDS_MAX;
  if (b > g.TY) b = g.TY;
  return b < 1 ? 1 : (int)b;
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
  int* vslot;  // (2 N B) first slot and number of slots of each (view, band); B = 1 on the count -> scan path
  int* stile;  // (N*T) per slot: view * T + tile
  int4* units2;  // (unit_cap) the same units, heaviest first inside each XCD range (k_unit_order)
  int4* units; // (unit_cap) {view*T + tile, first list entry (-1: every face of the view), entries, slot | multi<<31}
  int* list;   // list_cap
  unsigned long long* tkey;  // (N*T*64) per-slot (z, face) keys of tiles shared by several units
  int* sface;  // (N*T*64) per slot, per tile pixel (row-major 8x8): winning face record or -1
  ShadeRec* srec;  // (F) per-face shading inputs (fused path; F = faces of the shared mesh)
  // (F, 27) u64 + (F, 27) f32: the fused backward's per-face gradient totals, cleared by the forward.
  // Fixed point (MR_FIX_SHIFT fractional bits, two's complement) summed with 64-bit integer atomics:
  // integer addition is associative, so the totals do not depend on the order the backward's waves
  // add their per-(record, tile) runs in — bitwise deterministic vertex gradients with one launch
  // fewer than a fixed-order reduction of stored rows (round 4). The f32 rows take the rare run
  // component of magnitude >= MR_FIX_MAX = 2^24 (float atomics; see mr_common.h).
  int* sorder;
  unsigned long long* gfix;
  float* gflt;
  float4* frec;    // (N*T*64) fused path: per slot pixel the winner's fragment (b0, b1, b2, signed dist)
  int* sgrp;       // (N*T*64) fused path: each slot's winners grouped by record (k_shade<1>, for the backward)
  uint8_t* sgpix;  // (N*T*64) fused path: the tile pixel of each grouped position
  ClipRec* crec;   // (2 * Ftot) barycentric conversion of near-plane sub-triangles (by record id)
  // banded per-view binning of one shared mesh (bands > 1): each (view, band)'s records, listed by
  // k_band_bucket (bcap = 2 Ftot / N: both triangles of every face of the view), and their counts
  // (cleared by the record launch)
  int* bcnt;
  int* blist;
  int64_t bcap;
  int nbcnt;       // N * bands (0: no lists)
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
  off = align_up(off + sizeof(int) * 2 * MR_BANDS_MAX * (size_t)N, 256);
  w.stile = (int*)(b + off);
  off = align_up(off + sizeof(int) * NT, 256);
  w.units = (int4*)(b + off);
  off = align_up(off + sizeof(int4) * (size_t)g.unit_cap, 256);
  w.units2 = (int4*)(b + off);  // the units in the raster's order (k_unit_order)
  off = align_up(off + sizeof(int4) * (size_t)g.unit_cap, 256);
  w.list = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)g.list_cap, 256);
  w.tkey = (unsigned long long*)(b + off);
  off = align_up(off + sizeof(unsigned long long) * 64 * NT, 256);
  w.sface = (int*)(b + off);
  off = align_up(off + sizeof(int) * 64 * NT, 256);
  w.srec = (ShadeRec*)(b + off);  // MR_SREC_SLOTS slots of Fshade records (mr_render_reshade)
  off = align_up(off + sizeof(ShadeRec) * MR_SREC_SLOTS * (size_t)Fshade, 256);
  w.sorder = (int*)(b + off);  // the K-deep raster's slot order (k_slot_order)
  off = align_up(off + sizeof(int) * (size_t)NT, 256);
  w.gfix = (unsigned long long*)(b + off);
  off = align_up(off + sizeof(unsigned long long) * 27 * (size_t)Fshade, 256);
  w.gflt = (float*)(b + off);
  off = align_up(off + sizeof(float) * 27 * (size_t)Fshade, 256);
  w.frec = (float4*)(b + off);
  off = align_up(off + sizeof(float4) * (Fshade > 0 ? 64 * NT : 0), 256);
  w.sgrp = (int*)(b + off);
  off = align_up(off + sizeof(int) * (Fshade > 0 ? 64 * NT : 0), 256);
  w.sgpix = (uint8_t*)(b + off);
  off = align_up(off + (Fshade > 0 ? 64 * NT : 0), 256);
  w.crec = (ClipRec*)(b + off);
  off = align_up(off + sizeof(ClipRec) * 2 * (size_t)(Ftot > 0 ? Ftot : 1), 256);
  const int B = bin_bands(N, g);
  w.nbcnt = B > 1 ? (int)(N * B) : 0;
  w.bcap = B > 1 ? 2 * ((Ftot > 0 ? Ftot : 1) + N - 1) / N : 0;
  w.bcnt = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)w.nbcnt, 256);
  w.blist = (int*)(b + off);
  off = align_up(off + sizeof(int) * (size_t)w.nbcnt * (size_t)w.bcap, 256);
  w.bytes = off;
  return w;
}
// Bytes to clear from w.ctr before a forward: the counters and, on the count -> scan path, the
// per-tile counts and per-view totals.
static size_t zero_bytes(int64_t N, const BinGeom& g, bool view_path) {
  return sizeof(int) * (view_path ? (size_t)CTR_COUNT : (size_t)N * g.T + (size_t)N + CTR_COUNT);
}
