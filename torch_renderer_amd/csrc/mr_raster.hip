// mi355r — MI355X (gfx950, CDNA4) rasterizer kernels + C ABI (one translation unit: the stage headers
// below are included in order; this file holds the extern "C" entry points of include/mi355r.h).
//
// Pipeline for a batch of N views (all launches async on one stream, no host sync):
//   1. binning (mr_bin.h): k_bin_rect_world projects every (view, face) — OpenCV pose conversion and
//      near-plane clipping inline — and writes its 64-B FaceRec and 8x8-tile rectangle; one 1024-thread
//      workgroup per view (k_bin_view) histograms, scans and fills the view's tile lists in LDS and
//      emits slots (non-empty tiles) and work UNITS of <= 64 (tile, face) entries. Large grids take
//      the count -> scan -> fill path.
//   2. K = 1 raster (mr_tile_raster.h): k_tile_raster, a persistent grid of independent waves
//      (XCD-partitioned units, 3-deep unit/list/record prefetch); each lane turns one face into an 8x8
//      coverage mask, the wave evaluates the (face, pixel) pairs 64 at a time exactly and keeps the
//      per-pixel minimum packed (z, face) key with ds_min_u64 (= the CPU's "strictly nearer, earlier
//      face wins"); the same waves stream the background. k_shade then recomputes each winner's
//      fragment and writes PyTorch3D Fragments (M = 0) or shaded depth / silhouette / rgb (M = 1).
//      K > 1 (mr_kdeep.h): k_fill, then the pair-enumerating register-list raster (K <= 64).
//   3. backward (mr_bwd.h): k_bwd_fused — per covered tile: shading backward (record handed over in
//      LDS), raster + projection backward, per-face rows summed over runs of equal faces (segmented
//      DPP scan) with float atomics per run, per-slot R/T partials. k_raster_bwd_slots is the
//      modular _C.rasterize_meshes_backward (any K).
//   4. vertex kernels (mr_vertex.h) gather per-face rows through a CSR vertex adjacency
//      (deterministic order) and chain the vertex-normal backward.
//   5. K-deep shading over stored fragments (mr_frag_shade.h) and the fused pose loss (mr_loss.h).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdarg.h>
#include <stdlib.h>

#include "../../include/mi355r.h"
#include "mr_common.h"
#include "mr_shade.h"

#include "mr_runtime.h"
#include "mr_bin.h"
#include "mr_tile_raster.h"
#include "mr_kdeep.h"
#include "mr_bwd.h"
#include "mr_vertex.h"
#include "mr_frag_shade.h"
#include "mr_loss.h"

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* mr_last_error(void) { return g_err; }


int32_t mr_version(void) { return 5; }

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
  memset(&P, 0, sizeof(P));
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
  P.bcnt = w.bcnt;
  P.nbcnt = w.nbcnt;
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
#define MR_BG_CPW_RENDER 12  // 5 KB chunks (depth, silhouette, RGB); 8 -> 12: render 259.0k -> 260.4k, 260.7k -> 263.1k frames/s (profiles/r4k_ab.txt)
#endif
#ifndef MR_BG_CPW_FRAG
#define MR_BG_CPW_FRAG 8    // 7 KB chunks (PyTorch3D fragments; 4 -> 8: fragment pass 166 -> 162 us)
#endif
#ifndef MR_BG_RECT_ROWS
#define MR_BG_RECT_ROWS 16  // fragment background rows of the record launch (each ceil(F / 256) workgroups)
#endif
#ifndef MR_BG_RECT_CPW
#define MR_BG_RECT_CPW 4    // chunks per wave of those rows
#endif
#ifndef MR_VIEW_LDS
#define MR_VIEW_LDS 98304  // k_bin_view's LDS: the tile histogram + the list stage
#endif
#ifndef MR_VIEW_LDS_BANDED
#define MR_VIEW_LDS_BANDED 65536  // ... with several bands per view: two workgroups per CU
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
// Background workgroups of the k_bin_view launch: the workgroup slots the binning (nbin = views x bands
// workgroups) and the ShadeRec packing (sb) leave free — one per CU with one workgroup per view (98 KB
// of LDS each), MR_BG_WG_PER_CU per CU with bands (64 KB: two fit a CU, so a background workgroup can
// stream stores on every CU beside a binning one).
#ifndef MR_BG_WG_PER_CU
#define MR_BG_WG_PER_CU 1
#endif
static int64_t bin_bg_wgs(int64_t nbin, int64_t sb, bool banded) {
  return (int64_t)num_cus() * (banded ? MR_BG_WG_PER_CU : 1) - nbin - sb;
}
// ShadeRec workgroups of the k_bin_view launch and their faces each (a multiple of 256, pack_shade_recs' pass).
// 1024 faces per workgroup: smaller shares took workgroups from the background and slowed the headline's raster
// (r6n: sb 6 -> 23, k_tile_raster +3 us), and with the corner-parallel packing 1024 faces take ~13 us, under the
// binning's critical path at C5 (20 us) and at the headline (38 us).
#ifndef MR_SREC_FPW
#define MR_SREC_FPW 1024
#endif
static int64_t srec_wgs(int64_t F, int64_t nbin, int* fpw_out = nullptr) {
  (void)nbin;
  if (F <= 0) return 0;
  if (fpw_out) *fpw_out = MR_SREC_FPW;
  return ceil_div(F, MR_SREC_FPW);
}
// Background chunks the k_bin_view launch takes over (chunks of 64 lanes x 4 pixels when W % 4 == 0,
// else 64 pixels); 0 when the binning leaves no workgroup slot free.
static int64_t bg_chunks(int64_t N, int64_t nbin, int64_t sb, int H, int W, int mode) {
  const int64_t nbg = bin_bg_wgs(nbin, sb, nbin > N);
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
    V.srec = Pf ? (ShadeRec*)Pf->srec : w.srec;  // the call's ShadeRec slot
    V.Fs = F;
  }
  V.T = g.T; V.TX = g.TX; V.TY = g.TY; V.mfpb = g.mfpb; V.clipz = SP.clipz;
  const int B = bin_bands(N, g);
  V.bands = B;
  const int64_t nbin = N * B;
  if (S) sb = srec_wgs(F, nbin, &V.srec_fpw);
  V.nsrec_wg = (int)sb;
  V.list_cap = g.list_cap; V.NF = SP.NF;
  V.rects = w.rects; V.first = first; V.view_count = view_count; V.F = F;
  V.cnt = w.cnt; V.start = w.start; V.vbase = w.vbase; V.tdone = w.tdone; V.vslot = w.vslot; V.stile = w.stile;
  V.units = w.units; V.ctr = w.ctr; V.tkey = w.tkey; V.list = w.list;
  if (B > 1 && !first && !view_count && w.nbcnt == N * B && F > 0) {
    // one shared mesh: each band's records listed first (the record launch cleared the counts)
    MR_TIMED(KID_BAND_BUCKET, st, (k_band_bucket<<<dim3((unsigned)ceil_div(F, 1024), (unsigned)N), 1024, 0, st>>>(
                                       w.rects, F, SP.NF, SP.clipz ? 2 : 1, g.TY, B, w.bcnt, w.blist, w.bcap)));
    MR_CHECK_LAUNCH("k_band_bucket");
    V.blist = w.blist;
    V.bcnt = w.bcnt;
    V.bcap = w.bcap;
  }
  const int Tb = ((g.TY + B - 1) / B) * g.TX;  // tiles of the largest band
  const size_t hist_b = sizeof(int) * (size_t)((Tb + (Tb >> 6) + 3) & ~3);
  const size_t shm = std::max(hist_b, B > 1 ? (size_t)MR_VIEW_LDS_BANDED : view_lds_bytes());
  V.stage_cap = (int)((shm - hist_b) / sizeof(int));
  if constexpr (MODE >= 0) {
    const int64_t nbg = bin_bg_wgs(nbin, sb, B > 1);
    if (Pf && nbg > 0 && (MODE != 0 || Pf->K == 1)) {
      Pf->fill_first = (int)bg_chunks(N, nbin, sb, Pf->H, Pf->W, MODE);
      MR_TIMED(KID_BIN_VIEW, st, (k_bin_view<MODE, CH><<<(unsigned)(nbin + sb + nbg), 1024, shm, st>>>(V, *Pf)));
      MR_CHECK_LAUNCH("k_bin_view");
      return MR_OK;
    }
  }
  MR_TIMED(KID_BIN_VIEW, st, (k_bin_view<<<(unsigned)(nbin + sb), 1024, shm, st>>>(V)));
  MR_CHECK_LAUNCH("k_bin_view");
  return MR_OK;
}
}  // extern "C++"

int32_t mr_per_view_binning(int64_t N, int64_t total_faces, int32_t H, int32_t W) {
  if (N <= 0 || H <= 0 || W <= 0) return 0;
  const int64_t Ft = total_faces > 0 ? total_faces : 1;
  return view_binning(bin_geom(H, W, N, Ft, 0), N, Ft) ? 1 : 0;
}

int64_t mr_binning_background_pixels(int64_t N, int64_t F, int32_t H, int32_t W, int32_t mode) {
  if (N <= 0 || H <= 0 || W <= 0) return 0;
  BinGeom g = bin_geom(H, W, N, N * (F > 0 ? F : 1), 0);
  if (!view_binning(g, N, N * (F > 0 ? F : 1))) return 0;
  const int64_t nbin = N * bin_bands(N, g);
  const int64_t sb = mode == 1 ? srec_wgs(F, nbin) : 0;
  const int64_t px = bg_chunks(N, nbin, sb, H, W, mode) * ((W & 3) == 0 ? 256 : 64);
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
    P.emit_frag = (s->W & 3) == 0;  // per-tile counts (ranges) for the raster's background skip
    if ((rc = launch_bin_view<0, 3>(SP, w, g, N, first, count, 0, P.emit_frag != 0, st, nullptr, &P))) return rc;
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

// View records from the pose arrays (either convention, cv_view_elem), the count -> scan path of the
// fused render.
__global__ void __launch_bounds__(256) k_views_from_cv(CvPoses C, int64_t N) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < N * 16) C.out[i] = cv_view_elem(C, i >> 4, (int)(i & 15));
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
  // K = 1, W % 4 == 0: background chunks past k_bin_view's share go to extra rows of the record
  // launch (up to MR_BG_RECT_ROWS rows of MR_BG_RECT_CPW chunks per wave), the rest to the raster
  FragBg FB{};
  int64_t rect_bg0 = 0, rect_bgn = 0;
  if (s->faces_per_pixel == 1 && (s->W & 3) == 0 && MR_BG_RECT_ROWS > 0) {
    const int64_t total = N * (((int64_t)s->H * s->W / 4 + 63) / 64);
    rect_bg0 = bg_chunks(N, N * bin_bands(N, g), 0, s->H, s->W, 0);  // = the k_bin_view share launch_bin_view takes
    rect_bgn = std::min<int64_t>(total - rect_bg0, (int64_t)MR_BG_RECT_ROWS * rgrid.x * 4 * MR_BG_RECT_CPW);
    if (rect_bgn > 0) {
      FB.p2f = p2f; FB.zbuf = zbuf; FB.dists = dists; FB.bary = bary;
      FB.H = s->H; FB.W = s->W; FB.nviews = (int)N; FB.first = (int)rect_bg0; FB.count = (int)rect_bgn;
      rgrid.y += MR_BG_RECT_ROWS;
    }
  }
  if (SP.clipz) MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_world<true><<<rgrid, 256, 0, st>>>(SP, verts, faces, F, (const ViewRec*)views_out, NA, w.ctr, C, FB)));
  else MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_world<false><<<rgrid, 256, 0, st>>>(SP, verts, faces, F, (const ViewRec*)views_out, NA, w.ctr, C, FB)));
  MR_CHECK_LAUNCH("k_bin_rect_world");
  if (s->faces_per_pixel > 1) {
    if ((rc = launch_bin_view(SP, w, g, N, nullptr, nullptr, F, true, st))) return rc;
    return launch_raster_k(P, g, N, st);
  }
  P.emit_frag = (s->W & 3) == 0;  // per-tile counts (ranges) for the raster's background skip
  if ((rc = launch_bin_view<0, 3>(SP, w, g, N, nullptr, nullptr, F, P.emit_frag != 0, st, nullptr, &P))) return rc;
  if (rect_bgn > 0) P.fill_first = (int)(rect_bg0 + rect_bgn);  // the raster writes the chunks after the record launch's
  return launch_raster_and_shade<0, 3>(P, g, N, st, s->clip_z != 0);
}

// ---------------- fused soft silhouette (MeshRenderer(MeshRasterizer(K > 1), SoftSilhouetteShader)) --------
struct SilWS {
  float4* spix;
  int4* sent;
  size_t bytes;
};
static SilWS carve_sil(void* base, size_t raster_bytes, int64_t NT, int K) {
  SilWS w;
  char* b = (char*)base;
  size_t off = align_up(raster_bytes, 256);
  w.spix = (float4*)(b + off);
  off = align_up(off + sizeof(float4) * 64 * (size_t)NT, 256);
  w.sent = (int4*)(b + off);
  off = align_up(off + sizeof(int4) * 64 * (size_t)K * (size_t)NT, 256);
  w.bytes = off;
  return w;
}
size_t mr_soft_silhouette_workspace(int64_t N, int64_t F, int32_t H, int32_t W, int32_t K, int32_t max_faces_per_bin) {
  const int64_t Fb = N * F > 0 ? N * F : 1;
  BinGeom g = bin_geom(H, W, N, Fb, max_faces_per_bin);
  const size_t rb = carve_raster_ws(nullptr, N, Fb, H, W, g).bytes;
  return carve_sil(nullptr, rb, N * (int64_t)g.T, K > 0 ? K : 1).bytes;
}

int32_t mr_soft_silhouette_forward(const float* verts, int64_t V, const int32_t* faces, int64_t F,
                                   const mr_poses_t* poses, int64_t N, const mr_raster_settings_t* s, float sigma,
                                   mr_view_t* views_out, float* face_verts, float* rgba, void* ws, size_t ws_bytes,
                                   void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  const int K = s->faces_per_pixel;
  if (K < 2 || K > 64) return set_err(MR_EUNSUPPORTED, "fused soft silhouette: 2 <= faces_per_pixel <= 64 (got %d)", K);
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "N must be in [1, 65535] (got %lld)", (long long)N);
  if (F <= 0 || V <= 0 || N * F >= (1ll << 30)) return set_err(MR_EINVAL, "F / V out of range");
  if ((int64_t)N * s->H * s->W >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "N*H*W >= 2^31");
  if (!(sigma > 0.0f)) return set_err(MR_EINVAL, "sigma must be > 0");
  if (!poses || !poses->R || !poses->T || !poses->intr || !views_out || !verts || !faces || !face_verts || !rgba)
    return set_err(MR_EINVAL, "NULL argument");
  if (poses->R_stride < 0 || poses->T_stride < 0 || poses->intr_stride < 0) return set_err(MR_EINVAL, "negative stride");
  const int64_t Fb = N * F;
  BinGeom g = bin_geom(s->H, s->W, N, Fb, s->max_faces_per_bin);
  if (!view_binning(g, N, Fb)) return set_err(MR_EUNSUPPORTED, "fused soft silhouette: per-view binning sizes only");
  if ((int64_t)N * g.T * 64 * K >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "N*T*64*K >= 2^31");
  RasterWS w = carve_raster_ws(ws, N, Fb, s->H, s->W, g);
  SilWS sw = carve_sil(ws, w.bytes, N * (int64_t)g.T, K);
  if (ws_bytes < sw.bytes) return set_err(MR_EWORKSPACE, "workspace too small: %zu < %zu", ws_bytes, sw.bytes);
  hipStream_t st = (hipStream_t)stream;
  CvPoses C;
  C.R = poses->R; C.sR = poses->R_stride; C.t = poses->T; C.sT = poses->T_stride;
  C.intr = poses->intr; C.sI = poses->intr_stride; C.out = (float*)views_out; C.opencv = 0;
  SetupParams SP = make_setup(s, g, w);
  SP.NF = Fb;
  SP.fv_out = face_verts;
  FwdParams P = make_fwd(s, g, w, N, nullptr, F, Fb);
  P.sil = rgba;
  P.isig = 1.0f / sigma;  // = mr_shade_params_t.sigma_sil's reciprocal in make_shade
  P.spix = sw.spix; P.sent = sw.sent;
  NormalsArgs NA;
  memset(&NA, 0, sizeof(NA));
  dim3 rgrid((unsigned)ceil_div(F, 256), (unsigned)N + 1);  // row 0: counter clear
  if (SP.clipz) MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_world<true><<<rgrid, 256, 0, st>>>(SP, verts, faces, F, (const ViewRec*)views_out, NA, w.ctr, C, FragBg{})));
  else MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_world<false><<<rgrid, 256, 0, st>>>(SP, verts, faces, F, (const ViewRec*)views_out, NA, w.ctr, C, FragBg{})));
  MR_CHECK_LAUNCH("k_bin_rect_world");
  if ((rc = launch_bin_view(SP, w, g, N, nullptr, nullptr, F, true, st))) return rc;
  launch_raster_sil(P, g, N, st);
  MR_CHECK_LAUNCH("k_raster_kp (silhouette)");
  return MR_OK;
}

int32_t mr_soft_silhouette_backward(const float* face_verts, int64_t N, int64_t F, const mr_raster_settings_t* s,
                                    float sigma, const float* grad_rgba, const void* ws, float* grad_face_verts,
                                    void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  if (N <= 0 || N > 65535 || F <= 0) return set_err(MR_EINVAL, "bad sizes");
  if (!face_verts || !grad_rgba || !ws || !grad_face_verts) return set_err(MR_EINVAL, "NULL argument");
  const int K = s->faces_per_pixel;
  if (K < 2 || K > 64 || !(sigma > 0.0f)) return set_err(MR_EINVAL, "bad faces_per_pixel / sigma");
  hipStream_t st = (hipStream_t)stream;
  const int64_t Fb = N * F;
  if (hipMemsetAsync(grad_face_verts, 0, sizeof(float) * 9 * (size_t)Fb, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  BinGeom g = bin_geom(s->H, s->W, N, Fb, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws((void*)ws, N, Fb, s->H, s->W, g);
  SilWS sw = carve_sil((void*)ws, w.bytes, N * (int64_t)g.T, K);
  SilBwdParams P;
  memset(&P, 0, sizeof(P));
  P.R.N = (int)N; P.R.H = s->H; P.R.W = s->W; P.R.NBX = ceil_div(s->W, MR_BT); P.R.K = K;
  P.R.persp = s->perspective_correct; P.R.clipb = s->clip_barycentric_coords;
  P.R.cull = s->cull_backfaces; P.R.clipz = s->clip_z != 0; P.R.zc = s->z_clip_value;
  P.R.blur = s->blur_radius; P.R.bbox_pad = sqrtf(s->blur_radius);
  P.R.fv = face_verts; P.R.gfv = grad_face_verts;
  P.T = g.T; P.TX = g.TX; P.isig = 1.0f / sigma;
  P.ctr = w.ctr; P.stile = w.stile; P.sent = sw.sent; P.spix = sw.spix;
  P.grad_rgba = grad_rgba;
  static int grid = 0;
  if (!grid) grid = resident_grid(k_sil_bwd, 256, 8);
  MR_TIMED(KID_RASTER_BWD, st, (k_sil_bwd<<<grid, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_sil_bwd");
  return MR_OK;
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

static int srec_slot(const mr_shade_params_t* sp) { return (sp->out_flags >> MR_SREC_SLOT_SHIFT) & (MR_SREC_SLOTS - 1); }

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
  S.zbuf_mode = (sp->out_flags & MR_OUT_ZBUF) ? 1 : 0;
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
int32_t mr_render_forward_poses(const mr_mesh_t* m, const mr_poses_t* poses, mr_view_t* views_out, int64_t N,
                                const float* cc, int64_t ncc, const mr_raster_settings_t* s,
                                const mr_shade_params_t* sp, float* depth, float* sil, float* rgb, int32_t* p2f32,
                                void* ws, size_t ws_bytes, void* stream) {
  if (!poses || !poses->R || !poses->T || !poses->intr || !views_out) return set_err(MR_EINVAL, "NULL pose argument");
  if (poses->R_stride < 0 || poses->T_stride < 0 || poses->intr_stride < 0) return set_err(MR_EINVAL, "negative stride");
  CvPoses C;
  C.R = poses->R; C.sR = poses->R_stride; C.t = poses->T; C.sT = poses->T_stride;
  C.intr = poses->intr; C.sI = poses->intr_stride; C.out = (float*)views_out;
  C.opencv = 0;
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
  P.srec = w.srec + (size_t)srec_slot(sp) * m->F;
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
    memset(&NA, 0, sizeof(NA));
    NA.V = m->V; NA.ptr = m->vadj_ptr; NA.adj = m->vadj;
    NA.vn = vb ? m->vnormals_out : nullptr;
    NA.vraw = m->vraw_out;
    // the backward's face totals: all 27 components per face, whatever this call's texture. A reshade
    // of the same raster may carry another texture kind (a depth render, then a vertex-colour Phong
    // reshade: ACC 27) and its backward, the first over this workspace, skips the clear
    // (MR_GRAD_ROWS_CLEARED); 27 columns cost 0.6 MB more stores at the bench config
    const int64_t nacc = (int64_t)27 * m->F;
    NA.zero4 = (float4*)w.gfix;
    NA.nzero4 = (nacc + 1) / 2;
    NA.zero4b = (float4*)w.gflt;
    NA.nzero4b = (nacc + 3) / 4;
    const int64_t bx = std::max<int64_t>(ceil_div(maxvf, 256), ceil_div(m->V, 256));
    dim3 rgrid((unsigned)(bx > 0 ? bx : 1), (unsigned)N + 1);  // row 0: normals + counter clear
    if (SP.clipz) MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_world<true><<<rgrid, 256, 0, st>>>(SP, m->verts, m->faces, m->F, (const ViewRec*)views, NA, w.ctr, C, FragBg{})));
    else MR_TIMED(KID_BIN_RECT, st, (k_bin_rect_world<false><<<rgrid, 256, 0, st>>>(SP, m->verts, m->faces, m->F, (const ViewRec*)views, NA, w.ctr, C, FragBg{})));
    MR_CHECK_LAUNCH("k_bin_rect_world");
    if (sp->rgb_channels == 4) {
      if ((rc = launch_bin_view<1, 4>(SP, w, g, N, m->view_face_first, m->view_face_count, m->F, false, st, &P.S, &P))) return rc;
      return launch_raster_and_shade<1, 4>(P, g, N, st, s->clip_z != 0);
    }
    if ((rc = launch_bin_view<1, 3>(SP, w, g, N, m->view_face_first, m->view_face_count, m->F, false, st, &P.S, &P))) return rc;
    return launch_raster_and_shade<1, 3>(P, g, N, st, s->clip_z != 0);
  }
  if (hipMemsetAsync(w.gfix, 0, sizeof(unsigned long long) * 27 * (size_t)m->F, st) != hipSuccess ||
      hipMemsetAsync(w.gflt, 0, sizeof(float) * 27 * (size_t)m->F, st) != hipSuccess)
    return set_err(MR_ELAUNCH, "memset failed");
  if (C.R) {  // count -> scan path: the view records first
    if (C.opencv) {
      k_views_from_opencv<<<ceil_div(N * 16, 256), 256, 0, st>>>(C.R, C.sR, C.t, C.sT, C.intr, C.sI, N, C.out);
      MR_CHECK_LAUNCH("k_views_from_opencv");
    } else {
      k_views_from_cv<<<ceil_div(N * 16, 256), 256, 0, st>>>(C, N);
      MR_CHECK_LAUNCH("k_views_from_cv");
    }
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
    MR_TIMED(KID_BIN_FILL, st, (k_bin_fill_world<true><<<fgrid, 256, shm, st>>>(SP, m->F, fpt, (int)N, P.S, (ShadeRec*)P.srec)));
  else
    MR_TIMED(KID_BIN_FILL, st, (k_bin_fill_world<false><<<fgrid, 256, 0, st>>>(SP, m->F, fpt, (int)N, P.S, (ShadeRec*)P.srec)));
  MR_CHECK_LAUNCH("k_bin_fill_world");
  if (sp->rgb_channels == 4) return launch_raster_and_shade<1, 4>(P, g, N, st, s->clip_z != 0);
  return launch_raster_and_shade<1, 3>(P, g, N, st, s->clip_z != 0);
}

int32_t mr_render_reshade(const mr_mesh_t* m, const mr_view_t* views, int64_t N, const float* cc, int64_t ncc,
                          const mr_raster_settings_t* s, const mr_shade_params_t* sp, float* depth, float* sil,
                          float* rgb, int32_t* p2f32, void* ws, size_t ws_bytes, void* stream) {
  int rc = check_settings(s);
  if (rc) return rc;
  rc = check_mesh(m, sp);
  if (rc) return rc;
  if (s->faces_per_pixel != 1) return set_err(MR_EUNSUPPORTED, "the fused render path is K = 1");
  if (sp->out_flags & MR_OUT_HARD) return set_err(MR_EUNSUPPORTED, "hard_rgb_blend runs on the fragment-shader path");
  if (N <= 0 || N > 65535) return set_err(MR_EINVAL, "N out of range");
  const bool multi = m->view_face_first != nullptr;
  const int64_t NF = multi ? m->F : N * m->F;
  if ((int64_t)N * s->H * s->W >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "N*H*W >= 2^31");
  if (!views || !ws) return set_err(MR_EINVAL, "NULL views / workspace");
  if ((sp->out_flags & MR_OUT_DEPTH) && !depth) return set_err(MR_EINVAL, "depth output NULL");
  if ((sp->out_flags & MR_OUT_SIL) && !sil) return set_err(MR_EINVAL, "silhouette output NULL");
  if ((sp->out_flags & MR_OUT_RGB) && !rgb) return set_err(MR_EINVAL, "rgb output NULL");
  if (sp->light_kind == 0 && (!cc || (ncc != 1 && ncc != N))) return set_err(MR_EINVAL, "camera centres");
  hipStream_t st = (hipStream_t)stream;
  BinGeom g = bin_geom(s->H, s->W, N, NF, s->max_faces_per_bin);
  RasterWS w = carve_raster_ws(ws, N, NF, s->H, s->W, g, m->F);
  if (ws_bytes < w.bytes) return set_err(MR_EWORKSPACE, "workspace too small: %zu < %zu", ws_bytes, w.bytes);
  FwdParams P = make_fwd(s, g, w, N, m->view_face_first, multi ? 0 : m->F, NF);
  P.view_count = m->view_face_count;
  P.S = make_shade(m, sp, cc, ncc);
  P.srec = w.srec + (size_t)srec_slot(sp) * m->F;
  P.out_flags = sp->out_flags;
  P.depth = depth;
  P.sil = sil;
  P.rgb = rgb;
  P.p2f32 = p2f32;
  // this call's vertex normals (as the forward's first launch), when its shading reads them: Phong RGB only
  if (sp->light_kind == 0 && m->vnormals_out && (sp->out_flags & MR_OUT_RGB)) {
    if (!m->vraw_out) return set_err(MR_EINVAL, "vnormals_out without vraw_out");
    P.S.vnormals = m->vnormals_out;
    MR_TIMED(KID_VNORMALS, st, (k_vertex_normals<<<ceil_div(m->V, 256), 256, 0, st>>>(m->verts, m->V, m->faces, m->vadj_ptr, m->vadj, m->vnormals_out, m->vraw_out)));
    MR_CHECK_LAUNCH("k_vertex_normals");
  }
  MR_TIMED(KID_SHADE_REC, st, (k_shade_rec<<<ceil_div(m->F, 256), 256, 0, st>>>(P.S, m->F, (ShadeRec*)P.srec)));
  MR_CHECK_LAUNCH("k_shade_rec");
  static int fg3 = 0, fg4 = 0, sg3 = 0, sg4 = 0;
  const int64_t slots_cap = N * (int64_t)g.T;
  auto shade_grid = [&](int gr) {
    int sg = (int)(slots_cap / 4 + 1 < gr ? slots_cap / 4 + 1 : gr);
    return (sg + 7) / 8 * 8;  // XCD-partitioned slot ranges
  };
  if (sp->rgb_channels == 4) {
    if (!fg4) fg4 = resident_grid(k_fill<1, 4>, 256, 8);
    if (!sg4) sg4 = resident_grid(k_shade<1, 4>, 256, 6);
    MR_TIMED(KID_FILL_FRAG, st, (k_fill<1, 4><<<fg4, 256, 0, st>>>(P)));
    MR_CHECK_LAUNCH("k_fill");
    MR_TIMED(KID_SHADE_RENDER, st, (k_shade<1, 4><<<shade_grid(sg4), 256, 0, st>>>(P)));
  } else {
    if (!fg3) fg3 = resident_grid(k_fill<1, 3>, 256, 8);
    if (!sg3) sg3 = resident_grid(k_shade<1, 3>, 256, 6);
    MR_TIMED(KID_FILL_FRAG, st, (k_fill<1, 3><<<fg3, 256, 0, st>>>(P)));
    MR_CHECK_LAUNCH("k_fill");
    MR_TIMED(KID_SHADE_RENDER, st, (k_shade<1, 3><<<shade_grid(sg3), 256, 0, st>>>(P)));
  }
  MR_CHECK_LAUNCH("k_shade");
  return MR_OK;
}

size_t mr_render_backward_workspace(int64_t N, int64_t V, int64_t F, int32_t H, int32_t W) {
  const int64_t NT = N * (int64_t)ceil_div(W, MR_TS) * ceil_div(H, MR_TS);
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
  if (m->F * 27 >= (1ll << 30)) return set_err(MR_EUNSUPPORTED, "F >= 2^30 / 27 faces");  // 32-bit row offsets
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
  // the per-face totals (fixed point + float remainder) live in the forward's workspace, which the
  // forward cleared; a second backward over the same forward (MR_GRAD_ROWS_CLEARED not set) clears
  // them again
  unsigned long long* gfix = w.gfix;
  float* gface = w.gflt;
  if (!(sp->out_flags & MR_GRAD_ROWS_CLEARED) &&
      (hipMemsetAsync(gfix, 0, sizeof(unsigned long long) * ACC * (size_t)m->F, st) != hipSuccess ||
       hipMemsetAsync(gface, 0, sizeof(float) * ACC * (size_t)m->F, st) != hipSuccess))
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
  P.srec = w.srec + (size_t)srec_slot(sp) * m->F;  // the forward's ShadeRec slot
  P.F = multi ? 0 : m->F;
  P.NF = NF;
  P.crec = w.crec;
  P.zc = s->z_clip_value;
  P.views = (const ViewRec*)views;
  P.gfix = gfix;
  P.gface = gface;
  P.fflag = w.ctr + CTR_FLT;
  P.rt_part = rt_part;
  P.frec = w.frec;
  P.sgrp = w.sgrp;
  P.sgpix = w.sgpix;
#ifndef MR_BWD_GRID_MUL
#define MR_BWD_GRID_MUL 1
#endif
  auto cap = [&](int gr) {  // enough waves for every tile, a multiple of 8 (XCD-partitioned slot ranges)
    gr *= MR_BWD_GRID_MUL;
    const int c = (int)(NT / 4 + 1 < gr ? NT / 4 + 1 : gr);
    return (c + 7) / 8 * 8;
  };
  static int f18 = 0, f27 = 0, f18c = 0, f27c = 0, g18 = 0, g27 = 0, g18c = 0, g27c = 0;
  if (!f18) f18 = resident_grid(k_bwd_fused<18, false>, 256, 3);
  if (!f27) f27 = resident_grid(k_bwd_fused<27, false>, 256, 2);
  if (!f18c) f18c = resident_grid(k_bwd_fused<18, true>, 256, 3);
  if (!f27c) f27c = resident_grid(k_bwd_fused<27, true>, 256, 2);
  if (!g18) g18 = resident_grid(k_bwd_fused<18, false, true>, 256, 4);
  if (!g27) g27 = resident_grid(k_bwd_fused<27, false, true>, 256, 4);
  if (!g18c) g18c = resident_grid(k_bwd_fused<18, true, true>, 256, 4);
  if (!g27c) g27c = resident_grid(k_bwd_fused<27, true, true>, 256, 4);
  // no RGB gradient (a depth / silhouette render's backward): the geometry-only instantiation
  const bool geo = P.gRGB == nullptr;
  // the drop-in Phong render (UV map with an 8-bit copy, point light, RGB, relu depth): the specialised one
#ifndef MR_BWD_SPEC
#define MR_BWD_SPEC 1
#endif
  const bool spec = MR_BWD_SPEC && !geo && !vcol && !s->clip_z && m->tex_kind == 2 && m->tex_u8 && m->tex_lut &&
                    sp->light_kind == 0 && sp->rgb_channels == 3 && !(sp->out_flags & (MR_OUT_ZBUF | MR_OUT_SIL_RGBA));
  static int f18s = 0;
  if (!f18s) f18s = resident_grid(k_bwd_fused<18, false, false, 1>, 256, 3);
  if (s->clip_z) {
    if (geo) {
      if (vcol) MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<27, true, true><<<cap(g27c), 256, 0, st>>>(P)));
      else MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<18, true, true><<<cap(g18c), 256, 0, st>>>(P)));
    } else if (vcol) MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<27, true><<<cap(f27c), 256, 0, st>>>(P)));
    else MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<18, true><<<cap(f18c), 256, 0, st>>>(P)));
  } else {
    if (geo) {
      if (vcol) MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<27, false, true><<<cap(g27), 256, 0, st>>>(P)));
      else MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<18, false, true><<<cap(g18), 256, 0, st>>>(P)));
    } else if (vcol) MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<27, false><<<cap(f27), 256, 0, st>>>(P)));
    else if (spec) MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<18, false, false, 1><<<cap(f18s), 256, 0, st>>>(P)));
    else MR_TIMED(KID_BWD_FUSED, st, (k_bwd_fused<18, false><<<cap(f18), 256, 0, st>>>(P)));
  }
  MR_CHECK_LAUNCH("k_bwd_fused");
  const int use_n = sp->light_kind == 0;
  const int vb = ceil_div(m->V * MR_VL, 256);
  // the forward's slot ranges: one per (view, band) on the per-view binning, one per view otherwise
  const int bands = view_binning(g, N, NF) ? bin_bands(N, g) : 1;
  RtReduce RR;
  RR.part = rt_part; RR.vslot = w.vslot; RR.N = (int)N; RR.bands = bands;
  RR.gviews = gviews; RR.gRcv = gRcv; RR.gtcv = gtcv;
  const int vbw = ceil_div(m->V * MR_VL, MR_VGRAD_NT);  // vertex-gather workgroups of k_rt_vgrad_a / _b
  if (!use_n) {  // no normal chain: the R/T reduction and the vertex gathers in one launch
    if (vcol) MR_TIMED(KID_RT_VGRAD_B, st, (k_rt_vgrad_b<27><<<(unsigned)(N + vbw), MR_VGRAD_NT, 0, st>>>(RR, m->V, m->vadj_ptr, m->vadj, gfix, gface, P.fflag, gverts, gcol)));
    else MR_TIMED(KID_RT_VGRAD_B, st, (k_rt_vgrad_b<18><<<(unsigned)(N + vbw), MR_VGRAD_NT, 0, st>>>(RR, m->V, m->vadj_ptr, m->vadj, gfix, gface, P.fflag, gverts, gcol)));
    MR_CHECK_LAUNCH("k_rt_vgrad_b");
    return MR_OK;
  }
  if (vcol) MR_TIMED(KID_RT_VGRAD_A, st, (k_rt_vgrad_a<27><<<(unsigned)(N + vbw), MR_VGRAD_NT, 0, st>>>(RR, m->V, m->vadj_ptr, m->vadj, gfix, gface, P.fflag, vraw, gnu)));
  else MR_TIMED(KID_RT_VGRAD_A, st, (k_rt_vgrad_a<18><<<(unsigned)(N + vbw), MR_VGRAD_NT, 0, st>>>(RR, m->V, m->vadj_ptr, m->vadj, gfix, gface, P.fflag, vraw, gnu)));
  MR_CHECK_LAUNCH("k_rt_vgrad_a");
  if (vcol) {
    MR_TIMED(KID_VGRAD_B, st, (k_vgrad_b<27><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, gfix, gface, P.fflag, gnu, use_n, gverts, gcol)));
  } else {
    MR_TIMED(KID_VGRAD_B, st, (k_vgrad_b<18><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, gfix, gface, P.fflag, gnu, use_n, gverts, gcol)));
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
  P.sorted = (sp->out_flags & MR_FRAG_SORTED) ? 1 : 0;
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
  const bool sil = (sp->out_flags & MR_OUT_SIL) != 0, hard = !sil && (sp->out_flags & MR_OUT_HARD);
  if (!grad_rgba || !fwd_ws || !bws || !g_verts || (!g_zbuf && !sil && !hard) || (!g_bary && !sil) ||
      (!g_dists && !hard))
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
    if ((g_zbuf && hipMemsetAsync(g_zbuf, 0, sizeof(float) * slots, st) != hipSuccess) ||
        (g_dists && hipMemsetAsync(g_dists, 0, sizeof(float) * slots, st) != hipSuccess) ||
        (g_bary && hipMemsetAsync(g_bary, 0, sizeof(float) * 3 * slots, st) != hipSuccess))
      return set_err(MR_ELAUNCH, "memset failed");
  }
  if (vcol) MR_TIMED(KID_FRAG_SHADE_BWD, st, (k_frag_shade_bwd<27><<<grid, 256, 0, st>>>(P)));
  else MR_TIMED(KID_FRAG_SHADE_BWD, st, (k_frag_shade_bwd<18><<<grid, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_frag_shade_bwd");
  // vertex gradients of the attribute rows (interpolated positions and normals, vertex colours)
  const int use_n = sp->light_kind == 0 && !P.sil;
  const int vb = ceil_div(m->V * MR_VL, 256);
  if (use_n) {
    RtReduce R0;
    memset(&R0, 0, sizeof(R0));
    R0.bands = 1;
    const int vbw = ceil_div(m->V * MR_VL, MR_VGRAD_NT);
    if (vcol) k_rt_vgrad_a<27><<<(unsigned)vbw, MR_VGRAD_NT, 0, st>>>(R0, m->V, m->vadj_ptr, m->vadj, nullptr, gface, nullptr, vraw, gnu);
    else k_rt_vgrad_a<18><<<(unsigned)vbw, MR_VGRAD_NT, 0, st>>>(R0, m->V, m->vadj_ptr, m->vadj, nullptr, gface, nullptr, vraw, gnu);
    MR_CHECK_LAUNCH("k_rt_vgrad_a");
  }
  if (vcol) k_vgrad_b<27><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, nullptr, gface, nullptr, gnu, use_n, g_verts, g_vcolors);
  else k_vgrad_b<18><<<vb, 256, 0, st>>>(m->V, m->verts, m->faces, m->vadj_ptr, m->vadj, nullptr, gface, nullptr, gnu, use_n, g_verts, g_vcolors);
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

int32_t mr_workspace_counters(const void* ws, int64_t N, int64_t Ftot, int32_t H, int32_t W, int32_t mfpb, int32_t* out8,
                              void* stream) {
  if (!ws || !out8 || N <= 0 || N > 65535) return set_err(MR_EINVAL, "bad arguments");
  hipStream_t st = (hipStream_t)stream;
  BinGeom g = bin_geom(H, W, N, Ftot > 0 ? Ftot : 1, mfpb);
  RasterWS w = carve_raster_ws((void*)ws, N, Ftot > 0 ? Ftot : 1, H, W, g);
  if (hipMemcpyAsync(out8, w.ctr, sizeof(int) * CTR_COUNT, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return set_err(MR_ELAUNCH, "counter copy failed");
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
#ifdef MR_XP_BWD_STAMP
// experiment builds only: the last k_bwd_fused launch's per-wave stamps (8 u64 per wave, MR_XP_WAVES waves)
int32_t mr_xp_bwd_stamps(unsigned long long* out, int32_t waves) {
  if (waves > MR_XP_WAVES) waves = MR_XP_WAVES;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bwd_stamp), sizeof(unsigned long long) * 8 * (size_t)waves, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? MR_OK : MR_ELAUNCH;
}
#endif
#ifdef MR_XP_BV_STAMP
// experiment builds only: the last k_bin_view<MODE, CH> launch's per-workgroup stamps (8 u64 per workgroup)
int32_t mr_xp_bv_stamps(unsigned long long* out, int32_t wgs) {
  if (wgs > MR_XP_BV_WGS) wgs = MR_XP_BV_WGS;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bv_stamp), sizeof(unsigned long long) * 8 * (size_t)wgs, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? MR_OK : MR_ELAUNCH;
}
#endif

static int pose_loss_params(PoseLossParams& P, const float* depth, const float* sil, int64_t sil_stride,
                            const float* rgb, int64_t rgb_stride, const uint8_t* mask, const float* depth_ref,
                            const float* rgb_ref, int64_t npix, float delta, float w_color) {
  if (npix <= 0) return set_err(MR_EINVAL, "npix must be > 0");
  if (!depth || !sil || !rgb || !mask || !depth_ref || !rgb_ref) return set_err(MR_EINVAL, "NULL loss input");
  if (rgb_stride != 3 && rgb_stride != 4) return set_err(MR_EINVAL, "rgb_stride must be 3 or 4");
  if (sil_stride != 1 && sil_stride != 4) return set_err(MR_EINVAL, "sil_stride must be 1 or 4");
  if (!(delta > 0.0f)) return set_err(MR_EINVAL, "huber delta must be > 0");
  P.depth = depth; P.sil = sil; P.sil_stride = sil_stride; P.rgb = rgb; P.rgb_stride = rgb_stride; P.mask = mask;
  P.depth_ref = depth_ref; P.rgb_ref = rgb_ref; P.npix = npix; P.delta = delta; P.w_color = w_color;
  return MR_OK;
}

// Loss workspace: per-block partials of the one-pixel-per-thread pass (3 floats + a count per 256
// pixels), the masked-pixel total, k_mask_count's partials and the backward's count.
struct LossWS {
  float* part;
  int* pcnt;
  int64_t* count;
  int64_t* mtot;
  int* mcnt;
  size_t bytes;
};
static LossWS carve_loss(void* ws, int64_t npix) {
  const size_t nb = (size_t)std::max<int64_t>(ceil_div(npix, 256 * MR_LOSS_PPT), 1);
  LossWS w;
  char* b = (char*)ws;
  size_t off = 0;
  w.part = (float*)(b + off);
  off = align_up(off + sizeof(float) * 3 * nb, 256);
  w.pcnt = (int*)(b + off);
  off = align_up(off + sizeof(int) * nb, 256);
  w.count = (int64_t*)(b + off);
  w.mtot = w.count + 1;
  off = align_up(off + 2 * sizeof(int64_t), 256);
  w.mcnt = (int*)(b + off);
  off = align_up(off + sizeof(int) * MR_LOSS_BLOCKS, 256);
  w.bytes = off;
  return w;
}

size_t mr_pose_loss_workspace(int64_t npix) { return carve_loss(nullptr, npix).bytes; }

// The loss (and, with gradient buffers, its gradients for dL/dtotal = 1): mask count, one pass over the
// pixels, final reduction.
static int32_t pose_loss_run(const PoseLossParams& P, float* total, float* terms, void* ws, float* g_depth,
                             float* g_sil, float* g_rgb, hipStream_t st) {
  LossWS w = carve_loss(ws, P.npix);
  const int64_t nb = ceil_div(P.npix, 256 * MR_LOSS_PPT);
  if (nb >= (1ll << 31)) return set_err(MR_EUNSUPPORTED, "npix too large");
  const bool grads = g_depth != nullptr;
  if (grads) {
    const int nm = (int)std::min<int64_t>(MR_LOSS_BLOCKS, ceil_div(P.npix, 256));
    k_mask_count<<<nm, 256, 0, st>>>(P.mask, P.npix, w.mcnt);
    MR_CHECK_LAUNCH("k_mask_count");
    k_mask_total<<<1, 256, 0, st>>>(w.mcnt, nm, w.mtot);
    MR_CHECK_LAUNCH("k_mask_total");
    MR_TIMED(KID_POSE_LOSS, st, (k_pose_loss_fused<true><<<(unsigned)nb, 256, 0, st>>>(P, w.mtot, w.part, w.pcnt, g_depth, g_sil, g_rgb)));
  } else {
    MR_TIMED(KID_POSE_LOSS, st, (k_pose_loss_fused<false><<<(unsigned)nb, 256, 0, st>>>(P, w.mtot, w.part, w.pcnt, nullptr, nullptr, nullptr)));
  }
  MR_CHECK_LAUNCH("k_pose_loss_fused");
  k_pose_loss_final<<<1, 1024, 0, st>>>(P, w.part, w.pcnt, (int)nb, total, terms, w.count);
  MR_CHECK_LAUNCH("k_pose_loss_final");
  return MR_OK;
}

int32_t mr_pose_loss_forward(const float* depth, const float* sil, int64_t sil_stride, const float* rgb,
                             int64_t rgb_stride, const uint8_t* mask, const float* depth_ref, const float* rgb_ref,
                             int64_t npix, float delta, float w_color, float* out, void* ws, size_t ws_bytes,
                             void* stream) {
  PoseLossParams P;
  int rc = pose_loss_params(P, depth, sil, sil_stride, rgb, rgb_stride, mask, depth_ref, rgb_ref, npix, delta, w_color);
  if (rc) return rc;
  if (!out || !ws) return set_err(MR_EINVAL, "NULL output / workspace");
  if (ws_bytes < mr_pose_loss_workspace(npix)) return set_err(MR_EWORKSPACE, "loss workspace too small");
  return pose_loss_run(P, out, out + 1, ws, nullptr, nullptr, nullptr, (hipStream_t)stream);
}

// The forward writing the gradients for dL/dtotal = 1 too (see k_pose_loss_fused); mr_pose_loss_scale
// turns them into the backward's for any dL/dtotal.
int32_t mr_pose_loss_forward_grad(const float* depth, const float* sil, int64_t sil_stride, const float* rgb,
                                  int64_t rgb_stride, const uint8_t* mask, const float* depth_ref, const float* rgb_ref,
                                  int64_t npix, float delta, float w_color, float* total, float* terms, void* ws,
                                  size_t ws_bytes, float* g_depth, float* g_sil, float* g_rgb, void* stream) {
  PoseLossParams P;
  int rc = pose_loss_params(P, depth, sil, sil_stride, rgb, rgb_stride, mask, depth_ref, rgb_ref, npix, delta, w_color);
  if (rc) return rc;
  if (!total || !terms || !ws) return set_err(MR_EINVAL, "NULL output / workspace");
  const bool grads = g_depth || g_sil || g_rgb;
  if (grads && !(g_depth && g_sil && g_rgb)) return set_err(MR_EINVAL, "gradient buffers: all three or none");
  if (ws_bytes < mr_pose_loss_workspace(npix)) return set_err(MR_EWORKSPACE, "loss workspace too small");
  if (grads && ((sil_stride == 4 && ((uintptr_t)g_sil & 15)) || (rgb_stride == 4 && ((uintptr_t)g_rgb & 15))))
    return set_err(MR_EINVAL, "RGBA gradient buffers must be 16-byte aligned");
  return pose_loss_run(P, total, terms, ws, g_depth, g_sil, g_rgb, (hipStream_t)stream);
}

int32_t mr_pose_loss_scale(const float* g_total, int64_t npix, int64_t sil_stride, int64_t rgb_stride, float* g_depth,
                           float* g_sil, float* g_rgb, void* stream) {
  if (npix <= 0) return set_err(MR_EINVAL, "npix must be > 0");
  if (!g_total || !g_depth || !g_sil || !g_rgb) return set_err(MR_EINVAL, "NULL argument");
  if ((sil_stride != 1 && sil_stride != 4) || (rgb_stride != 3 && rgb_stride != 4))
    return set_err(MR_EINVAL, "bad strides");
  hipStream_t st = (hipStream_t)stream;
  MR_TIMED(KID_POSE_LOSS_SCALE, st, (k_pose_loss_scale<<<1024, 256, 0, st>>>(g_total, npix, npix * sil_stride, npix * rgb_stride,
                                                                             g_depth, g_sil, g_rgb)));
  MR_CHECK_LAUNCH("k_pose_loss_scale");
  return MR_OK;
}

int32_t mr_pose_loss_backward(const float* depth, const float* sil, int64_t sil_stride, const float* rgb,
                              int64_t rgb_stride, const uint8_t* mask, const float* depth_ref, const float* rgb_ref,
                              int64_t npix, float delta, float w_color, const float* g_total, const void* fwd_ws,
                              float* g_depth, float* g_sil, float* g_rgb, void* stream) {
  PoseLossParams P;
  int rc = pose_loss_params(P, depth, sil, sil_stride, rgb, rgb_stride, mask, depth_ref, rgb_ref, npix, delta, w_color);
  if (rc) return rc;
  if (!g_total || !fwd_ws || !g_depth || !g_sil || !g_rgb) return set_err(MR_EINVAL, "NULL gradient argument");
  const int64_t* count = carve_loss((void*)fwd_ws, npix).count;
  if ((sil_stride == 4 && ((uintptr_t)g_sil & 15)) || (rgb_stride == 4 && ((uintptr_t)g_rgb & 15)))
    return set_err(MR_EINVAL, "RGBA gradient buffers must be 16-byte aligned");
  k_pose_loss_bwd<<<(unsigned)ceil_div(npix, 256), 256, 0, (hipStream_t)stream>>>(P, g_total, count, g_depth, g_sil, g_rgb);
  MR_CHECK_LAUNCH("k_pose_loss_bwd");
  return MR_OK;
}

int32_t mr_quaternion_to_matrix(const float* q, int64_t q_stride, int64_t N, float* R, void* stream) {
  if (N < 0 || q_stride < 4) return set_err(MR_EINVAL, "bad quaternion batch");
  if (N == 0) return MR_OK;
  if (!q || !R) return set_err(MR_EINVAL, "NULL argument");
  k_quat_to_matrix<<<ceil_div(N, 256), 256, 0, (hipStream_t)stream>>>(q, q_stride, N, R);
  MR_CHECK_LAUNCH("k_quat_to_matrix");
  return MR_OK;
}

int32_t mr_quaternion_to_matrix_backward(const float* q, int64_t q_stride, const float* gR, int64_t N, float* gq,
                                         void* stream) {
  if (N < 0 || q_stride < 4) return set_err(MR_EINVAL, "bad quaternion batch");
  if (N == 0) return MR_OK;
  if (!q || !gR || !gq) return set_err(MR_EINVAL, "NULL argument");
  k_quat_to_matrix_bwd<<<ceil_div(N, 256), 256, 0, (hipStream_t)stream>>>(q, q_stride, gR, N, gq);
  MR_CHECK_LAUNCH("k_quat_to_matrix_bwd");
  return MR_OK;
}

}  // extern "C"
