// mi355r — Binning: wave / workgroup scan primitives, then the count -> scan -> fill path and the
// per-view path (k_bin_rect_* -> k_bin_view) that build each 8x8 tile's face list and the raster's work units.
// Part of the single translation unit mr_raster.hip (included there, in this order).
#pragma once

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
  int* bcnt;  // band-list counts cleared by the record launch (nbcnt of them)
  int nbcnt;
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

// Four inclusive scans over a 1024-thread workgroup in one pass: the four DPP wave scans, ONE LDS exchange
// of the 4 x 16 wave totals, two LDS-only barriers (three block_incl_sum calls take six). Uniform call only.
MR_DEV void block_incl_sum4(const int (&v)[4], int (*part4)[16], int (&incl)[4], int (&tot)[4]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) w[k] = wave_incl_sum(v[k]);
  if (lane == 63) {
#pragma unroll
    for (int k = 0; k < 4; ++k) part4[k][wave] = w[k];
  }
  lds_barrier();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ws = wave_incl_sum(lane < 16 ? part4[k][lane] : 0);
    tot[k] = __builtin_amdgcn_readlane(ws, 15);
    const int before = __shfl(ws, wave > 0 ? wave - 1 : 0, 64);
    incl[k] = w[k] + (wave > 0 ? before : 0);
  }
  lds_barrier();  // part4 is reused by the next call
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
#ifndef MR_VIEW_FMAX
#define MR_VIEW_FMAX 1048576            // faces per view (mean) above which the count -> scan path is used
#endif
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
  float4* zero4;   // the fused backward's fixed-point face totals, cleared here (nzero4 16-B words; NULL: none)
  int64_t nzero4;
  float4* zero4b;  // ... and their float remainder rows (nzero4b 16-B words)
  int64_t nzero4b;
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
// m 16-B words per pixel quad of a chunk of nq quads, all of the same value, written
// lane-contiguously: store k of the wave covers the chunk's words [64 k, 64 k + 64) (one 1-KB
// burst per store instruction; a lane writing its quad's m consecutive words strides every store
// by 16 m bytes: fragment pass 164 -> 161 us, tools/micro/store_bw.hip 103 -> 89 us for the whole
// fragment background). The fused render's background keeps the per-lane layout: its
// lane-contiguous version measured 221 -> 244 us per step (profiles/r3s_fill_ab.txt).
template <int M, typename T4>
MR_DEV void fill_words(T4* __restrict__ base, int nq, int lane, const T4& v) {
#pragma unroll
  for (int k = 0; k < M; ++k)
    if (k * 64 + lane < M * nq) base[k * 64 + lane] = v;
}

// PyTorch3D fragment background chunks (64 pixel quads each, view-major, W % 4 == 0) that a
// k_bin_rect_world launch writes from grid rows past the views: the record pass stores ~100 B per
// face at ~2.6 TB/s, so its launch has store bandwidth to spare for part of the 470-MB background
// the binning and raster launches otherwise stream (count 0: none).
struct FragBg {
  int64_t* p2f;
  float *zbuf, *dists, *bary;
  int H, W, nviews;
  int first, count;  // chunks [first, first + count)
};
MR_DEV void frag_bg_rows(const FragBg& B, int row) {
  const int lane = threadIdx.x & 63;
  const int w = (row * (int)gridDim.x + (int)blockIdx.x) * 4 + (int)(threadIdx.x >> 6);
  const int G = ((int)gridDim.y - 1 - B.nviews) * (int)gridDim.x * 4;
  const int64_t HW = (int64_t)B.H * B.W;
  const int cpv = (int)((HW / 4 + 63) / 64);
  const float4 m1 = make_float4(-1.f, -1.f, -1.f, -1.f);
  const longlong2 l1 = make_longlong2(-1ll, -1ll);
#pragma unroll 1
  for (int c = B.first + w; c < B.first + B.count; c += G) {
    const int n = c / cpv;
    const int64_t q0 = (int64_t)(c - n * cpv) * 64;
    const int nq = (int)min((int64_t)64, HW / 4 - q0);
    const int64_t pix = (int64_t)n * HW + 4 * q0;
    fill_words<2>((longlong2*)(B.p2f + pix), nq, lane, l1);
    fill_words<1>((float4*)(B.zbuf + pix), nq, lane, m1);
    fill_words<1>((float4*)(B.dists + pix), nq, lane, m1);
    fill_words<3>((float4*)(B.bary + pix * 3), nq, lane, m1);
  }
}

template <bool CLIP>
__global__ void __launch_bounds__(256) k_bin_rect_world(SetupParams P, const float* __restrict__ verts,
                                                        const int32_t* __restrict__ faces, int64_t F,
                                                        const ViewRec* __restrict__ views, NormalsArgs NA,
                                                        int* __restrict__ ctr, CvPoses C, FragBg B) {
  const int n = (int)blockIdx.y - 1;
  if (B.count > 0 && n >= B.nviews) {
    frag_bg_rows(B, n - B.nviews);
    return;
  }
  if (n >= 0 && C.R && blockIdx.x == 0 && threadIdx.x < 16) C.out[(int64_t)n * 16 + threadIdx.x] = cv_view_elem(C, n, threadIdx.x);
  if (n < 0) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < CTR_COUNT) ctr[threadIdx.x] = 0;
    for (int64_t i = v; i < P.nbcnt; i += (int64_t)gridDim.x * blockDim.x) P.bcnt[i] = 0;
    for (int64_t i = v; i < NA.nzero4; i += (int64_t)gridDim.x * blockDim.x) NA.zero4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = v; i < NA.nzero4b; i += (int64_t)gridDim.x * blockDim.x) NA.zero4b[i] = make_float4(0.f, 0.f, 0.f, 0.f);
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
  int T, TX, TY, mfpb, clipz;
  int nviews;
  int bands;   // workgroups per view: band b bins tile rows [b TY / bands, (b + 1) TY / bands)
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
  int srec_fpw;  // faces per ShadeRec workgroup (a multiple of 256: srec_wgs)
  int stage_cap;  // list entries of a view staged in LDS (after the histogram)
  // bands > 1: the records of each (view, band) listed by k_band_bucket (blist[(n B + b) bcap + e],
  // bcnt[n B + b] of them); NULL: every band reads all of the view's rectangles
  const int* blist;
  const int* bcnt;
  int64_t bcap;
};

// The band holding tile row ty (bands b hold rows [b TY / B, (b + 1) TY / B)).
MR_DEV int band_of(int ty, int TY, int B) { return ((ty + 1) * B - 1) / TY; }


// Tiles of a rectangle (0 for MR_RECT_NONE).
MR_DEV int rect_size(uint32_t r) {
  const int tx0 = r & 255, tx1 = (r >> 8) & 255, ty0 = (r >> 16) & 255, ty1 = r >> 24;
  return tx1 < tx0 ? 0 : (tx1 - tx0 + 1) * (ty1 - ty0 + 1);
}

// Band lists for the banded per-view binning of one shared mesh: every record of view n (one thread per
// face, both triangles of a split face) is appended to the list of each band its tile rectangle meets,
// one global atomic per (band, workgroup) — so a band's workgroup in k_bin_view reads its ~F / B records
// instead of all F rectangles of the view (C5: 81,920 faces, one view, 64 bands). The order inside a list
// is arbitrary; nothing downstream depends on it (the raster's keys are order-free, the backward groups a
// tile's pixels by record, slots stay in tile order).
__global__ void __launch_bounds__(1024) k_band_bucket(const uint32_t* __restrict__ rects, int64_t F, int64_t NF, int nq,
                                                       int TY, int B, int* __restrict__ bcnt, int* __restrict__ blist,
                                                       int64_t bcap) {
  __shared__ int lcnt[MR_BANDS_MAX], lbase[MR_BANDS_MAX];
  const int n = blockIdx.y, t = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * 1024 + t;
  if (t < B) lcnt[t] = 0;
  __syncthreads();
  int rid[2], b0[2], b1[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    rid[q] = (int)((q ? NF : 0) + (int64_t)n * F + i);
    const uint32_t r = (q < nq && i < F) ? rects[rid[q]] : MR_RECT_NONE;
    const bool any = rect_size(r) > 0;
    b0[q] = any ? band_of((int)((r >> 16) & 255), TY, B) : 1;
    b1[q] = any ? band_of((int)(r >> 24), TY, B) : 0;
    for (int b = b0[q]; b <= b1[q]; ++b) atomicAdd(&lcnt[b], 1);
  }
  __syncthreads();
  if (t < B) {
    lbase[t] = lcnt[t] > 0 ? atomicAdd(&bcnt[n * B + t], lcnt[t]) : 0;
    lcnt[t] = 0;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q)
    for (int b = b0[q]; b <= b1[q]; ++b) {
      const int pos = lbase[b] + atomicAdd(&lcnt[b], 1);
      if (pos < bcap) blist[(int64_t)(n * B + b) * bcap + pos] = rid[q];
    }
}

// The band-local tiles (ty - by0) * TX + tx of rectangle r inside tile rows [by0, by1).
template <typename Fn>
MR_DEV void rect_tiles(uint32_t r, int TX, int by0, int by1, Fn&& fn) {
  const int tx0 = r & 255, tx1 = (r >> 8) & 255;
  const int ty0 = max((int)((r >> 16) & 255), by0), ty1 = min((int)(r >> 24), by1 - 1);
  for (int ty = ty0; ty <= ty1; ++ty)
    for (int tx = tx0; tx <= tx1; ++tx) fn((ty - by0) * TX + tx);
}

// One 1024-thread workgroup per (view, band of tile rows): every band reads all of the view's
// rectangles (4 B each, L2-resident after the first band) and bins the part of each inside its rows.
// Bands share nothing, so a view's binning runs on `bands` CUs at once instead of one (a single
// workgroup per view was the fragment pass's 26-us critical path with 64 views on 256 CUs).
#ifdef MR_XP_BV_STAMP  // experiment builds only: phase ends of a binning workgroup (k_bin_view's stamps)
__shared__ unsigned long long g_bv_ph[5];
#define BV_PH(i) do { if (threadIdx.x == 0) g_bv_ph[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define BV_PH(i) do { } while (0)
#endif
MR_DEV void bin_view_body(const ViewBinParams& P) {
  extern __shared__ __attribute__((aligned(16))) int hist[];  // Tb (+ Tb/64 pad): counts, then fill cursors
  __shared__ int part[16];
  __shared__ int part4[4][16];
  __shared__ long long base[3];
  __shared__ int nmulti;
  __shared__ int multi_slot[MR_SCAN_MULTI];
  const int blk = blockIdx.x, t = threadIdx.x;
  const int B = P.bands;
  if (blk >= P.nviews * B) {  // ShadeRec workgroups (they run on the CUs the views leave idle)
    const int64_t fa = (int64_t)(blk - P.nviews * B) * P.srec_fpw;
    const int64_t nf = P.Fs - fa < P.srec_fpw ? P.Fs - fa : P.srec_fpw;
    if (nf > 0) pack_shade_recs(P.S, P.srec, fa, nf, (float*)hist);
    return;
  }
  const int n = blk / B, b = blk - n * B;
  const int by0 = b * P.TY / B, by1 = (b + 1) * P.TY / B;  // this band's tile rows
  const int T0 = by0 * P.TX, Tb = (by1 - by0) * P.TX;      // its first tile and tile count
  // band tile lt lives at hist[lt + lt / 64] (the scan's per-thread runs of C tiles spread over the
  // banks); a view's rectangles are read in chunks of MR_VIEW_RPT per thread, all loads of a
  // chunk in flight together, and a view of one chunk keeps them in registers for the fill.
  const int j = t;
  const int64_t f0 = P.first ? P.first[n] : (int64_t)n * P.F;
  const int vcount = (int)(P.view_count ? (P.view_count[n] < 0x7fffffffll ? P.view_count[n] : 0x7fffffffll) : P.F);
  const int HS = (Tb + (Tb >> 6) + 3) & ~3;  // the histogram's ints (padded)
  for (int i = t; i < HS; i += 1024) hist[i] = 0;
  if (t == 0) nmulti = 0;
  lds_barrier();
  BV_PH(0);
  const int nq = P.clipz ? 2 : 1;
  // the entries this workgroup bins: the view's records (both triangles of a split face per entry), or
  // with band lists the records k_band_bucket listed for this band (one per entry)
  const bool lists = P.blist != nullptr;
  const int* bl = lists ? P.blist + (int64_t)blk * P.bcap : nullptr;
  const int nent = lists ? (int)min((int64_t)P.bcnt[blk], P.bcap) : vcount;
  uint32_t rr[MR_VIEW_RPT][2];
  int rid_[MR_VIEW_RPT][2];
  auto load_chunk = [&](int i0) {
    if (lists) {
#pragma unroll
      for (int k = 0; k < MR_VIEW_RPT; ++k) {
        const int i = i0 + k * 1024 + j;
        rid_[k][0] = i < nent ? bl[i] : 0;
        rid_[k][1] = 0;
      }
#pragma unroll
      for (int k = 0; k < MR_VIEW_RPT; ++k) {
        rr[k][0] = i0 + k * 1024 + j < nent ? P.rects[rid_[k][0]] : MR_RECT_NONE;
        rr[k][1] = MR_RECT_NONE;
      }
      return;
    }
#pragma unroll
    for (int k = 0; k < MR_VIEW_RPT; ++k)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = i0 + k * 1024 + j;
        rid_[k][q] = (int)((q ? P.NF : 0) + f0 + i);
        rr[k][q] = (q < nq && i < vcount) ? P.rects[rid_[k][q]] : MR_RECT_NONE;
      }
  };
  // count
#pragma unroll 1
  for (int i0 = 0; i0 < nent; i0 += 1024 * MR_VIEW_RPT) {
    load_chunk(i0);
#pragma unroll
    for (int k = 0; k < MR_VIEW_RPT; ++k)
#pragma unroll
      for (int q = 0; q < 2; ++q) rect_tiles(rr[k][q], P.TX, by0, by1, [&](int tt) { atomicAdd(&hist[tt + (tt >> 6)], 1); });
  }
  lds_barrier();
  BV_PH(1);
  // scan: each thread owns a run of C consecutive tiles (entries, units, slots in tile order)
  const int C = (Tb + 1023) / 1024;
  const int t0 = min(t * C, Tb), t1 = min(t0 + C, Tb);
  int le = 0, my_u = 0, my_s = 0;
  for (int tt = t0; tt < t1; ++tt) {
    const int cc = hist[tt + (tt >> 6)];
    le += cc;
    const bool mo = P.mfpb > 0 && cc > P.mfpb;  // PyTorch3D's per-bin cap: the whole-view path
    my_u += cc == 0 ? 0 : mo ? 1 : (cc + MR_UE - 1) / MR_UE;
    my_s += cc > 0 ? 1 : 0;
  }
  // a view of one chunk keeps its rectangles in registers for the fill
  const bool one = nent <= 1024 * MR_VIEW_RPT;
  int sc_in[4] = {le, my_u, my_s, 0}, sc_incl[4], sc_tot[4];
  block_incl_sum4(sc_in, part4, sc_incl, sc_tot);
  const int te = sc_tot[0], au = sc_tot[1], as = sc_tot[2];
  const int ex0 = sc_incl[0] - le, iu = sc_incl[1], is = sc_incl[2];
  // the allocations from separate waves: their round trips overlap instead of queueing
  if (t == 0) {
    base[0] = atomicAdd(&P.ctr[CTR_UNITS], au);
  } else if (t == 64) {
    // slot range of (view, band): the R/T reduction walks a view's bands in order
    const int b1 = atomicAdd(&P.ctr[CTR_SLOTS], as);
    base[1] = b1;
    P.vslot[blk] = b1;
    P.vslot[P.nviews * B + blk] = as;
  } else if (t == 128) {
    base[2] = (long long)atomicAdd((unsigned long long*)(P.ctr + CTR_ENTRIES64), (unsigned long long)te);
  }
  lds_barrier();
  BV_PH(2);
  const long long vb = base[2];
  // tile list starts are absolute pool positions here (view base 0): a view's bands take separate
  // ranges of the pool. (Readers use vbase[n] + start[tile], as on the count -> scan path.)
  if (t == 0 && b == 0) P.vbase[n] = 0;
  int u0 = (int)base[0] + iu - my_u, slot = (int)base[1] + is - my_s;
  for (int tt = t0, ex = ex0; tt < t1; ++tt) {
    const int cc = hist[tt + (tt >> 6)];
    const int gt = n * P.T + T0 + tt;
    if (P.ranges) {
      P.cnt[gt] = cc;
      // clamped: a list past the pool's end keeps start + cnt > list_cap (its overflow test)
      P.start[gt] = (int)min(vb + ex, (long long)P.list_cap);
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
  BV_PH(3);
  const int nm = min(nmulti, MR_SCAN_MULTI);
  for (int i = t; i < nm * 64; i += 1024) P.tkey[(int64_t)multi_slot[i >> 6] * 64 + (i & 63)] = MR_KEY_EMPTY;
  // fill: the band's entries occupy [vb, vb + te) of the pool; the first stage_cap of them are
  // staged in LDS and stored as consecutive lines afterwards (scattered 4-B stores issue one
  // lane per cycle), the rest (a band larger than the stage) go straight to the pool
  int* stage = hist + HS;
  const int lst = min(te, P.stage_cap);
#pragma unroll 1
  for (int i0 = 0; i0 < nent; i0 += 1024 * MR_VIEW_RPT) {
    if (!one) load_chunk(i0);
#pragma unroll
    for (int k = 0; k < MR_VIEW_RPT; ++k)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int rid = rid_[k][q];
        rect_tiles(rr[k][q], P.TX, by0, by1, [&](int tt) {
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
  BV_PH(4);
  for (int i = t; i < lst; i += 1024)
    if (vb + i < P.list_cap) P.list[vb + i] = stage[i];
}
__global__ void __launch_bounds__(1024) k_bin_view(ViewBinParams P) { bin_view_body(P); }
