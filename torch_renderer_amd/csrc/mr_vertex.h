// mi355r — Vertex kernels: normals and the gradient gathers through the CSR vertex adjacency.
// Part of the single translation unit mr_raster.hip (included there, in this order).
#pragma once

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

// A: gNu[v] = normalize_bwd(raw[v], sum of the face totals' normal rows)
// (face totals: fixed-point gfix + float gface on the fused path, gfix NULL: float gface alone)
#define MR_VL 8  // lanes per vertex in the CSR gathers of the vertex-gradient kernels
template <int ACC>
MR_DEV void vgrad_a_block(int64_t V, const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj,
                          const unsigned long long* __restrict__ gfix, const float* __restrict__ gface,
                          const int* __restrict__ fflag, const float* __restrict__ vraw, float* __restrict__ gnu,
                          int64_t blk) {
  const bool rem = !fflag || *fflag != 0;  // float remainder rows written (else all zero: not read)
  // MR_VL lanes per vertex split its CSR entries, then a fixed xor-tree sums them (deterministic)
  const int64_t gid = blk * blockDim.x + threadIdx.x;
  const int64_t v = gid / MR_VL;
  const int j = (int)(gid % MR_VL);
  const bool act = v < V;
  float g[3] = {0.f, 0.f, 0.f};
  if (act) {
    for (int e = ptr[v] + j; e < ptr[v + 1]; e += MR_VL) {
      const int f = adj[e] >> 2, c = adj[e] & 3;
      float t[3];
      fix_totals<3>(gfix, gface, (int64_t)f * ACC + col_nrm<ACC>(c, 0), rem, t);
      for (int k = 0; k < 3; ++k) g[k] += t[k];
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
// The vertex gathers' blocks in XCD-contiguous order: the hardware deals a launch's workgroups round-robin over
// the 8 XCDs (each with its own L2), so block j of nb is remapped to vertex range x * nb / 8 + j / 8 of its XCD x
// (= j mod 8 up to a fixed rotation) — neighbouring vertices, which gather the same face rows, share an L2
// instead of fetching each row from HBM once per XCD. A bijection on [0, nb).
MR_DEV int64_t xcd_block(int64_t j, int64_t nb) {
  const int64_t x = j & 7, q = nb >> 3, r = nb & 7;
  return x * q + (x < r ? x : r) + (j >> 3);
}
// (blocks [0, N): rt_reduce_view, one workgroup per view)
struct RtReduce {
  const float* part;
  const int* vslot;
  int N, bands;
  float *gviews, *gRcv, *gtcv;
};
// threads per workgroup of k_rt_vgrad_a / _b: the view reduction's rows in flight (C5's single view: k_rt_vgrad_b
// 22.3 us at 256, 18.9-19.2 at 512; 1024 slowed the headline's k_rt_vgrad_a 7.6 -> 8.7 us; r6n_vgrad_nt_ab.txt)
#ifndef MR_VGRAD_NT
#define MR_VGRAD_NT 512
#endif
template <int ACC>
__global__ void __launch_bounds__(MR_VGRAD_NT) k_rt_vgrad_a(RtReduce R, int64_t V,
                                                            const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj,
                                                            const unsigned long long* __restrict__ gfix,
                                                            const float* __restrict__ gface, const int* __restrict__ fflag,
                                                            const float* __restrict__ vraw, float* __restrict__ gnu) {
  if ((int)blockIdx.x < R.N) rt_reduce_view<MR_VGRAD_NT>(R.part, R.vslot, R.N, R.bands, R.gviews, R.gRcv, R.gtcv, blockIdx.x);
  else vgrad_a_block<ACC>(V, ptr, adj, gfix, gface, fflag, vraw, gnu,
                          xcd_block((int64_t)blockIdx.x - R.N, (int64_t)gridDim.x - R.N));
}

// B: grad_verts[v] = sum over incident (f, c) of position rows + cross-product backward of the face normal.
template <int ACC>
MR_DEV void vgrad_b_block(int64_t V, const float* __restrict__ verts, const int32_t* __restrict__ faces,
                          const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj,
                          const unsigned long long* __restrict__ gfix, const float* __restrict__ gface,
                          const int* __restrict__ fflag, const float* __restrict__ gnu, int use_normals,
                          float* __restrict__ gverts, float* __restrict__ gcol, int64_t blk) {
  const bool rem = !fflag || *fflag != 0;  // float remainder rows written (else all zero: not read)
  const int64_t gid = blk * blockDim.x + threadIdx.x;
  const int64_t v = gid / MR_VL;
  const int j = (int)(gid % MR_VL);
  const bool act = v < V;
  float g[3] = {0.f, 0.f, 0.f}, gc[3] = {0.f, 0.f, 0.f};
  const int e0 = act ? ptr[v] + j : 0, e1 = act ? ptr[v + 1] : 0;
  for (int e = e0; e < e1; e += MR_VL) {
    const int f = adj[e] >> 2, c = adj[e] & 3;
    if (ACC == 27) {  // a corner's position and colour columns are adjacent: 48 B in three 16-B loads
      float t[6];
      fix_totals<6>(gfix, gface, (int64_t)f * ACC + col_pos<ACC>(c, 0), rem, t);
      for (int k = 0; k < 3; ++k) {
        g[k] += t[k];
        gc[k] += t[3 + k];
      }
    } else {
      float t[3];
      fix_totals<3>(gfix, gface, (int64_t)f * ACC + col_pos<ACC>(c, 0), rem, t);
      for (int k = 0; k < 3; ++k) g[k] += t[k];
    }
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
template <int ACC>
__global__ void __launch_bounds__(256) k_vgrad_b(int64_t V, const float* __restrict__ verts,
                                                 const int32_t* __restrict__ faces, const int32_t* __restrict__ ptr,
                                                 const int32_t* __restrict__ adj, const unsigned long long* __restrict__ gfix,
                                                 const float* __restrict__ gface, const int* __restrict__ fflag,
                                                 const float* __restrict__ gnu, int use_normals, float* __restrict__ gverts,
                                                 float* __restrict__ gcol) {
  vgrad_b_block<ACC>(V, verts, faces, ptr, adj, gfix, gface, fflag, gnu, use_normals, gverts, gcol,
                     xcd_block(blockIdx.x, gridDim.x));
}
// Without vertex normals in the shading (no k_vgrad_a step): the per-view R/T reduction (blocks [0, N)) and
// the vertex gradients (the rest) read disjoint inputs, so one launch runs both side by side (C5: a single
// view's reduction is one long-running workgroup that the gathers now overlap).
template <int ACC>
__global__ void __launch_bounds__(MR_VGRAD_NT) k_rt_vgrad_b(RtReduce R, int64_t V, const int32_t* __restrict__ ptr,
                                                            const int32_t* __restrict__ adj,
                                                            const unsigned long long* __restrict__ gfix,
                                                            const float* __restrict__ gface, const int* __restrict__ fflag,
                                                            float* __restrict__ gverts, float* __restrict__ gcol) {
  if ((int)blockIdx.x < R.N) rt_reduce_view<MR_VGRAD_NT>(R.part, R.vslot, R.N, R.bands, R.gviews, R.gRcv, R.gtcv, blockIdx.x);
  else vgrad_b_block<ACC>(V, nullptr, nullptr, ptr, adj, gfix, gface, fflag, nullptr, 0, gverts, gcol,
                          xcd_block((int64_t)blockIdx.x - R.N, (int64_t)gridDim.x - R.N));
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
