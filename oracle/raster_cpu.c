/*
 * ORACLE — test infrastructure only. NOT part of the product path.
 *
 * Plain-C restatement of PyTorch3D's CPU mesh rasterizer, the algorithm the
 * reference repo reaches on the CPU through
 *   torch_renderer.py:97-121,141-159   (MeshRasterizer / MeshRenderer calls)
 *   renderer.py:87-101
 * -> pytorch3d.renderer.mesh.rasterize_meshes.rasterize_meshes (bin_size=0 on CPU)
 * -> pytorch3d._C.rasterize_meshes  == RasterizeMeshesNaiveCpu        (forward)
 * -> pytorch3d._C.rasterize_meshes_backward == RasterizeMeshesBackwardCpu
 * PyTorch3D (facebookresearch/pytorch3d, >= 0.5, version unpinned by the
 * reference) is NOT vendored under /root/reference and is not installed, so
 * this file restates the published algorithm (csrc/rasterize_meshes/
 * rasterize_meshes_cpu.cpp + csrc/utils/geometry_utils.h) as described in
 * SURVEY.md §8a rows a6/a7.  Parity is therefore pinned by analytic
 * known-answer tests and a float64 NumPy spec (oracle/spec_np.py), not by
 * reference-produced vectors (the reference holds none: SURVEY.md §4, §8c).
 *
 * Floating point: every expression keeps PyTorch3D's operand order; build with
 * -ffp-contract=off so no FMA contraction happens (x86 PyTorch builds do not
 * contract these scalar loops either).  kEpsilon is the *double* 1e-8 as in
 * geometry_utils.h (`const auto kEpsilon = 1e-8;` on non-MSVC builds), so
 * `area = E(v2,v0,v1) + kEpsilon` is evaluated in double and rounded to float.
 *
 * Deliberate, documented divergences from PyTorch3D:
 *   - faces whose projected coordinates are non-finite are skipped
 *     (PyTorch3D's std::sort over NaN keys is undefined behaviour);
 *   - the final K entries are written in ascending (z, face) order (the CUDA
 *     path's order; identical to CPU for K=1);
 *   - z-clipping: clipped_faces_neighbor_idx (the two triangles a face clipped
 *     into a quadrilateral is split into) follows the CPU rule as restated in
 *     orc_raster_fwd_ex; the clipping itself is restated in oracle.py.
 *
 * Also restated here: the world->NDC projection used by the MI355X kernels
 * (explicit operand order, see DESIGN.md "Projection"), so parity tests can
 * feed bit-identical face_verts to both sides.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define K_EPS_D 1e-8 /* geometry_utils.h: const auto kEpsilon = 1e-8 (double) */

typedef struct { float x, y; } v2f;

/* std::max / std::min semantics (a < b ? b : a), including NaN propagation */
static inline float smax(float a, float b) { return (a < b) ? b : a; }
static inline float smin(float a, float b) { return (b < a) ? b : a; }

/* geometry_utils.h EdgeFunctionForward */
static inline float edge_fn(v2f p, v2f a, v2f b) {
  return (p.x - a.x) * (b.y - a.y) - (p.y - a.y) * (b.x - a.x);
}

static inline float dot2(v2f a, v2f b) { return a.x * b.x + a.y * b.y; }

/* rasterization_utils.h NonSquareNdcRange / PixToNonSquareNdc */
static inline float pix_to_ndc(int i, int S1, int S2) {
  float range = 2.0f;
  if (S1 > S2) range = ((float)S1 * range) / (float)S2;
  const float offset = range / 2.0f;
  return -offset + (range * (float)i + offset) / (float)S1;
}

/* geometry_utils.h BarycentricCoordinatesForward */
static inline void bary_fwd(v2f p, v2f v0, v2f v1, v2f v2, float w[3]) {
  const float area = (float)((double)edge_fn(v2, v0, v1) + K_EPS_D);
  w[0] = edge_fn(p, v1, v2) / area;
  w[1] = edge_fn(p, v2, v0) / area;
  w[2] = edge_fn(p, v0, v1) / area;
}

/* geometry_utils.h BarycentricPerspectiveCorrectionForward */
static inline void persp_fwd(const float b[3], float z0, float z1, float z2, float o[3]) {
  const float w0_top = b[0] * z1 * z2;
  const float w1_top = b[1] * z0 * z2;
  const float w2_top = b[2] * z0 * z1;
  const float denom = smax(w0_top + w1_top + w2_top, (float)K_EPS_D); /* std::max<T>(., kEpsilon) */
  o[0] = w0_top / denom;
  o[1] = w1_top / denom;
  o[2] = w2_top / denom;
}

/* geometry_utils.h BarycentricClipForward: clamp below at 0, renormalise */
static inline void clip_fwd(const float b[3], float o[3]) {
  const float w0 = smax(b[0], 0.0f), w1 = smax(b[1], 0.0f), w2 = smax(b[2], 0.0f);
  const float s = smax(w0 + w1 + w2, 1e-5f);
  o[0] = w0 / s;
  o[1] = w1 / s;
  o[2] = w2 / s;
}

/* geometry_utils.h PointLineDistanceForward (squared distance) */
static inline float pt_line_dist(v2f p, v2f v0, v2f v1) {
  const v2f v1v0 = {v1.x - v0.x, v1.y - v0.y};
  const float l2 = dot2(v1v0, v1v0);
  if ((double)l2 <= K_EPS_D) {
    const v2f d = {p.x - v1.x, p.y - v1.y};
    return dot2(d, d);
  }
  const v2f pv0 = {p.x - v0.x, p.y - v0.y};
  const float t = dot2(v1v0, pv0) / l2;
  const float tt = smin(smax(t, 0.0f), 1.0f);
  const v2f proj = {v0.x + tt * v1v0.x, v0.y + tt * v1v0.y};
  const v2f d = {p.x - proj.x, p.y - proj.y};
  return dot2(d, d);
}

/* geometry_utils.h PointTriangleDistanceForward */
static inline float pt_tri_dist(v2f p, v2f v0, v2f v1, v2f v2) {
  const float e01 = pt_line_dist(p, v0, v1);
  const float e02 = pt_line_dist(p, v0, v2);
  const float e12 = pt_line_dist(p, v1, v2);
  return smin(smin(e01, e02), e12);
}

typedef struct {
  float z;
  int64_t f;
  float d, b0, b1, b2;
} frag_t;

static int frag_cmp(const frag_t* a, const frag_t* b) { /* std::tuple operator< on (z, f, ...) */
  if (a->z < b->z) return -1;
  if (b->z < a->z) return 1;
  if (a->f < b->f) return -1;
  if (b->f < a->f) return 1;
  return 0;
}

static void frag_sort(frag_t* q, int n) { /* insertion sort, n <= K+1 */
  for (int i = 1; i < n; ++i) {
    frag_t t = q[i];
    int j = i - 1;
    while (j >= 0 && frag_cmp(&q[j], &t) > 0) { q[j + 1] = q[j]; --j; }
    q[j + 1] = t;
  }
}

static inline int finite9(const float* fv) {
  for (int i = 0; i < 9; ++i)
    if (!isfinite(fv[i])) return 0;
  return 1;
}

/*
 * RasterizeMeshesNaiveCpu restated.
 * face_verts (F,3,3) f32 NDC xy + view z; mesh_first/mesh_count (N) i64.
 * neighbor (F) i64 or NULL: clipped_faces_neighbor_idx (-1 = none). When face f's neighbour
 * (the other half of its clipped quadrilateral) is already among the pixel's kept faces, f
 * replaces it iff f's unsigned distance is smaller than the neighbour's |signed distance|, and
 * is otherwise dropped; f is handled as a normal face when the neighbour is not kept.
 * Pixel window [y0, y1) x [x0, x1) (the whole image when y1 <= 0): outputs outside it keep the
 * background, so a large image can be checked on a crop.
 * Outputs (N,H,W,K): p2f i64, zbuf f32, dists f32; bary (N,H,W,K,3).
 * Background: -1 everywhere (as torch::full(..., -1)).
 */
/* Per-(pixel, face) evaluation of the naive loop body; returns 1 if kept (fills *o). */
static int eval_pixel_face(const float* fv, v2f p, float bbox_pad, float blur_radius, int perspective_correct,
                           int clip_barycentric_coords, int cull_backfaces, frag_t* o, float* dist_out) {
  if (!finite9(fv)) return 0;
  const float x0 = fv[0], y0 = fv[1], z0 = fv[2];
  const float x1 = fv[3], y1 = fv[4], z1 = fv[5];
  const float x2 = fv[6], y2 = fv[7], z2 = fv[8];
  const v2f v0 = {x0, y0}, v1 = {x1, y1}, v2 = {x2, y2};
  const float face_area = edge_fn(v0, v1, v2);
  if (cull_backfaces && face_area < 0.0f) return 0;
  if ((double)face_area <= K_EPS_D && (double)face_area >= -1.0f * K_EPS_D) return 0;
  const float xmin = smin(x0, smin(x1, x2)), xmax = smax(x0, smax(x1, x2));
  const float ymin = smin(y0, smin(y1, y2)), ymax = smax(y0, smax(y1, y2));
  const float zmax = smax(z0, smax(z1, z2));
  if (zmax < 0.0f) return 0;
  if (p.x > xmax + bbox_pad || p.x < xmin - bbox_pad || p.y > ymax + bbox_pad || p.y < ymin - bbox_pad) return 0;
  float b0[3], b[3], bc[3];
  bary_fwd(p, v0, v1, v2, b0);
  if (perspective_correct) persp_fwd(b0, z0, z1, z2, b);
  else memcpy(b, b0, sizeof(b));
  if (clip_barycentric_coords) clip_fwd(b, bc);
  else memcpy(bc, b, sizeof(bc));
  const float pz = bc[0] * z0 + bc[1] * z1 + bc[2] * z2;
  if (pz < 0.0f) return 0;
  const float dist = pt_tri_dist(p, v0, v1, v2);
  const int inside = b[0] > 0.0f && b[1] > 0.0f && b[2] > 0.0f;
  if (!inside && dist >= blur_radius) return 0;
  o->z = pz; o->d = inside ? -dist : dist;
  o->b0 = bc[0]; o->b1 = bc[1]; o->b2 = bc[2];
  *dist_out = dist;
  return 1;
}

/*
 * The MI355X kernels' resolution of a split face's two triangles (pair_mode = 1): evaluated
 * together at the pixel as ONE candidate (the second if both are kept and its distance is below
 * the first's |signed distance|, else whichever is kept), inserted like any face. Identical to
 * the CPU rule (pair_mode = 0) except when the first triangle was not among the K kept faces at
 * the moment the second is visited (it lost to K nearer faces earlier in packed order): there the
 * CPU keeps the second as a normal face. Documented deviation.
 */
void orc_raster_fwd_pairs(const float* face_verts, const int64_t* mesh_first, const int64_t* mesh_count,
                          const int64_t* neighbor, int N, int H, int W, int K, float blur_radius,
                          int perspective_correct, int clip_barycentric_coords, int cull_backfaces, int64_t* p2f,
                          float* zbuf, float* bary, float* dists) {
  const float bbox_pad = sqrtf(blur_radius);
#pragma omp parallel for collapse(2) schedule(dynamic, 1)
  for (int n = 0; n < N; ++n) {
    for (int yi = 0; yi < H; ++yi) {
      frag_t* q = (frag_t*)malloc(sizeof(frag_t) * (size_t)(K + 1));
      const int64_t f0 = mesh_first[n], f1 = mesh_first[n] + mesh_count[n];
      const float yf = pix_to_ndc(H - 1 - yi, H, W);
      for (int xi = 0; xi < W; ++xi) {
        const v2f p = {pix_to_ndc(W - 1 - xi, W, H), yf};
        int qn = 0;
        for (int64_t f = f0; f < f1; ++f) {
          const int64_t nb = neighbor ? neighbor[f] : -1;
          if (nb != -1 && nb < f) continue;  /* the second triangle: resolved with the first */
          frag_t c;
          float dist;
          int kept = eval_pixel_face(face_verts + f * 9, p, bbox_pad, blur_radius, perspective_correct,
                                     clip_barycentric_coords, cull_backfaces, &c, &dist);
          c.f = f;
          if (nb != -1) {
            frag_t c2;
            float dist2;
            const int k2 = eval_pixel_face(face_verts + nb * 9, p, bbox_pad, blur_radius, perspective_correct,
                                           clip_barycentric_coords, cull_backfaces, &c2, &dist2);
            c2.f = nb;
            if (k2 && (!kept || dist2 < fabsf(c.d))) c = c2;
            kept = kept || k2;
          }
          if (!kept) continue;
          q[qn++] = c;
          if (qn > K) { frag_sort(q, qn); --qn; }
        }
        frag_sort(q, qn);
        const int64_t pix = (((int64_t)n * H + yi) * W + xi) * K;
        for (int k = 0; k < K; ++k) {
          const int v = k < qn;
          p2f[pix + k] = v ? q[k].f : -1; zbuf[pix + k] = v ? q[k].z : -1.0f; dists[pix + k] = v ? q[k].d : -1.0f;
          bary[(pix + k) * 3 + 0] = v ? q[k].b0 : -1.0f; bary[(pix + k) * 3 + 1] = v ? q[k].b1 : -1.0f;
          bary[(pix + k) * 3 + 2] = v ? q[k].b2 : -1.0f;
        }
      }
      free(q);
    }
  }
}

void orc_raster_fwd_ex(const float* face_verts, const int64_t* mesh_first, const int64_t* mesh_count,
                       const int64_t* neighbor, int N, int H, int W, int K, float blur_radius,
                       int perspective_correct, int clip_barycentric_coords, int cull_backfaces, int wy0, int wy1,
                       int wx0, int wx1, int64_t* p2f, float* zbuf, float* bary, float* dists) {
  const float bbox_pad = sqrtf(blur_radius);
  if (wy1 <= 0) { wy0 = 0; wy1 = H; wx0 = 0; wx1 = W; }
#pragma omp parallel for collapse(2) schedule(dynamic, 1)
  for (int n = 0; n < N; ++n) {
    for (int yi = 0; yi < H; ++yi) {
      frag_t* q = (frag_t*)malloc(sizeof(frag_t) * (size_t)(K + 1));
      const int64_t f0 = mesh_first[n], f1 = mesh_first[n] + mesh_count[n];
      const float yf = pix_to_ndc(H - 1 - yi, H, W);
      for (int xi = 0; xi < W; ++xi) {
        const float xf = pix_to_ndc(W - 1 - xi, W, H);
        const v2f p = {xf, yf};
        int qn = 0;
        const int in_win = yi >= wy0 && yi < wy1 && xi >= wx0 && xi < wx1;
        for (int64_t f = f0; in_win && f < f1; ++f) {
          const float* fv = face_verts + f * 9;
          if (!finite9(fv)) continue;
          const float x0 = fv[0], y0 = fv[1], z0 = fv[2];
          const float x1 = fv[3], y1 = fv[4], z1 = fv[5];
          const float x2 = fv[6], y2 = fv[7], z2 = fv[8];
          const v2f v0 = {x0, y0}, v1 = {x1, y1}, v2 = {x2, y2};
          /* ComputeFaceAreas: E(v0, v1, v2) */
          const float face_area = edge_fn(v0, v1, v2);
          if (cull_backfaces && face_area < 0.0f) continue;
          if ((double)face_area <= K_EPS_D && (double)face_area >= -1.0f * K_EPS_D) continue;
          /* ComputeFaceBoundingBoxes + CheckPointOutsideBoundingBox */
          const float xmin = smin(x0, smin(x1, x2)), xmax = smax(x0, smax(x1, x2));
          const float ymin = smin(y0, smin(y1, y2)), ymax = smax(y0, smax(y1, y2));
          const float zmax = smax(z0, smax(z1, z2));
          if (zmax < 0.0f) continue;
          if (xf > xmax + bbox_pad || xf < xmin - bbox_pad || yf > ymax + bbox_pad ||
              yf < ymin - bbox_pad)
            continue;
          float b0[3], b[3], bc[3];
          bary_fwd(p, v0, v1, v2, b0);
          if (perspective_correct) persp_fwd(b0, z0, z1, z2, b);
          else memcpy(b, b0, sizeof(b));
          if (clip_barycentric_coords) clip_fwd(b, bc);
          else memcpy(bc, b, sizeof(bc));
          const float pz = bc[0] * z0 + bc[1] * z1 + bc[2] * z2;
          if (pz < 0.0f) continue;
          const float dist = pt_tri_dist(p, v0, v1, v2);
          const int inside = b[0] > 0.0f && b[1] > 0.0f && b[2] > 0.0f;
          const float sdist = inside ? -dist : dist;
          if (!inside && dist >= blur_radius) continue;
          const int64_t nb = neighbor ? neighbor[f] : -1;
          int at = -1;
          for (int i = 0; nb != -1 && i < qn; ++i)
            if (q[i].f == nb) { at = i; break; }
          if (at >= 0) {  /* the other half of a clipped quad is kept: keep the nearer-edged one */
            if (dist < fabsf(q[at].d)) {
              q[at].z = pz; q[at].f = f; q[at].d = sdist;
              q[at].b0 = bc[0]; q[at].b1 = bc[1]; q[at].b2 = bc[2];
            }
            continue;
          }
          q[qn].z = pz; q[qn].f = f; q[qn].d = sdist;
          q[qn].b0 = bc[0]; q[qn].b1 = bc[1]; q[qn].b2 = bc[2];
          ++qn;
          if (qn > K) { frag_sort(q, qn); --qn; }
        }
        frag_sort(q, qn);
        const int64_t pix = (((int64_t)n * H + yi) * W + xi) * K;
        for (int k = 0; k < K; ++k) {
          if (k < qn) {
            p2f[pix + k] = q[k].f; zbuf[pix + k] = q[k].z; dists[pix + k] = q[k].d;
            bary[(pix + k) * 3 + 0] = q[k].b0; bary[(pix + k) * 3 + 1] = q[k].b1;
            bary[(pix + k) * 3 + 2] = q[k].b2;
          } else {
            p2f[pix + k] = -1; zbuf[pix + k] = -1.0f; dists[pix + k] = -1.0f;
            bary[(pix + k) * 3 + 0] = -1.0f; bary[(pix + k) * 3 + 1] = -1.0f;
            bary[(pix + k) * 3 + 2] = -1.0f;
          }
        }
      }
      free(q);
    }
  }
}

void orc_raster_fwd(const float* face_verts, const int64_t* mesh_first, const int64_t* mesh_count,
                    int N, int H, int W, int K, float blur_radius, int perspective_correct,
                    int clip_barycentric_coords, int cull_backfaces, int64_t* p2f, float* zbuf,
                    float* bary, float* dists) {
  orc_raster_fwd_ex(face_verts, mesh_first, mesh_count, NULL, N, H, W, K, blur_radius, perspective_correct,
                    clip_barycentric_coords, cull_backfaces, 0, 0, 0, 0, p2f, zbuf, bary, dists);
}

/* ---------------- backward helpers (geometry_utils.h) ---------------- */

/* EdgeFunctionBackward: returns (dp, dv0, dv1) * grad */
static inline void edge_bwd(v2f p, v2f v0, v2f v1, float g, v2f* dp, v2f* dv0, v2f* dv1) {
  dp->x = (v1.y - v0.y) * g;  dp->y = (v0.x - v1.x) * g;
  dv0->x = (p.y - v1.y) * g;  dv0->y = (v1.x - p.x) * g;
  dv1->x = (v0.y - p.y) * g;  dv1->y = (p.x - v0.x) * g;
}

static inline v2f add2(v2f a, v2f b) { v2f r = {a.x + b.x, a.y + b.y}; return r; }

/* BarycentricCoordsBackward: grads of w = E/(area+eps) wrt v0, v1, v2 */
static void bary_bwd(v2f p, v2f v0, v2f v1, v2f v2, const float g[3], v2f* dv0, v2f* dv1, v2f* dv2) {
  const float area = (float)((double)edge_fn(v2, v0, v1) + K_EPS_D);
  const float area2 = area * area;
  const float area_inv = 1.0f / area;
  const float e0 = edge_fn(p, v1, v2), e1 = edge_fn(p, v2, v0), e2 = edge_fn(p, v0, v1);
  v2f a, b, c, d, e, f;
  /* w0 */
  const float dl_w0area = g[0] * (-e0 / area2), dl_e0 = g[0] * area_inv;
  edge_bwd(p, v1, v2, dl_e0, &a, &b, &c);           /* de0: (p, v1, v2) */
  edge_bwd(v2, v0, v1, dl_w0area, &d, &e, &f);      /* darea: (v2, v0, v1) */
  const v2f w0_v0 = e, w0_v1 = add2(b, f), w0_v2 = add2(c, d);
  /* w1 */
  const float dl_w1area = g[1] * (-e1 / area2), dl_e1 = g[1] * area_inv;
  edge_bwd(p, v2, v0, dl_e1, &a, &b, &c);           /* de1: (p, v2, v0) */
  edge_bwd(v2, v0, v1, dl_w1area, &d, &e, &f);
  const v2f w1_v0 = add2(c, e), w1_v1 = f, w1_v2 = add2(b, d);
  /* w2 */
  const float dl_w2area = g[2] * (-e2 / area2), dl_e2 = g[2] * area_inv;
  edge_bwd(p, v0, v1, dl_e2, &a, &b, &c);           /* de2: (p, v0, v1) */
  edge_bwd(v2, v0, v1, dl_w2area, &d, &e, &f);
  const v2f w2_v0 = add2(b, e), w2_v1 = add2(c, f), w2_v2 = d;
  *dv0 = add2(add2(w0_v0, w1_v0), w2_v0);
  *dv1 = add2(add2(w0_v1, w1_v1), w2_v1);
  *dv2 = add2(add2(w0_v2, w1_v2), w2_v2);
}

/* BarycentricPerspectiveCorrectionBackward */
static void persp_bwd(const float b[3], float z0, float z1, float z2, const float go[3], float gb[3],
                      float gz[3]) {
  const float w0_top = b[0] * z1 * z2;
  const float w1_top = b[1] * z0 * z2;
  const float w2_top = b[2] * z0 * z1;
  const float denom = smax(w0_top + w1_top + w2_top, (float)K_EPS_D);
  const float gdt = -w0_top * go[0] - w1_top * go[1] - w2_top * go[2];
  const float gd = gdt / (denom * denom);
  const float g0 = gd + go[0] / denom;
  const float g1 = gd + go[1] / denom;
  const float g2 = gd + go[2] / denom;
  gb[0] = g0 * z1 * z2;
  gb[1] = g1 * z0 * z2;
  gb[2] = g2 * z0 * z1;
  gz[0] = g1 * b[1] * z2 + g2 * b[2] * z1;
  gz[1] = g0 * b[0] * z2 + g2 * b[2] * z0;
  gz[2] = g0 * b[0] * z1 + g1 * b[1] * z0;
}

/* BarycentricClipBackward */
static void clip_bwd(const float b[3], const float go[3], float gb[3]) {
  const float w0 = smax(b[0], 0.0f), w1 = smax(b[1], 0.0f), w2 = smax(b[2], 0.0f);
  const float s = smax(w0 + w1 + w2, 1e-5f);
  const float num = w0 * go[0] + w1 * go[1] + w2 * go[2];
  const float gsum = -num / (s * s);
  const float m0 = b[0] > 0.0f ? 1.0f : 0.0f;
  const float m1 = b[1] > 0.0f ? 1.0f : 0.0f;
  const float m2 = b[2] > 0.0f ? 1.0f : 0.0f;
  gb[0] = (go[0] / s + gsum) * m0;
  gb[1] = (go[1] / s + gsum) * m1;
  gb[2] = (go[2] / s + gsum) * m2;
}

/* PointLineDistanceBackward: grads wrt v0, v1 */
static void pt_line_bwd(v2f p, v2f v0, v2f v1, float g, v2f* gv0, v2f* gv1) {
  const v2f v1v0 = {v1.x - v0.x, v1.y - v0.y};
  const v2f pv0 = {p.x - v0.x, p.y - v0.y};
  const float t_bot = dot2(v1v0, v1v0);
  const float t_top = dot2(v1v0, pv0);
  const float t = t_top / t_bot;
  const float tt = smin(smax(t, 0.0f), 1.0f);
  const v2f proj = {(1.0f - tt) * v0.x + tt * v1.x, (1.0f - tt) * v0.y + tt * v1.y};
  const v2f d = {proj.x - p.x, proj.y - p.y};
  const float s0 = g * (1.0f - tt) * 2.0f;
  const float s1 = g * tt * 2.0f;
  gv0->x = s0 * d.x; gv0->y = s0 * d.y;
  gv1->x = s1 * d.x; gv1->y = s1 * d.y;
}

/* PointTriangleDistanceBackward: closest edge only (ties: e01, e02, e12) */
static void pt_tri_bwd(v2f p, v2f v0, v2f v1, v2f v2, float g, v2f* g0, v2f* g1, v2f* g2) {
  const float e01 = pt_line_dist(p, v0, v1);
  const float e02 = pt_line_dist(p, v0, v2);
  const float e12 = pt_line_dist(p, v1, v2);
  g0->x = g0->y = g1->x = g1->y = g2->x = g2->y = 0.0f;
  if (e01 <= e02 && e01 <= e12) pt_line_bwd(p, v0, v1, g, g0, g1);
  else if (e02 <= e01 && e02 <= e12) pt_line_bwd(p, v0, v2, g, g0, g2);
  else if (e12 <= e01 && e12 <= e02) pt_line_bwd(p, v1, v2, g, g1, g2);
}

/* RasterizeMeshesBackwardCpu restated: serial accumulation in (n, y, x, k) order */
void orc_raster_bwd(const float* face_verts, const int64_t* p2f, const float* grad_zbuf,
                    const float* grad_bary, const float* grad_dists, int N, int H, int W, int K,
                    int perspective_correct, int clip_barycentric_coords, float* grad_fv /* zeroed (F,3,3) */) {
  for (int n = 0; n < N; ++n)
    for (int y = 0; y < H; ++y) {
      const float yf = pix_to_ndc(H - 1 - y, H, W);
      for (int x = 0; x < W; ++x) {
        const float xf = pix_to_ndc(W - 1 - x, W, H);
        const v2f p = {xf, yf};
        for (int k = 0; k < K; ++k) {
          const int64_t pix = (((int64_t)n * H + y) * W + x) * K + k;
          const int64_t f = p2f[pix];
          if (f < 0) continue;
          const float* fv = face_verts + f * 9;
          const float z0 = fv[2], z1 = fv[5], z2 = fv[8];
          const v2f v0 = {fv[0], fv[1]}, v1 = {fv[3], fv[4]}, v2 = {fv[6], fv[7]};
          const float gd_up = grad_dists[pix], gz_up = grad_zbuf[pix];
          const float gb_up[3] = {grad_bary[pix * 3], grad_bary[pix * 3 + 1], grad_bary[pix * 3 + 2]};
          float b0[3], b[3], bc[3];
          bary_fwd(p, v0, v1, v2, b0);
          if (perspective_correct) persp_fwd(b0, z0, z1, z2, b);
          else memcpy(b, b0, sizeof(b));
          if (clip_barycentric_coords) clip_fwd(b, bc);
          else memcpy(bc, b, sizeof(bc));
          const int inside = b[0] > 0.0f && b[1] > 0.0f && b[2] > 0.0f;
          const float sign = inside ? -1.0f : 1.0f;
          v2f dd0, dd1, dd2;
          pt_tri_bwd(p, v0, v1, v2, sign * gd_up, &dd0, &dd1, &dd2);
          float gsum[3] = {gb_up[0] + gz_up * z0, gb_up[1] + gz_up * z1, gb_up[2] + gz_up * z2};
          float g0[3] = {gsum[0], gsum[1], gsum[2]};
          float dz[3] = {0.0f, 0.0f, 0.0f};
          if (clip_barycentric_coords) { float t[3]; clip_bwd(b, g0, t); memcpy(g0, t, sizeof(t)); }
          if (perspective_correct) { float t[3]; persp_bwd(b0, z0, z1, z2, g0, t, dz); memcpy(g0, t, sizeof(t)); }
          v2f db0, db1, db2;
          bary_bwd(p, v0, v1, v2, g0, &db0, &db1, &db2);
          float* gf = grad_fv + f * 9;
          gf[0] += db0.x + dd0.x; gf[1] += db0.y + dd0.y; gf[2] += gz_up * bc[0] + dz[0];
          gf[3] += db1.x + dd1.x; gf[4] += db1.y + dd1.y; gf[5] += gz_up * bc[1] + dz[1];
          gf[6] += db2.x + dd2.x; gf[7] += db2.y + dd2.y; gf[8] += gz_up * bc[2] + dz[2];
        }
      }
    }
}

/*
 * Projection used by the MI355X path (DESIGN.md "Projection"), restated with
 * the identical operand order so face_verts are bit-identical:
 *   v   = ((X*R00 + Y*R10) + Z*R20) + T0      (row-vector convention X @ R + T)
 *   ndc = (ax * (vx / vz) + bx, ay * (vy / vz) + by, vz)
 * views: N records of 16 floats {R[9] row-major, T[3], ax, bx, ay, by}.
 * shared=1: every view renders the same (V,3)/(F,3) mesh, output (N*F,3,3).
 */
void orc_project_faces(const float* verts, const int32_t* faces, int64_t F, const float* views, int N,
                       float* face_verts) {
  for (int n = 0; n < N; ++n) {
    const float* vw = views + 16 * n;
    for (int64_t f = 0; f < F; ++f) {
      for (int c = 0; c < 3; ++c) {
        const float* X = verts + 3 * (int64_t)faces[3 * f + c];
        const float vx = ((X[0] * vw[0] + X[1] * vw[3]) + X[2] * vw[6]) + vw[9];
        const float vy = ((X[0] * vw[1] + X[1] * vw[4]) + X[2] * vw[7]) + vw[10];
        const float vz = ((X[0] * vw[2] + X[1] * vw[5]) + X[2] * vw[8]) + vw[11];
        float* o = face_verts + (((int64_t)n * F + f) * 3 + c) * 3;
        o[0] = vw[12] * (vx / vz) + vw[13];
        o[1] = vw[14] * (vy / vz) + vw[15];
        o[2] = vz;
      }
    }
  }
}

int orc_version(void) { return 1; }

/* OpenMP threads of the restated CPU rasterizer (bench.py's 1-core CPU baseline). */
#ifdef _OPENMP
#include <omp.h>
#endif
void orc_set_threads(int n) {
#ifdef _OPENMP
  omp_set_num_threads(n > 0 ? n : 1);
#else
  (void)n;
#endif
}
