// mi355r — MI355X (gfx950) differentiable mesh rasterizer: shared device math.
//
// Every function here restates PyTorch3D's rasterization math (the path the
// reference reaches via torch_renderer.py:97-121 / renderer.py:87-101 ->
// pytorch3d.renderer.mesh.rasterize_meshes -> pytorch3d._C.rasterize_meshes)
// with the SAME operand order as the CPU implementation, so that integer
// outputs (pix_to_face) are bit-identical to the CPU path. The library is built
// with -ffp-contract=off (no FMA contraction) and HIP's default correctly
// rounded f32 division; see DESIGN.md "Bit-exactness".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MR_KEPS_D 1e-8  // geometry_utils.h: `const auto kEpsilon = 1e-8;` (a double)
#define MR_DEV __device__ __forceinline__
// FMA contraction allowed inside shading / gradient arithmetic (tolerance-compared, never a raster
// decision): the library builds with -ffp-contract=off so that every raster expression keeps the
// CPU oracle's rounding, and these blocks opt back in.
#define MR_FP_FAST _Pragma("clang fp contract(fast)")

// Fast math for the shading and gradient arithmetic (never for raster decisions, pix_to_face,
// zbuf, bary or dists, which stay IEEE and bit-exact with the CPU): 1-ulp hardware reciprocal,
// square root, exp2 and log2 instead of the multi-instruction correctly rounded sequences. The
// shaded images and gradients are compared with the oracle within 1e-4, which these errors
// (a few ulp) do not approach.
MR_DEV float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
MR_DEV float fdiv(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
MR_DEV float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
MR_DEV float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
// a^b for a >= 0 (a = 0 -> 0 for b > 0, the only use: Phong's specular power)
MR_DEV float fpow(float a, float b) { return a > 0.0f ? __builtin_amdgcn_exp2f(b * __builtin_amdgcn_logf(a)) : (b == 0.0f ? 1.0f : 0.0f); }

// Fixed-point gradient accumulation (the fused backward's per-face totals): a value is stored as the
// two's-complement integer round(x * 2^MR_FIX_SHIFT) and summed with 64-bit integer atomics. Integer
// addition is associative, so a total is the same bits whatever order the addends arrive in
// (deterministic without a fixed-order reduction pass); wrap-around in intermediate sums cancels, so
// only the final total must lie within +-2^(63 - MR_FIX_SHIFT) = +-2^31. Resolution 2^-32 = 2.3e-10
// absolute, far below the 1e-4 bar; an addend of magnitude >= MR_FIX_MAX takes a float atomic into the
// face's float remainder row instead. The cutoff is 2^24 so that a face's fixed-point part can reach
// 2^31 only through >= 128 same-sign addends each near the cutoff (one addend is one (view, tile) run of
// the face's pixels); the largest run totals of the parity workloads are ~1e6 on sliver faces, and a
// loss scaled up until runs reach 2^24 is accumulated in float (correct, no longer bitwise
// deterministic) — tests/test_gpu_round6.py::test_large_run_totals_take_the_float_rows.
#define MR_FIX_SHIFT 32
#define MR_FIX_MAX 16777216.0f  // 2^24
MR_DEV long long fix_of(float x) { return __float2ll_rn(x * 4294967296.0f); }
MR_DEV float fix_to_f(unsigned long long v) { return (float)((double)(long long)v * (1.0 / 4294967296.0)); }
// Columns of a face's gradient-total row: ACC = 18 holds the three corners' position then normal columns
// (3 c + k, 9 + 3 c + k); ACC = 27 (vertex colours) keeps each corner's position and colour columns adjacent
// (6 c + k, 6 c + 3 + k; normals 18 + 3 c + k), so that a vertex gathers one 48-B piece of each incident face's
// row instead of two 24-B pieces 144 B apart (the C5 gathers are HBM-bound: r6n_pmc_c5.json).
template <int ACC> MR_DEV constexpr int col_pos(int c, int k) { return ACC == 27 ? 6 * c + k : 3 * c + k; }
template <int ACC> MR_DEV constexpr int col_rgb(int c, int k) { return 6 * c + 3 + k; }
template <int ACC> MR_DEV constexpr int col_nrm(int c, int k) { return ACC == 27 ? 18 + 3 * c + k : 9 + 3 * c + k; }
// Per-face total component i: the fixed-point sum plus the float-atomic remainder.
// (rem false: the float remainder rows are all zero and not read — fix_to_f never returns -0, so the
// sum with a zero remainder is the same bits)
MR_DEV float fix_total(const unsigned long long* __restrict__ gfix, const float* __restrict__ gflt, int64_t i,
                       bool rem = true) {
  return gfix ? (rem ? fix_to_f(gfix[i]) + gflt[i] : fix_to_f(gfix[i])) : gflt[i];
}
// NC consecutive totals (components i .. i + NC - 1, NC even or 3), the fixed-point words read 16 B at a time: the
// vertex gathers' lanes each read a different face row, so every load instruction is ~64 cache-line requests and
// the C5 gathers were bound by those requests, not by bytes (r6n_pmc_c5.json: 49 MB over ~16 us). Bitwise
// fix_total's values. (Rows are 8-B aligned: 16-B loads at 8-B alignment, which gfx950's global loads take.)
typedef unsigned long long mr_u64x2 __attribute__((ext_vector_type(2), aligned(8)));
template <int NC>
MR_DEV void fix_totals(const unsigned long long* __restrict__ gfix, const float* __restrict__ gflt, int64_t i, bool rem,
                       float (&out)[NC]) {
  if (!gfix) {
#pragma unroll
    for (int k = 0; k < NC; ++k) out[k] = gflt[i + k];
    return;
  }
  unsigned long long w[NC];
#pragma unroll
  for (int k = 0; k + 1 < NC; k += 2) {
    const mr_u64x2 q = *(const mr_u64x2*)(gfix + i + k);
    w[k] = q.x;
    w[k + 1] = q.y;
  }
  if (NC & 1) w[NC - 1] = gfix[i + NC - 1];
#pragma unroll
  for (int k = 0; k < NC; ++k) out[k] = rem ? fix_to_f(w[k]) + gflt[i + k] : fix_to_f(w[k]);
}

// std::max/std::min semantics (a < b ? b : a) — NaN handling follows the CPU code.
MR_DEV float smax(float a, float b) { return (a < b) ? b : a; }
MR_DEV float smin(float a, float b) { return (b < a) ? b : a; }

// rasterization_utils.h PixToNonSquareNdc
MR_DEV float pix_to_ndc(int i, int S1, int S2) {
  float range = 2.0f;
  if (S1 > S2) range = ((float)S1 * range) / (float)S2;
  const float offset = range / 2.0f;
  return -offset + (range * (float)i + offset) / (float)S1;
}
// NDC of output column xi / row yi (both flipped: +X left, +Y up).
MR_DEV float col_ndc(int xi, int H, int W) { return pix_to_ndc(W - 1 - xi, W, H); }
MR_DEV float row_ndc(int yi, int H, int W) { return pix_to_ndc(H - 1 - yi, H, W); }

// geometry_utils.h EdgeFunctionForward: E(p, a, b)
MR_DEV float edge_fn(float px, float py, float ax, float ay, float bx, float by) {
  return (px - ax) * (by - ay) - (py - ay) * (bx - ax);
}

// Face record written by the setup kernel (one per rasterized face instance,
// index = PyTorch3D packed face id). 64 B, 16-B aligned -> 4 x dwordx4 loads.
struct __attribute__((aligned(16))) FaceRec {
  float x0, y0, z0, x1, y1, z1, x2, y2, z2;  // NDC xy, view z
  float area;                                // float(double(E(v2,v0,v1)) + 1e-8)
  float xmin, xmax, ymin, ymax;              // NDC bbox (not padded)
  uint32_t flags;                            // FR_VALID | FR_FAST
  uint32_t face;                             // mesh face index (into faces array)
};
enum : uint32_t { FR_VALID = 1u, FR_FAST = 2u, FR_CLIP = 4u, FR_PAIR = 8u };
// Record load as four 16-B vector loads straight into registers (an aggregate copy through a
// computed index may be lowered to a memcpy through scratch).
MR_DEV FaceRec load_rec(const FaceRec* __restrict__ recs, int64_t id) {
  const float4* q = (const float4*)(recs + id);
  const float4 a = q[0], b = q[1], c = q[2], d = q[3];
  FaceRec r;
  r.x0 = a.x; r.y0 = a.y; r.z0 = a.z; r.x1 = a.w;
  r.y1 = b.x; r.z1 = b.y; r.x2 = b.z; r.y2 = b.w;
  r.z2 = c.x; r.area = c.y; r.xmin = c.z; r.xmax = c.w;
  r.ymin = d.x; r.ymax = d.y; r.flags = __float_as_uint(d.z); r.face = __float_as_uint(d.w);
  return r;
}
// FR_CLIP: the record is a sub-triangle of a face clipped at the near plane (its ClipRec holds
// the barycentric conversion to the original face). FR_PAIR: one of the two triangles a face
// with one corner behind the plane is split into; record id rid (< NF) is the first, NF + rid the
// second (NF = number of face instances), each the other's clipped_faces_neighbor_idx.

// BarycentricPerspectiveCorrectionForward
MR_DEV void persp_fwd(float w0, float w1, float w2, float z0, float z1, float z2, float& o0, float& o1,
                      float& o2) {
  const float t0 = w0 * z1 * z2;
  const float t1 = w1 * z0 * z2;
  const float t2 = w2 * z0 * z1;
  const float d = smax(t0 + t1 + t2, (float)MR_KEPS_D);
  o0 = t0 / d;
  o1 = t1 / d;
  o2 = t2 / d;
}

// BarycentricClipForward (lower clamp + renormalise)
MR_DEV void clip_fwd(float b0, float b1, float b2, float& o0, float& o1, float& o2) {
  const float w0 = smax(b0, 0.0f), w1 = smax(b1, 0.0f), w2 = smax(b2, 0.0f);
  const float s = smax(w0 + w1 + w2, 1e-5f);
  o0 = w0 / s;
  o1 = w1 / s;
  o2 = w2 / s;
}

// PointLineDistanceForward (squared)
MR_DEV float pt_line_dist(float px, float py, float ax, float ay, float bx, float by) {
  const float dx = bx - ax, dy = by - ay;
  const float l2 = dx * dx + dy * dy;
  if ((double)l2 <= MR_KEPS_D) {
    const float ex = px - bx, ey = py - by;
    return ex * ex + ey * ey;
  }
  const float t = (dx * (px - ax) + dy * (py - ay)) / l2;
  const float tt = smin(smax(t, 0.0f), 1.0f);
  const float qx = ax + tt * dx, qy = ay + tt * dy;
  const float ex = px - qx, ey = py - qy;
  return ex * ex + ey * ey;
}

MR_DEV float pt_tri_dist(float px, float py, const FaceRec& r) {
  const float e01 = pt_line_dist(px, py, r.x0, r.y0, r.x1, r.y1);
  const float e02 = pt_line_dist(px, py, r.x0, r.y0, r.x2, r.y2);
  const float e12 = pt_line_dist(px, py, r.x1, r.y1, r.x2, r.y2);
  return smin(smin(e01, e02), e12);
}

// Full per-(pixel, face) evaluation, exactly the CPU naive loop body after the
// face-level skips. Returns true if the face is kept for this pixel.
struct FragEval {
  float pz, sdist, b0, b1, b2;  // bary after perspective correction + clip
  float w0, w1, w2;             // uncorrected barycentrics
  float c0, c1, c2;             // perspective corrected (pre-clip)
  bool inside;
};

MR_DEV bool eval_face(const FaceRec& r, float px, float py, float bbox_pad, float blur, bool persp,
                      bool clipb, FragEval& o) {
  if (px > r.xmax + bbox_pad || px < r.xmin - bbox_pad || py > r.ymax + bbox_pad || py < r.ymin - bbox_pad)
    return false;
  const float e0 = edge_fn(px, py, r.x1, r.y1, r.x2, r.y2);
  const float e1 = edge_fn(px, py, r.x2, r.y2, r.x0, r.y0);
  const float e2 = edge_fn(px, py, r.x0, r.y0, r.x1, r.y1);
  o.w0 = e0 / r.area;
  o.w1 = e1 / r.area;
  o.w2 = e2 / r.area;
  if (persp) persp_fwd(o.w0, o.w1, o.w2, r.z0, r.z1, r.z2, o.c0, o.c1, o.c2);
  else { o.c0 = o.w0; o.c1 = o.w1; o.c2 = o.w2; }
  if (clipb) clip_fwd(o.c0, o.c1, o.c2, o.b0, o.b1, o.b2);
  else { o.b0 = o.c0; o.b1 = o.c1; o.b2 = o.c2; }
  o.pz = o.b0 * r.z0 + o.b1 * r.z1 + o.b2 * r.z2;
  if (o.pz < 0.0f) return false;
  o.inside = o.c0 > 0.0f && o.c1 > 0.0f && o.c2 > 0.0f;
  if (!o.inside && !(blur > 0.0f)) return false;  // dist >= 0 == blur (finite faces only)
  const float dist = pt_tri_dist(px, py, r);
  o.sdist = o.inside ? -dist : dist;
  if (!o.inside && dist >= blur) return false;
  return true;
}

// Cheap exact pre-test (blur == 0): the face can only be kept if the pixel is
// strictly inside in edge-function sign. Valid when FR_FAST is set (finite,
// non-zero area; for perspective correction additionally all z > 0).
MR_DEV bool fast_reject(const FaceRec& r, float px, float py) {
  const float e0 = edge_fn(px, py, r.x1, r.y1, r.x2, r.y2);
  const float e1 = edge_fn(px, py, r.x2, r.y2, r.x0, r.y0);
  const float e2 = edge_fn(px, py, r.x0, r.y0, r.x1, r.y1);
  const bool pos = r.area > 0.0f;
  const bool in = pos ? (e0 > 0.0f && e1 > 0.0f && e2 > 0.0f) : (e0 < 0.0f && e1 < 0.0f && e2 < 0.0f);
  return !in;
}

MR_DEV bool rec_finite(const FaceRec& r) {
  return __builtin_isfinite(r.x0) && __builtin_isfinite(r.y0) && __builtin_isfinite(r.z0) &&
         __builtin_isfinite(r.x1) && __builtin_isfinite(r.y1) && __builtin_isfinite(r.z1) &&
         __builtin_isfinite(r.x2) && __builtin_isfinite(r.y2) && __builtin_isfinite(r.z2);
}

// Lexicographic (z, face) order == std::sort over (pz, f, ...) tuples.
MR_DEV bool frag_less(float za, int64_t fa, float zb, int64_t fb) {
  return za < zb || (!(zb < za) && fa < fb);
}

// ---------------------------------------------------------------------------
// Near-plane clipping (upstream mesh/clip.py clip_faces, restated in oracle.py clip_faces_ref
// with the same operation order): corners (x_ndc, y_ndc, z_view); c = z_clip_value.
//   nb = #corners with z < c: 0 unchanged, 3 culled;
//   nb = 2 (front corner i): one triangle, slot i = p_i, slot j = p_ij, slot k = p_ik;
//   nb = 1 (behind corner i): t1 = (p_ij, p_j, p_k), t2 = (p_ik, p_ij, p_k) in slots (i, j, k);
// j = i+1, k = i+2 (mod 3); p_ab = the point of edge a->b at z = c, w_ab = (c - z_a) / (z_b - z_a):
// perspective: xy = (xy_a z_a + w (xy_b z_b - xy_a z_a)) / c, else xy_a + w (xy_b - xy_a); z = c.
// ---------------------------------------------------------------------------
struct __attribute__((aligned(16))) ClipRec {
  float conv[9];  // row s = original-face barycentrics of the sub-triangle's slot-s vertex
  float wj, wk;   // interpolation weights of p_ij, p_ik
  uint32_t info;  // nb (bits 0-1) | corner i << 2 | second triangle of a pair << 4
};

MR_DEV void clip_point(const float a[3], const float b[3], float w, float c, bool persp, float q[3]) {
  if (persp) {
    const float axw = a[0] * a[2], ayw = a[1] * a[2];
    const float bxw = b[0] * b[2], byw = b[1] * b[2];
    q[0] = (axw + w * (bxw - axw)) / c;
    q[1] = (ayw + w * (byw - ayw)) / c;
  } else {
    q[0] = a[0] + w * (b[0] - a[0]);
    q[1] = a[1] + w * (b[1] - a[1]);
  }
  q[2] = c;
}

// Number of corners behind the plane and the odd corner i (the front one for nb = 2, the behind
// one for nb = 1; argmax order as the oracle: the first such corner).
MR_DEV int clip_class(const float v[3][3], float c, int& i) {
  const bool b0 = v[0][2] < c, b1 = v[1][2] < c, b2 = v[2][2] < c;
  const int nb = (int)b0 + (int)b1 + (int)b2;
  if (nb == 2) i = !b0 ? 0 : !b1 ? 1 : 2;
  else i = b0 ? 0 : b1 ? 1 : 2;
  return nb;
}

// Sub-triangle `sub` (0 or 1) of a clipped face: corners out[3][3] and its ClipRec.
MR_DEV void clip_sub(const float v[3][3], int nb, int i, int sub, float c, bool persp, float out[3][3],
                     ClipRec& cr) {
  const int j = i == 2 ? 0 : i + 1, k = j == 2 ? 0 : j + 1;
  const float wj = (c - v[i][2]) / (v[j][2] - v[i][2]);
  const float wk = (c - v[i][2]) / (v[k][2] - v[i][2]);
  float pij[3], pik[3];
  clip_point(v[i], v[j], wj, c, persp, pij);
  clip_point(v[i], v[k], wk, c, persp, pik);
  for (int q = 0; q < 9; ++q) cr.conv[q] = 0.0f;
  cr.wj = wj;
  cr.wk = wk;
  cr.info = (uint32_t)nb | ((uint32_t)i << 2) | ((uint32_t)sub << 4);
  const float* s_i;
  const float* s_j;
  const float* s_k;
  if (nb == 2) {  // (p_i, p_ij, p_ik)
    s_i = v[i]; s_j = pij; s_k = pik;
    cr.conv[3 * i + i] = 1.0f;
    cr.conv[3 * j + i] = 1.0f - wj; cr.conv[3 * j + j] = wj;
    cr.conv[3 * k + i] = 1.0f - wk; cr.conv[3 * k + k] = wk;
  } else if (sub == 0) {  // t1 = (p_ij, p_j, p_k)
    s_i = pij; s_j = v[j]; s_k = v[k];
    cr.conv[3 * i + i] = 1.0f - wj; cr.conv[3 * i + j] = wj;
    cr.conv[3 * j + j] = 1.0f;
    cr.conv[3 * k + k] = 1.0f;
  } else {  // t2 = (p_ik, p_ij, p_k)
    s_i = pik; s_j = pij; s_k = v[k];
    cr.conv[3 * i + i] = 1.0f - wk; cr.conv[3 * i + k] = wk;
    cr.conv[3 * j + i] = 1.0f - wj; cr.conv[3 * j + j] = wj;
    cr.conv[3 * k + k] = 1.0f;
  }
  for (int q = 0; q < 3; ++q) {
    out[i][q] = s_i[q];
    out[j][q] = s_j[q];
    out[k][q] = s_k[q];
  }
}

// Original-face barycentrics of a sub-triangle fragment: sum_s b_sub[s] * conv[s] ((s0 + s1) + s2).
MR_DEV void clip_unconvert(const ClipRec& cr, float b0, float b1, float b2, float& o0, float& o1, float& o2) {
  o0 = (b0 * cr.conv[0] + b1 * cr.conv[3]) + b2 * cr.conv[6];
  o1 = (b0 * cr.conv[1] + b1 * cr.conv[4]) + b2 * cr.conv[7];
  o2 = (b0 * cr.conv[2] + b1 * cr.conv[5]) + b2 * cr.conv[8];
}

// Chain rule of the clip for one fragment of a sub-triangle.
//  v: the original corners; gb_orig: gradient w.r.t. the original barycentrics; b_sub: the
//  sub-triangle's barycentrics (rasterizer output); gfv_sub: gradient w.r.t. the sub-triangle's
//  corners as returned by raster_bwd_pixel (given gb_sub from clip_gb_sub). Accumulates the
//  gradient w.r.t. the original corners into gfv (the sub-vertex z = c is a constant).
MR_DEV void clip_gb_sub(const ClipRec& cr, const float g[3], float gs[3]) {
  for (int s = 0; s < 3; ++s) gs[s] = (cr.conv[3 * s] * g[0] + cr.conv[3 * s + 1] * g[1]) + cr.conv[3 * s + 2] * g[2];
}

MR_DEV void clip_point_bwd(const float a[3], const float b[3], float w, float c, bool persp, const float gq[3],
                           float ga[3], float gbv[3], float& gw) {
  if (persp) {
    const float rc = 1.0f / c;
    ga[0] += gq[0] * a[2] * (1.0f - w) * rc;
    ga[1] += gq[1] * a[2] * (1.0f - w) * rc;
    ga[2] += (gq[0] * a[0] + gq[1] * a[1]) * (1.0f - w) * rc;
    gbv[0] += gq[0] * w * b[2] * rc;
    gbv[1] += gq[1] * w * b[2] * rc;
    gbv[2] += (gq[0] * b[0] + gq[1] * b[1]) * w * rc;
    gw += (gq[0] * (b[0] * b[2] - a[0] * a[2]) + gq[1] * (b[1] * b[2] - a[1] * a[2])) * rc;
  } else {
    ga[0] += gq[0] * (1.0f - w);
    ga[1] += gq[1] * (1.0f - w);
    gbv[0] += gq[0] * w;
    gbv[1] += gq[1] * w;
    gw += gq[0] * (b[0] - a[0]) + gq[1] * (b[1] - a[1]);
  }
}

MR_DEV void clip_bwd_chain(const ClipRec& cr, const float v[3][3], float c, bool persp, const float b_sub[3],
                           const float g_orig[3], const float gfv_sub[3][3], float gfv[3][3]) {
  const int nb = (int)(cr.info & 3u), i = (int)((cr.info >> 2) & 3u), sub = (int)((cr.info >> 4) & 1u);
  const int j = i == 2 ? 0 : i + 1, k = j == 2 ? 0 : j + 1;
  float gwj = 0.0f, gwk = 0.0f;
  // conversion entries (1 - w, w): dL/dconv[s][o] = b_sub[s] * g_orig[o]
  if (nb == 2) {
    gwj += b_sub[j] * (g_orig[j] - g_orig[i]);
    gwk += b_sub[k] * (g_orig[k] - g_orig[i]);
    for (int q = 0; q < 3; ++q) gfv[i][q] += gfv_sub[i][q];
    clip_point_bwd(v[i], v[j], cr.wj, c, persp, gfv_sub[j], gfv[i], gfv[j], gwj);
    clip_point_bwd(v[i], v[k], cr.wk, c, persp, gfv_sub[k], gfv[i], gfv[k], gwk);
  } else if (sub == 0) {
    gwj += b_sub[i] * (g_orig[j] - g_orig[i]);
    clip_point_bwd(v[i], v[j], cr.wj, c, persp, gfv_sub[i], gfv[i], gfv[j], gwj);
    for (int q = 0; q < 3; ++q) {
      gfv[j][q] += gfv_sub[j][q];
      gfv[k][q] += gfv_sub[k][q];
    }
  } else {
    gwk += b_sub[i] * (g_orig[k] - g_orig[i]);
    gwj += b_sub[j] * (g_orig[j] - g_orig[i]);
    clip_point_bwd(v[i], v[k], cr.wk, c, persp, gfv_sub[i], gfv[i], gfv[k], gwk);
    clip_point_bwd(v[i], v[j], cr.wj, c, persp, gfv_sub[j], gfv[i], gfv[j], gwj);
    for (int q = 0; q < 3; ++q) gfv[k][q] += gfv_sub[k][q];
  }
  // w_ab = (c - z_a) / (z_b - z_a)
  const float dj = v[j][2] - v[i][2], dk = v[k][2] - v[i][2];
  gfv[i][2] += gwj * ((c - v[j][2]) / (dj * dj)) + gwk * ((c - v[k][2]) / (dk * dk));
  gfv[j][2] += gwj * (-cr.wj / dj);
  gfv[k][2] += gwk * (-cr.wk / dk);
}
