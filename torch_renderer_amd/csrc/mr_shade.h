// mi355r — per-pixel shading (forward + analytic backward) and the rasterizer's
// per-pixel backward, as device functions fused into the render kernels.
//
// Restates (K = faces_per_pixel = 1):
//  * SoftPhongShader -> phong_shading / _apply_lighting / PointLights.diffuse,
//    .specular / Materials (upstream pytorch3d/renderer/mesh/shading.py,
//    lighting.py), used at torch_renderer.py:141-153 and renderer.py:88-98;
//  * TexturesUV.sample_textures (grid_sample bilinear, align_corners=True,
//    padding 'border', map flipped vertically) / TexturesVertex;
//  * softmax_rgb_blend (ColorRender, torch_renderer.py:155-159) and
//    sigmoid_alpha_blend (DepthRender silhouette, torch_renderer.py:102-121);
//  * RasterizeMeshesBackwardCpu per (pixel, k) (geometry_utils.h backward fns);
//  * the projection X_view = X @ R + T, ndc = (ax*x/z+bx, ay*y/z+by, z) and its
//    derivative w.r.t. X, R and T (MeshRasterizer.transform).
#pragma once
#include "mr_common.h"

struct ShadeParams {
  // geometry
  const float* verts;     // (V,3) world
  const int32_t* faces;   // (F,3)
  const float* vnormals;  // (V,3) normalized vertex normals
  // texture
  int tex_kind;             // 0 = white, 1 = per-vertex colours, 2 = UV map
  const float* vcolors;     // (V,3)
  const float* verts_uvs;   // (Vt,2)
  const int32_t* faces_uvs; // (F,3)
  const float4* tex;        // (Ht,Wt) RGBA-padded, row 0 = first image row (unflipped)
  const uchar4* tex8;       // optional 8-bit copy (value = tex_lut[u8]); read instead of tex
  const float* tex_lut;
  int tex_h, tex_w;
  // lighting / materials
  int light_kind;  // 0 = point light, 1 = ambient only
  float light_loc[3], light_amb[3], light_diff[3], light_spec[3];
  float mat_amb[3], mat_diff[3], mat_spec[3], shininess;
  const float* cam_centers;  // (Nc,3) world-space camera centre used for specular
  int cam_center_stride;     // 0 (single camera) or 3
  // blending
  float sigma_rgb, gamma, bg[3], znear, zfar;
  float sigma_sil;
  // reciprocals precomputed on the host (multiplications in the per-pixel code)
  float inv_sigma_rgb, inv_gamma, inv_zrange, inv_sigma_sil;
  int zbuf_mode;  // MR_OUT_ZBUF: the depth output is zbuf[..., 0] (background -1), not relu(zbuf)
};

struct ViewRec {  // 16 floats, matches mr_view_t
  float R[9], T[3], ax, bx, ay, by;
};

struct ShadeOut {
  float depth, sil, rgb[3], alpha;
};

// ---- F.normalize(x, eps=1e-6) forward/backward ----
MR_DEV void normalize3(const float x[3], float y[3], float& nrm, float& den) {
  MR_FP_FAST
  nrm = fsqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
  den = smax(nrm, 1e-6f);
  const float r = frcp(den);
  y[0] = x[0] * r;
  y[1] = x[1] * r;
  y[2] = x[2] * r;
}
MR_DEV void normalize3_bwd(const float x[3], float nrm, float den, const float g[3], float gx[3]) {
  MR_FP_FAST
  const float r = frcp(den);
  const float gd = -((g[0] * x[0] + g[1] * x[1]) + g[2] * x[2]) * (r * r);
  const float gn = (nrm >= 1e-6f && nrm > 0.0f) ? gd * frcp(nrm) : 0.0f;
  gx[0] = g[0] * r + gn * x[0];
  gx[1] = g[1] * r + gn * x[1];
  gx[2] = g[2] * r + gn * x[2];
}
MR_DEV float dot3(const float a[3], const float b[3]) {
  MR_FP_FAST
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
MR_DEV float sigmoidf_(float x) { return frcp(1.0f + fexp(-x)); }
// sigmoid_alpha_blend's per-fragment probability sigmoid(-d / sigma)
MR_DEV float frag_prob(float d, float inv_sigma) { return sigmoidf_((-d) * inv_sigma); }
// sigmoid(x) and 1 - sigmoid(x), each to a few ulp of ITS OWN value. 1 - p is not formed as a
// difference: near saturation (p -> 1, i.e. a pixel a few sigma inside a face) that cancels every
// significant bit, and the blends' derivative p (1 - p) / sigma (x 1e4) carries the loss straight into
// the vertex gradients (torch's sigmoid backward has the same cancellation; the oracle's float64
// shadow does not, and tests.helpers.report measures against both).
MR_DEV void sigmoid2(float x, float& p, float& q) {
  const float t = fexp(-fabsf(x));  // (0, 1]
  const float r = frcp(1.0f + t);
  const float big = r, small = t * r;  // 1 / (1 + t), t / (1 + t)
  p = x >= 0.0f ? big : small;
  q = x >= 0.0f ? small : big;
}

// ---- texture: grid_sample(bilinear, align_corners=True, border) on flipped map ----
struct TexTap {
  float ix, iy;     // clipped pixel coords in the flipped map
  bool gx_ok, gy_ok;  // border-clip gradient pass-through
  int x0, y0;
  // 8-bit maps: the four texels as loaded (pre: valid), so that the backward's second look-up
  // (tex_sample_bwd) reads no memory
  bool pre;
  uint32_t raw[4];
};
// The four bilinear taps (x0|x0+1, y0|y0+1); out-of-range taps read as zero. The addresses are
// clamped and all four loads issued unconditionally, then the values selected: written as
// guarded loads, the compiler sinks each into its own branch with a load + wait per tap. The
// empty asm consumes the loaded values unconditionally, so the loads cannot be sunk.
// The 256-entry u8 -> float texture table staged in LDS by kernels that call stage_tex_lut (a
// namespace-scope LDS array, so its reads are ds_read by construction).
__shared__ float g_tex_lut[256];

// lds_lut: read the table from g_tex_lut (the kernel staged it) instead of S.tex_lut. Texel indices
// are 32-bit (maps < 2^32 texels): one 64-bit address add per tap instead of 64-bit index math.
// The four 8-bit texels of cell (x0, y0) as raw words (unconditional loads of clamped indices).
MR_DEV void tex_taps_raw(const ShadeParams& S, int x0, int y0, uint32_t (&raw)[4]) {
  const int xs[2] = {x0, x0 + 1}, ys[2] = {y0, y0 + 1};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int xc = xs[i & 1], yc = ys[i >> 1];
    const bool ok = (unsigned)xc < (unsigned)S.tex_w && (unsigned)yc < (unsigned)S.tex_h;
    const int x = ok ? xc : 0, y = ok ? yc : S.tex_h - 1;
    raw[i] = ((const uint32_t*)S.tex8)[(uint32_t)(S.tex_h - 1 - y) * (uint32_t)S.tex_w + (uint32_t)x];
  }
}
// tex_taps' values from raw texels (tex_taps_raw): the table look-ups and the out-of-range zeros.
MR_DEV void taps_from_raw(const ShadeParams& S, int x0, int y0, const uint32_t (&raw)[4], float4& a, float4& b,
                          float4& c, float4& d, bool lds_lut) {
  const int xs[2] = {x0, x0 + 1}, ys[2] = {y0, y0 + 1};
  float4 v[4];
  bool ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int xc = xs[i & 1], yc = ys[i >> 1];
    ok[i] = (unsigned)xc < (unsigned)S.tex_w && (unsigned)yc < (unsigned)S.tex_h;
    const uint32_t w = raw[i];
    const uint32_t r = w & 255u, g = (w >> 8) & 255u, bl = (w >> 16) & 255u;
    if (lds_lut) v[i] = make_float4(g_tex_lut[r], g_tex_lut[g], g_tex_lut[bl], 0.0f);  // (separate branches:
    else v[i] = make_float4(S.tex_lut[r], S.tex_lut[g], S.tex_lut[bl], 0.0f);          // no flat load via a phi)
  }
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  a = ok[0] ? v[0] : z;
  b = ok[1] ? v[1] : z;
  c = ok[2] ? v[2] : z;
  d = ok[3] ? v[3] : z;
}

MR_DEV void tex_taps(const ShadeParams& S, int x0, int y0, float4& a, float4& b, float4& c, float4& d,
                     bool lds_lut = false) {
  const int xs[2] = {x0, x0 + 1}, ys[2] = {y0, y0 + 1};
  bool ok[4];
  float4 v[4];
  uint32_t idx[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int xc = xs[i & 1], yc = ys[i >> 1];
    ok[i] = (unsigned)xc < (unsigned)S.tex_w && (unsigned)yc < (unsigned)S.tex_h;
    const int x = ok[i] ? xc : 0, y = ok[i] ? yc : S.tex_h - 1;
    idx[i] = (uint32_t)(S.tex_h - 1 - y) * (uint32_t)S.tex_w + (uint32_t)x;  // torch.flip(maps, [H])
  }
  if (S.tex8) {  // 4-B texels, the exact values through the 256-entry table (LDS or L1-resident)
    uchar4 u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = S.tex8[idx[i]];
    asm volatile("" ::"v"(*(const int*)&u[0]), "v"(*(const int*)&u[1]), "v"(*(const int*)&u[2]),
                 "v"(*(const int*)&u[3]));
    if (lds_lut) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = make_float4(g_tex_lut[u[i].x], g_tex_lut[u[i].y], g_tex_lut[u[i].z], 0.0f);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = make_float4(S.tex_lut[u[i].x], S.tex_lut[u[i].y], S.tex_lut[u[i].z], 0.0f);
    }
    // consumed inside the branch: the table reads and the float-map loads below must not be merged
    // into one load through a phi of pointers (that is a flat load, LDS or global unknown)
    asm volatile("" ::"v"(v[0].x), "v"(v[0].y), "v"(v[0].z), "v"(v[1].x), "v"(v[1].y), "v"(v[1].z), "v"(v[2].x),
                 "v"(v[2].y), "v"(v[2].z), "v"(v[3].x), "v"(v[3].y), "v"(v[3].z));
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = S.tex[idx[i]];
    asm volatile("" ::"v"(v[0].x), "v"(v[0].y), "v"(v[0].z), "v"(v[1].x), "v"(v[1].y), "v"(v[1].z), "v"(v[2].x),
                 "v"(v[2].y), "v"(v[2].z), "v"(v[3].x), "v"(v[3].y), "v"(v[3].z));
  }
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  a = ok[0] ? v[0] : z;
  b = ok[1] ? v[1] : z;
  c = ok[2] ? v[2] : z;
  d = ok[3] ? v[3] : z;
}
// The sample position (and so the texel cell, where the bilinear gradient jumps) is computed in
// IEEE float32 with torch's operation order — uv = (b0 u0 + b1 u1) + b2 u2 (interpolate_face_
// attributes), uv * 2 - 1 (TexturesUV), ((g + 1) / 2) * (size - 1) (grid_sample, align_corners) —
// so that, given bitwise-equal barycentrics, the cell is the oracle's: a contracted (FMA) position
// one ulp off a texel boundary picks the neighbouring cell and a different gradient. The weights and
// the blend after it are continuous in the position and keep fast arithmetic.
MR_DEV void tex_blend(const ShadeParams& S, const TexTap& t, float out[3], bool lut);
// The sample position of (u, v) (tex_sample's first half): the cell, its weights' inputs and the border flags.
MR_DEV void tex_locate(const ShadeParams& S, float u, float v, TexTap& t) {
  const float gx = u * 2.0f - 1.0f, gy = v * 2.0f - 1.0f;
  float ix = ((gx + 1.0f) / 2.0f) * (float)(S.tex_w - 1);
  float iy = ((gy + 1.0f) / 2.0f) * (float)(S.tex_h - 1);
  t.gx_ok = !(ix < 0.0f) && !(ix > (float)(S.tex_w - 1));
  t.gy_ok = !(iy < 0.0f) && !(iy > (float)(S.tex_h - 1));
  ix = smin((float)(S.tex_w - 1), smax(ix, 0.0f));
  iy = smin((float)(S.tex_h - 1), smax(iy, 0.0f));
  t.ix = ix;
  t.iy = iy;
  t.x0 = (int)floorf(ix);
  t.y0 = (int)floorf(iy);
  t.pre = false;
}
// SPEC (specialised kernels): the map is known to have an 8-bit copy (S.tex8 non-null).
template <int SPEC = 0>
MR_DEV void tex_sample(const ShadeParams& S, float u, float v, float out[3], TexTap& t, bool lut = false) {
  tex_locate(S, u, v, t);
  if (SPEC || S.tex8) {  // the raw texels stay in the tap: a backward's second look-up (tex_sample_bwd) reloads nothing
    tex_taps_raw(S, t.x0, t.y0, t.raw);
    t.pre = true;
  }
  tex_blend(S, t, out, lut);
}
MR_DEV void tex_blend(const ShadeParams& S, const TexTap& t, float out[3], bool lut) {
  MR_FP_FAST
  const float ix = t.ix, iy = t.iy;
  const float x1 = (float)(t.x0 + 1), y1 = (float)(t.y0 + 1), x0 = (float)t.x0, y0 = (float)t.y0;
  const float nw = (x1 - ix) * (y1 - iy), ne = (ix - x0) * (y1 - iy);
  const float sw = (x1 - ix) * (iy - y0), se = (ix - x0) * (iy - y0);
  float4 a, b, c, d;
  if (t.pre) taps_from_raw(S, t.x0, t.y0, t.raw, a, b, c, d, lut);
  else tex_taps(S, t.x0, t.y0, a, b, c, d, lut);
  out[0] = ((a.x * nw + b.x * ne) + c.x * sw) + d.x * se;
  out[1] = ((a.y * nw + b.y * ne) + c.y * sw) + d.y * se;
  out[2] = ((a.z * nw + b.z * ne) + c.z * sw) + d.z * se;
}
// d(texel)/d(u,v) contracted with g (3 channels) -> (gu, gv)
MR_DEV void tex_sample_bwd(const ShadeParams& S, const TexTap& t, const float g[3], float& gu, float& gv,
                           bool lut = false) {
  MR_FP_FAST
  const float x1 = (float)(t.x0 + 1), y1 = (float)(t.y0 + 1), x0 = (float)t.x0, y0 = (float)t.y0;
  float4 a, b, c, d;
  if (t.pre) taps_from_raw(S, t.x0, t.y0, t.raw, a, b, c, d, lut);
  else tex_taps(S, t.x0, t.y0, a, b, c, d, lut);
  const float ga = (g[0] * a.x + g[1] * a.y) + g[2] * a.z;
  const float gb = (g[0] * b.x + g[1] * b.y) + g[2] * b.z;
  const float gc = (g[0] * c.x + g[1] * c.y) + g[2] * c.z;
  const float gd = (g[0] * d.x + g[1] * d.y) + g[2] * d.z;
  // factored as differences of taps: exactly 0 where the four taps are equal (a uniform texture
  // region), as in torch's grid_sample backward; the unfactored sum contracted into FMAs left the
  // rounding error of one product there (x (W - 1) x 1 / face area at the vertices).
  float gix = (gb - ga) * (y1 - t.iy) + (gd - gc) * (t.iy - y0);
  float giy = (gc - ga) * (x1 - t.ix) + (gd - gb) * (t.ix - x0);
  gix = t.gx_ok ? gix : 0.0f;
  giy = t.gy_ok ? giy : 0.0f;
  // ix = ((2u-1+1)/2)*(W-1)  ->  d ix / d u = W-1
  gu = gix * (float)(S.tex_w - 1);
  gv = giy * (float)(S.tex_h - 1);
}

// Stage the 256-entry u8 -> float texture table in the workgroup's LDS (g_tex_lut; uniform call, every
// thread of the workgroup; ends with a barrier). Returns the flag the shading functions take.
MR_DEV bool stage_tex_lut(const ShadeParams& S) {
  if (S.tex8)
    for (int i = threadIdx.x; i < 256; i += blockDim.x) g_tex_lut[i] = S.tex_lut[i];
  __syncthreads();
  return true;
}

// Per-pixel inputs gathered once for shading
struct PixGeom {
  float X[3][3];   // world positions of the 3 corners
  float Nv[3][3];  // vertex normals
  float uv[3][2];
  float col[3][3];
};

// Per-face shading inputs gathered once per call (k_shade_rec) so that per-pixel shading
// reads them with one 144-B record load indexed by the face id, instead of the dependent
// faces[f] -> verts / normals / uvs chain. A = uv (x, y, 0) or vertex colour per corner.
struct __attribute__((aligned(16))) ShadeRec {
  float X[9], N[9], A[9], pad[3];
};
static_assert(sizeof(ShadeRec) == 128, "ShadeRec is 8 float4 (pack_shade_recs, load_geom)");

MR_DEV void gather_geom(const ShadeParams& S, uint32_t face, PixGeom& G) {
  // Every field is written on every path and every loop is unrolled: a conditionally
  // initialised array element is otherwise demoted to scratch memory.
  const int32_t* fv = S.faces + 3 * (int64_t)face;
  const int32_t* fu = S.faces_uvs + 3 * (int64_t)face;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int32_t v = fv[c];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      G.X[c][k] = S.verts[3 * (int64_t)v + k];
      G.Nv[c][k] = S.light_kind == 0 ? S.vnormals[3 * (int64_t)v + k] : 0.0f;
      G.col[c][k] = S.tex_kind == 1 ? S.vcolors[3 * (int64_t)v + k] : 0.0f;
    }
    const int32_t t = S.tex_kind == 2 ? fu[c] : 0;
    G.uv[c][0] = S.tex_kind == 2 ? S.verts_uvs[2 * (int64_t)t] : 0.0f;
    G.uv[c][1] = S.tex_kind == 2 ? S.verts_uvs[2 * (int64_t)t + 1] : 0.0f;
  }
}

MR_DEV void make_shade_rec(const ShadeParams& S, uint32_t face, ShadeRec& R) {
  PixGeom G;
  gather_geom(S, face, G);
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      R.X[3 * c + k] = G.X[c][k];
      R.N[3 * c + k] = G.Nv[c][k];
      R.A[3 * c + k] = S.tex_kind == 1 ? G.col[c][k] : k < 2 ? G.uv[c][k] : 0.0f;
    }
  R.pad[0] = R.pad[1] = R.pad[2] = 0.0f;
}

// The ShadeRecs of faces [fa, fa + nf) packed by one 1024-thread workgroup, 256 faces per pass, bitwise
// make_shade_rec's records. Four lanes per face: lane c < 3 gathers corner c's vertex (one 12-B load per
// attribute instead of three 4-B ones), lane 3 the padding; the records are staged in LDS (`stage`, 32 KB) and
// stored as consecutive 16-B pieces. One lane per face writing its whole 128-B record made every store
// instruction touch ~64 cache lines, and the C5 render's 81,920 records took 13-19 us on 80 workgroups
// (profiles/r6n_binview_stamps.txt); the L1's address processing, not HBM, bounded it. Uniform call.
struct __attribute__((packed, aligned(4))) F3u {
  float x, y, z;
};
MR_DEV void pack_shade_recs(const ShadeParams& S, ShadeRec* __restrict__ out, int64_t fa, int64_t nf,
                            float* __restrict__ stage) {
  const int t = (int)threadIdx.x, lf = t >> 2, c = t & 3;
#pragma unroll 1
  for (int64_t p = 0; p < nf; p += 256) {
    const int np = (int)(nf - p < 256 ? nf - p : 256);
    float* r = stage + lf * 32;
    if (lf < np) {
      const int64_t f = fa + p + lf;
      if (c < 3) {
        const int64_t v = S.faces[3 * f + c];
        const F3u X = *(const F3u*)(S.verts + 3 * v);
        F3u Nn = {0.0f, 0.0f, 0.0f}, A = {0.0f, 0.0f, 0.0f};
        if (S.light_kind == 0) Nn = *(const F3u*)(S.vnormals + 3 * v);
        if (S.tex_kind == 1) {
          A = *(const F3u*)(S.vcolors + 3 * v);
        } else if (S.tex_kind == 2) {
          const int64_t tu = S.faces_uvs[3 * f + c];
          A.x = S.verts_uvs[2 * tu];
          A.y = S.verts_uvs[2 * tu + 1];
        }
        r[3 * c] = X.x; r[3 * c + 1] = X.y; r[3 * c + 2] = X.z;
        r[9 + 3 * c] = Nn.x; r[9 + 3 * c + 1] = Nn.y; r[9 + 3 * c + 2] = Nn.z;
        r[18 + 3 * c] = A.x; r[18 + 3 * c + 1] = A.y; r[18 + 3 * c + 2] = A.z;
      } else {
#pragma unroll
        for (int k = 27; k < 32; ++k) r[k] = 0.0f;
      }
    }
    __syncthreads();
    float4* o = (float4*)(out + fa + p);
    const float4* s4 = (const float4*)stage;
    for (int i = t; i < np * 8; i += 1024) o[i] = s4[i];
    __syncthreads();
  }
}

MR_DEV void load_geom(const ShadeRec* __restrict__ recs, uint32_t face, PixGeom& G) {
  const float4* q = (const float4*)(recs + face);
  float v[36];
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const float4 x = q[i];
    v[4 * i] = x.x; v[4 * i + 1] = x.y; v[4 * i + 2] = x.z; v[4 * i + 3] = x.w;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      G.X[c][k] = v[3 * c + k];
      G.Nv[c][k] = v[9 + 3 * c + k];
      G.col[c][k] = v[18 + 3 * c + k];
    }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    G.uv[c][0] = v[18 + 3 * c];
    G.uv[c][1] = v[18 + 3 * c + 1];
  }
}

// interpolate_face_attributes: sum_i b_i * attr_i
MR_DEV float interp3(float b0, float b1, float b2, float a0, float a1, float a2) {
  MR_FP_FAST
  return (b0 * a0 + b1 * a1) + b2 * a2;
}
// The same in IEEE float32, torch's order ((p0 + p1) + p2, no contraction): the uv interpolant that
// picks the texel cell (tex_sample).
MR_DEV float interp3_ieee(float b0, float b1, float b2, float a0, float a1, float a2) {
  return (b0 * a0 + b1 * a1) + b2 * a2;
}

// Intermediate values kept for the backward pass.
struct ShadeCache {
  float P[3], Nn[3], nh[3], nlen, nden, l[3], lh[3], llen, lden, v[3], vh[3], vlen, vden;
  float cosd, r[3], vr, as, spow, texel[3], amb[3], diff[3], spec[3], col[3];
  float ps, pc, zi, zimax, E, w, ex, delta, den;
  float qs, qc;  // 1 - ps, 1 - pc (unmasked: the derivatives' factor; sigmoid2)
  TexTap tap;
};

// Forward shading of one pixel (hit = face found). b = bary (after clip), z, sd = signed dist.
template <int SPEC = 0>
MR_DEV void shade_fwd(const ShadeParams& S, int n, bool hit, const PixGeom& G, float b0, float b1, float b2,
                      float z, float sd, ShadeOut& o, ShadeCache& C, bool lut = false) {
  MR_FP_FAST
  // SPEC 1: UV map with an 8-bit copy, point light, relu depth (the drop-in Phong render: compile-time
  // constants instead of the runtime switches)
  const int tex_kind = SPEC ? 2 : S.tex_kind, light_kind = SPEC ? 0 : S.light_kind;
  const int zbuf_mode = SPEC ? 0 : S.zbuf_mode;
  const float m = hit ? 1.0f : 0.0f;
  const float zb = hit ? z : -1.0f;    // zbuf background = -1
  const float dd = hit ? sd : -1.0f;   // dists background = -1
  // DepthRender: relu(zbuf[..., 0]); MeshRasterizer's zbuf[..., 0] itself in zbuf mode
  o.depth = (zbuf_mode || zb > 0.0f) ? zb : 0.0f;
  // SoftSilhouetteShader / sigmoid_alpha_blend
  sigmoid2((-dd) * S.inv_sigma_sil, C.ps, C.qs);
  C.ps *= m;
  o.sil = 1.0f - (1.0f - C.ps);
  // Phong colours (only meaningful for hit pixels; background weight is 0)
  for (int k = 0; k < 3; ++k) C.col[k] = 0.0f;
  if (hit) {
    for (int k = 0; k < 3; ++k) {
      C.P[k] = interp3(b0, b1, b2, G.X[0][k], G.X[1][k], G.X[2][k]);
      C.amb[k] = S.mat_amb[k] * S.light_amb[k];
    }
    if (tex_kind == 2) {
      const float u = interp3_ieee(b0, b1, b2, G.uv[0][0], G.uv[1][0], G.uv[2][0]);
      const float v = interp3_ieee(b0, b1, b2, G.uv[0][1], G.uv[1][1], G.uv[2][1]);
      tex_sample<SPEC>(S, u, v, C.texel, C.tap, lut);
    } else if (tex_kind == 1) {
      for (int k = 0; k < 3; ++k) C.texel[k] = interp3(b0, b1, b2, G.col[0][k], G.col[1][k], G.col[2][k]);
    } else {
      C.texel[0] = C.texel[1] = C.texel[2] = 1.0f;
    }
    if (light_kind == 0) {
      for (int k = 0; k < 3; ++k) C.Nn[k] = interp3(b0, b1, b2, G.Nv[0][k], G.Nv[1][k], G.Nv[2][k]);
      normalize3(C.Nn, C.nh, C.nlen, C.nden);
      for (int k = 0; k < 3; ++k) C.l[k] = S.light_loc[k] - C.P[k];
      normalize3(C.l, C.lh, C.llen, C.lden);
      C.cosd = dot3(C.nh, C.lh);
      const float angle = C.cosd > 0.0f ? C.cosd : 0.0f;
      const float* cc = S.cam_centers + (int64_t)n * S.cam_center_stride;
      for (int k = 0; k < 3; ++k) C.v[k] = cc[k] - C.P[k];
      normalize3(C.v, C.vh, C.vlen, C.vden);
      for (int k = 0; k < 3; ++k) C.r[k] = -C.lh[k] + 2.0f * (C.cosd * C.nh[k]);
      C.vr = dot3(C.vh, C.r);
      const float ms = C.cosd > 0.0f ? 1.0f : 0.0f;
      C.as = (C.vr > 0.0f ? C.vr : 0.0f) * ms;
      C.spow = fpow(C.as, S.shininess);
      for (int k = 0; k < 3; ++k) {
        C.diff[k] = S.mat_diff[k] * (S.light_diff[k] * angle);
        C.spec[k] = S.mat_spec[k] * (S.light_spec[k] * C.spow);
      }
    } else {
      for (int k = 0; k < 3; ++k) C.diff[k] = C.spec[k] = 0.0f;
    }
    for (int k = 0; k < 3; ++k) C.col[k] = (C.amb[k] + C.diff[k]) * C.texel[k] + C.spec[k];
  }
  // softmax_rgb_blend (K = 1)
  const float eps = 1e-10f;
  sigmoid2((-dd) * S.inv_sigma_rgb, C.pc, C.qc);
  C.pc *= m;
  const float alpha = 1.0f - C.pc;
  C.zi = ((S.zfar - zb) * S.inv_zrange) * m;
  C.zimax = smax(C.zi, eps);
  C.E = fexp((C.zi - C.zimax) * S.inv_gamma);
  C.w = C.pc * C.E;
  C.ex = fexp((eps - C.zimax) * S.inv_gamma);
  C.delta = smax(C.ex, eps);
  C.den = C.w + C.delta;
  const float rden = frcp(C.den);
  for (int k = 0; k < 3; ++k) o.rgb[k] = (C.w * C.col[k] + C.delta * S.bg[k]) * rden;
  o.alpha = 1.0f - alpha;
}

// Backward of shade_fwd for a hit pixel. Produces grads wrt z (zbuf), signed
// dist, bary (b0..b2), per-corner world positions / normals / vertex colours.
struct ShadeGrad {
  float gz, gsd, gb[3];
  float gX[3][3], gN[3][3], gC[3][3];  // per corner: b[c] * gP, b[c] * gNn, b[c] * gtex
  float gP[3], gNn[3], gtex[3];        // grads of the interpolated point, normal, texel
};

template <int SPEC = 0>
MR_DEV void shade_bwd(const ShadeParams& S, const PixGeom& G, float b0, float b1, float b2, float z,
                      const ShadeCache& C, float gD, float gS, const float gRGB[3], float gA, ShadeGrad& R,
                      bool lut = false) {
  MR_FP_FAST
  const int tex_kind = SPEC ? 2 : S.tex_kind, light_kind = SPEC ? 0 : S.light_kind;  // (as shade_fwd)
  const int zbuf_mode = SPEC ? 0 : S.zbuf_mode;
  const float b[3] = {b0, b1, b2};
  R.gz = 0.0f;
  R.gsd = 0.0f;
  for (int c = 0; c < 3; ++c) {
    R.gb[c] = 0.0f;
    for (int k = 0; k < 3; ++k) R.gX[c][k] = R.gN[c][k] = R.gC[c][k] = 0.0f;
  }
  // depth = relu(z) (zbuf mode: z)
  if (zbuf_mode || z > 0.0f) R.gz += gD;
  // silhouette: sil = 1 - (1 - ps), ps = sigmoid(-sd / sigma_sil)
  {
    const float gx = gS * (C.ps * C.qs);
    R.gsd += -(gx * S.inv_sigma_sil);
  }
  // rgb = (w*col + delta*bg) / den
  float gw = 0.0f, gdelta = 0.0f, gcol[3];
  {
    float gden = 0.0f;
    const float rden = frcp(C.den);
    for (int k = 0; k < 3; ++k) {
      const float num = C.w * C.col[k] + C.delta * S.bg[k];
      const float gnum = gRGB[k] * rden;
      gden += -gRGB[k] * num * (rden * rden);
      gw += gnum * C.col[k];
      gcol[k] = gnum * C.w;
      gdelta += gnum * S.bg[k];
    }
    gw += gden;
    gdelta += gden;
  }
  float gp = gA;  // A = 1 - (1 - p)
  float gzimax = 0.0f, gzi = 0.0f;
  {
    const float gu = (C.ex >= 1e-10f) ? gdelta * C.ex : 0.0f;  // clamp(min) backward
    gzimax += -(gu * S.inv_gamma);
    gp += gw * C.E;
    const float gE = gw * C.pc;
    const float gv = gE * C.E;
    gzi += gv * S.inv_gamma;
    gzimax += -(gv * S.inv_gamma);
    gzi += (C.zi >= 1e-10f) ? gzimax : 0.0f;  // max over K=1, then clamp(min=eps)
    R.gz += -(gzi * S.inv_zrange);
    const float gx = gp * (C.pc * C.qc);
    R.gsd += -(gx * S.inv_sigma_rgb);
  }
  // colours = (amb + diff) * texel + spec
  float gtex[3], gP[3] = {0.f, 0.f, 0.f}, gNn[3] = {0.f, 0.f, 0.f};
  for (int k = 0; k < 3; ++k) gtex[k] = gcol[k] * (C.amb[k] + C.diff[k]);
  if (light_kind == 0) {
    float gangle = 0.0f, gspow = 0.0f;
    for (int k = 0; k < 3; ++k) {
      gangle += gcol[k] * C.texel[k] * S.mat_diff[k] * S.light_diff[k];
      gspow += gcol[k] * S.mat_spec[k] * S.light_spec[k];
    }
    const float gas = (C.as > 0.0f) ? gspow * S.shininess * fpow(C.as, S.shininess - 1.0f) : 0.0f;
    const float ms = C.cosd > 0.0f ? 1.0f : 0.0f;
    const float gvr = (C.vr > 0.0f) ? gas * ms : 0.0f;
    float gvh[3], gr[3], glh[3], gnh[3];
    for (int k = 0; k < 3; ++k) {
      gvh[k] = gvr * C.r[k];
      gr[k] = gvr * C.vh[k];
    }
    // r = -lh + 2 * (cos * nh)
    float gcos = 2.0f * dot3(gr, C.nh);
    for (int k = 0; k < 3; ++k) {
      glh[k] = -gr[k];
      gnh[k] = 2.0f * C.cosd * gr[k];
    }
    gcos += (C.cosd > 0.0f) ? gangle : 0.0f;  // relu(cos) for diffuse
    for (int k = 0; k < 3; ++k) {
      gnh[k] += gcos * C.lh[k];
      glh[k] += gcos * C.nh[k];
    }
    float gl[3], gvv[3];
    normalize3_bwd(C.Nn, C.nlen, C.nden, gnh, gNn);
    normalize3_bwd(C.l, C.llen, C.lden, glh, gl);
    normalize3_bwd(C.v, C.vlen, C.vden, gvh, gvv);
    for (int k = 0; k < 3; ++k) gP[k] = -gl[k] - gvv[k];
  }
  for (int k = 0; k < 3; ++k) {
    R.gP[k] = gP[k];
    R.gNn[k] = gNn[k];
    R.gtex[k] = tex_kind == 1 ? gtex[k] : 0.0f;
  }
  for (int c = 0; c < 3; ++c) {
    R.gb[c] += dot3(G.X[c], gP);
    if (light_kind == 0) R.gb[c] += dot3(G.Nv[c], gNn);
    for (int k = 0; k < 3; ++k) {
      R.gX[c][k] = b[c] * gP[k];
      R.gN[c][k] = b[c] * gNn[k];
    }
  }
  if (tex_kind == 2) {
    float gu, gv;
    tex_sample_bwd(S, C.tap, gtex, gu, gv, lut);
    for (int c = 0; c < 3; ++c) R.gb[c] += G.uv[c][0] * gu + G.uv[c][1] * gv;
  } else if (tex_kind == 1) {
    for (int c = 0; c < 3; ++c) {
      R.gb[c] += dot3(G.col[c], gtex);
      for (int k = 0; k < 3; ++k) R.gC[c][k] = b[c] * gtex[k];
    }
  }
}

// ---------------- rasterizer backward (geometry_utils.h) ----------------
// FAST = false: IEEE divisions in the CPU's operand order (mr_rasterize_meshes_backward: per-fragment
// gradients bitwise equal to the CPU restatement, which matters on sliver faces whose gradients
// scale with 1/area^2); FAST = true: 1-ulp reciprocals (the fused render backward).
template <bool FAST> MR_DEV float bdiv(float a, float b) { return FAST ? a * frcp(b) : a / b; }
MR_DEV void edge_bwd(float px, float py, float ax, float ay, float bx, float by, float g, float d[6]) {
  // returns (dp.x, dp.y, da.x, da.y, db.x, db.y)
  d[0] = (by - ay) * g;
  d[1] = (ax - bx) * g;
  d[2] = (py - by) * g;
  d[3] = (bx - px) * g;
  d[4] = (ay - py) * g;
  d[5] = (px - ax) * g;
}

// BarycentricCoordsBackward -> dv[0..2] (x,y)
template <bool FAST>
MR_DEV void bary_bwd(float px, float py, const FaceRec& r, const float g[3], float dv[3][2]) {
  const float area = r.area;
  const float area2 = area * area;
  const float area_inv = bdiv<FAST>(1.0f, area);
  const float e0 = edge_fn(px, py, r.x1, r.y1, r.x2, r.y2);
  const float e1 = edge_fn(px, py, r.x2, r.y2, r.x0, r.y0);
  const float e2 = edge_fn(px, py, r.x0, r.y0, r.x1, r.y1);
  float de[6], da[6];
  // w0: e0 over (p, v1, v2); area over (v2, v0, v1)
  edge_bwd(px, py, r.x1, r.y1, r.x2, r.y2, g[0] * area_inv, de);
  edge_bwd(r.x2, r.y2, r.x0, r.y0, r.x1, r.y1, g[0] * bdiv<FAST>(-e0, area2), da);
  float v0x = da[2], v0y = da[3];
  float v1x = de[2] + da[4], v1y = de[3] + da[5];
  float v2x = de[4] + da[0], v2y = de[5] + da[1];
  // w1: e1 over (p, v2, v0)
  edge_bwd(px, py, r.x2, r.y2, r.x0, r.y0, g[1] * area_inv, de);
  edge_bwd(r.x2, r.y2, r.x0, r.y0, r.x1, r.y1, g[1] * bdiv<FAST>(-e1, area2), da);
  const float w1v0x = de[4] + da[2], w1v0y = de[5] + da[3];
  const float w1v1x = da[4], w1v1y = da[5];
  const float w1v2x = de[2] + da[0], w1v2y = de[3] + da[1];
  // w2: e2 over (p, v0, v1)
  edge_bwd(px, py, r.x0, r.y0, r.x1, r.y1, g[2] * area_inv, de);
  edge_bwd(r.x2, r.y2, r.x0, r.y0, r.x1, r.y1, g[2] * bdiv<FAST>(-e2, area2), da);
  const float w2v0x = de[2] + da[2], w2v0y = de[3] + da[3];
  const float w2v1x = de[4] + da[4], w2v1y = de[5] + da[5];
  const float w2v2x = da[0], w2v2y = da[1];
  dv[0][0] = (v0x + w1v0x) + w2v0x;
  dv[0][1] = (v0y + w1v0y) + w2v0y;
  dv[1][0] = (v1x + w1v1x) + w2v1x;
  dv[1][1] = (v1y + w1v1y) + w2v1y;
  dv[2][0] = (v2x + w1v2x) + w2v2x;
  dv[2][1] = (v2y + w1v2y) + w2v2y;
}

template <bool FAST>
MR_DEV void persp_bwd(float w0, float w1, float w2, float z0, float z1, float z2, const float go[3], float gb[3],
                      float gzv[3]) {
  const float t0 = w0 * z1 * z2, t1 = w1 * z0 * z2, t2 = w2 * z0 * z1;
  const float d = smax(t0 + t1 + t2, (float)MR_KEPS_D);
  const float gdt = -t0 * go[0] - t1 * go[1] - t2 * go[2];
  const float gd = bdiv<FAST>(gdt, d * d);
  const float g0 = gd + bdiv<FAST>(go[0], d), g1 = gd + bdiv<FAST>(go[1], d), g2 = gd + bdiv<FAST>(go[2], d);
  gb[0] = g0 * z1 * z2;
  gb[1] = g1 * z0 * z2;
  gb[2] = g2 * z0 * z1;
  gzv[0] = g1 * w1 * z2 + g2 * w2 * z1;
  gzv[1] = g0 * w0 * z2 + g2 * w2 * z0;
  gzv[2] = g0 * w0 * z1 + g1 * w1 * z0;
}

template <bool FAST>
MR_DEV void clip_bwd(float c0, float c1, float c2, const float go[3], float gb[3]) {
  const float w0 = smax(c0, 0.0f), w1 = smax(c1, 0.0f), w2 = smax(c2, 0.0f);
  const float s = smax(w0 + w1 + w2, 1e-5f);
  const float num = w0 * go[0] + w1 * go[1] + w2 * go[2];
  const float gs = bdiv<FAST>(-num, s * s);
  gb[0] = c0 > 0.0f ? bdiv<FAST>(go[0], s) + gs : 0.0f;
  gb[1] = c1 > 0.0f ? bdiv<FAST>(go[1], s) + gs : 0.0f;
  gb[2] = c2 > 0.0f ? bdiv<FAST>(go[2], s) + gs : 0.0f;
}

template <bool FAST>
MR_DEV void pt_line_bwd(float px, float py, float ax, float ay, float bx, float by, float g, float& gax,
                        float& gay, float& gbx, float& gby) {
  const float dx = bx - ax, dy = by - ay;
  const float t_bot = dx * dx + dy * dy;
  const float t_top = dx * (px - ax) + dy * (py - ay);
  const float t = bdiv<FAST>(t_top, t_bot);
  const float tt = smin(smax(t, 0.0f), 1.0f);
  const float qx = (1.0f - tt) * ax + tt * bx, qy = (1.0f - tt) * ay + tt * by;
  const float ex = qx - px, ey = qy - py;
  const float s0 = g * (1.0f - tt) * 2.0f, s1 = g * tt * 2.0f;
  gax = s0 * ex;
  gay = s0 * ey;
  gbx = s1 * ex;
  gby = s1 * ey;
}

// PointLineDistanceForward with a fast reciprocal: the backward only uses it to pick the
// closest edge (exact ties resolve as in the forward except within a few ulp).
MR_DEV float pt_line_dist_fast(float px, float py, float ax, float ay, float bx, float by) {
  const float dx = bx - ax, dy = by - ay;
  const float l2 = dx * dx + dy * dy;
  if ((double)l2 <= MR_KEPS_D) {
    const float ex = px - bx, ey = py - by;
    return ex * ex + ey * ey;
  }
  const float t = (dx * (px - ax) + dy * (py - ay)) * frcp(l2);
  const float tt = smin(smax(t, 0.0f), 1.0f);
  const float qx = ax + tt * dx, qy = ay + tt * dy;
  const float ex = px - qx, ey = py - qy;
  return ex * ex + ey * ey;
}

template <bool FAST>
MR_DEV void pt_tri_bwd(float px, float py, const FaceRec& r, float g, float gv[3][2]) {
  const float e01 = FAST ? pt_line_dist_fast(px, py, r.x0, r.y0, r.x1, r.y1) : pt_line_dist(px, py, r.x0, r.y0, r.x1, r.y1);
  const float e02 = FAST ? pt_line_dist_fast(px, py, r.x0, r.y0, r.x2, r.y2) : pt_line_dist(px, py, r.x0, r.y0, r.x2, r.y2);
  const float e12 = FAST ? pt_line_dist_fast(px, py, r.x1, r.y1, r.x2, r.y2) : pt_line_dist(px, py, r.x1, r.y1, r.x2, r.y2);
  // the closest edge (ties: e01, then e02, then e12; none when a distance is NaN), then ONE
  // pt_line_bwd on its endpoints (branch-free: per-lane selects instead of three divergent calls)
  const bool s01 = e01 <= e02 && e01 <= e12;
  const bool s02 = !s01 && e02 <= e01 && e02 <= e12;
  const bool s12 = !s01 && !s02 && e12 <= e01 && e12 <= e02;
  const int ia = s12 ? 1 : 0, ib = s01 ? 1 : 2;  // endpoint corners
  const float ax = ia ? r.x1 : r.x0, ay = ia ? r.y1 : r.y0;
  const float bx = ib == 1 ? r.x1 : r.x2, by = ib == 1 ? r.y1 : r.y2;
  float gax, gay, gbx, gby;
  pt_line_bwd<FAST>(px, py, ax, ay, bx, by, (s01 || s02 || s12) ? g : 0.0f, gax, gay, gbx, gby);
  const bool any = s01 || s02 || s12;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const bool isa = any && c == ia, isb = any && c == ib;
    gv[c][0] = isa ? gax : (isb ? gbx : 0.0f);
    gv[c][1] = isa ? gay : (isb ? gby : 0.0f);
  }
}

// RasterizeMeshesBackward for one (pixel, face): grads of (zbuf, bary, dists)
// -> grad of the face's NDC vertices gfv[corner][x,y,z].
template <bool FAST>
MR_DEV void raster_bwd_pixel(const FaceRec& r, float px, float py, bool persp, bool clipb, float gz, const float gb_up[3],
                             float gd, float gfv[3][3]) {
  const float e0 = edge_fn(px, py, r.x1, r.y1, r.x2, r.y2);
  const float e1 = edge_fn(px, py, r.x2, r.y2, r.x0, r.y0);
  const float e2 = edge_fn(px, py, r.x0, r.y0, r.x1, r.y1);
  // forward quantities recomputed for the derivative (with FAST, 1-ulp reciprocals: the signs,
  // hence `inside`, stay exact; the values feed gradients only)
  const float w0 = bdiv<FAST>(e0, r.area), w1 = bdiv<FAST>(e1, r.area), w2 = bdiv<FAST>(e2, r.area);
  float c0, c1, c2, b0, b1, b2;
  if (persp) {
    const float t0 = w0 * r.z1 * r.z2, t1 = w1 * r.z0 * r.z2, t2 = w2 * r.z0 * r.z1;
    const float d = smax(t0 + t1 + t2, (float)MR_KEPS_D);
    c0 = bdiv<FAST>(t0, d); c1 = bdiv<FAST>(t1, d); c2 = bdiv<FAST>(t2, d);
  } else { c0 = w0; c1 = w1; c2 = w2; }
  if (clipb) {
    const float u0 = smax(c0, 0.0f), u1 = smax(c1, 0.0f), u2 = smax(c2, 0.0f);
    const float sm = smax(u0 + u1 + u2, 1e-5f);
    b0 = bdiv<FAST>(u0, sm); b1 = bdiv<FAST>(u1, sm); b2 = bdiv<FAST>(u2, sm);
  } else { b0 = c0; b1 = c1; b2 = c2; }
  const bool inside = c0 > 0.0f && c1 > 0.0f && c2 > 0.0f;
  const float sign = inside ? -1.0f : 1.0f;
  float dd[3][2];
  pt_tri_bwd<FAST>(px, py, r, sign * gd, dd);
  float g0[3] = {gb_up[0] + gz * r.z0, gb_up[1] + gz * r.z1, gb_up[2] + gz * r.z2};
  float dz[3] = {0.0f, 0.0f, 0.0f};
  if (clipb) {
    float t[3];
    clip_bwd<FAST>(c0, c1, c2, g0, t);
    g0[0] = t[0]; g0[1] = t[1]; g0[2] = t[2];
  }
  if (persp) {
    float t[3];
    persp_bwd<FAST>(w0, w1, w2, r.z0, r.z1, r.z2, g0, t, dz);
    g0[0] = t[0]; g0[1] = t[1]; g0[2] = t[2];
  }
  float db[3][2];
  bary_bwd<FAST>(px, py, r, g0, db);
  const float bc[3] = {b0, b1, b2};
  for (int c = 0; c < 3; ++c) {
    gfv[c][0] = db[c][0] + dd[c][0];
    gfv[c][1] = db[c][1] + dd[c][1];
    gfv[c][2] = gz * bc[c] + dz[c];
  }
}

// ---------------- projection ----------------
MR_DEV void project_point(const ViewRec& V, const float X[3], float& vx, float& vy, float& vz, float& nx, float& ny) {
  vx = ((X[0] * V.R[0] + X[1] * V.R[3]) + X[2] * V.R[6]) + V.T[0];
  vy = ((X[0] * V.R[1] + X[1] * V.R[4]) + X[2] * V.R[7]) + V.T[1];
  vz = ((X[0] * V.R[2] + X[1] * V.R[5]) + X[2] * V.R[8]) + V.T[2];
  nx = V.ax * (vx / vz) + V.bx;
  ny = V.ay * (vy / vz) + V.by;
}

// g_ndc (x, y, z=view z) at world point X -> g_view; then g_X = R g_view,
// g_R += X (x) g_view, g_T += g_view.
MR_DEV void project_bwd(const ViewRec& V, const float X[3], const float gn[3], float gX[3], float gR[9], float gT[3]) {
  MR_FP_FAST
  const float vx = ((X[0] * V.R[0] + X[1] * V.R[3]) + X[2] * V.R[6]) + V.T[0];
  const float vy = ((X[0] * V.R[1] + X[1] * V.R[4]) + X[2] * V.R[7]) + V.T[1];
  const float vz = ((X[0] * V.R[2] + X[1] * V.R[5]) + X[2] * V.R[8]) + V.T[2];
  const float rz = frcp(vz);
  const float qx = vx * rz, qy = vy * rz;
  const float gqx = gn[0] * V.ax, gqy = gn[1] * V.ay;
  const float gv[3] = {gqx * rz, gqy * rz, gn[2] - gqx * qx * rz - gqy * qy * rz};
  for (int a = 0; a < 3; ++a) {
    gX[a] = (V.R[3 * a] * gv[0] + V.R[3 * a + 1] * gv[1]) + V.R[3 * a + 2] * gv[2];
    for (int bb = 0; bb < 3; ++bb) gR[3 * a + bb] += X[a] * gv[bb];
  }
  for (int bb = 0; bb < 3; ++bb) gT[bb] += gv[bb];
}

// ---------------- per-fragment Phong colour (K-deep soft shading) ----------------
// phong_shading for one (pixel, k) fragment: colour = (ambient + diffuse) * texel + specular,
// the same terms as shade_fwd's colour part, without the blend (softmax_rgb_blend couples the K
// fragments and is done by the caller). b = original-face barycentrics.
struct PhongCache {
  float P[3], Nn[3], nh[3], nlen, nden, l[3], lh[3], llen, lden, v[3], vh[3], vlen, vden;
  float cosd, r[3], vr, as, texel[3], amb[3], diff[3];
  TexTap tap;
};

MR_DEV void phong_fwd(const ShadeParams& S, int n, const PixGeom& G, float b0, float b1, float b2, float col[3],
                      PhongCache& C) {
  MR_FP_FAST
  for (int k = 0; k < 3; ++k) {
    C.P[k] = interp3(b0, b1, b2, G.X[0][k], G.X[1][k], G.X[2][k]);
    C.amb[k] = S.mat_amb[k] * S.light_amb[k];
  }
  if (S.tex_kind == 2) {
    const float u = interp3_ieee(b0, b1, b2, G.uv[0][0], G.uv[1][0], G.uv[2][0]);
    const float v = interp3_ieee(b0, b1, b2, G.uv[0][1], G.uv[1][1], G.uv[2][1]);
    tex_sample(S, u, v, C.texel, C.tap);
  } else if (S.tex_kind == 1) {
    for (int k = 0; k < 3; ++k) C.texel[k] = interp3(b0, b1, b2, G.col[0][k], G.col[1][k], G.col[2][k]);
  } else {
    C.texel[0] = C.texel[1] = C.texel[2] = 1.0f;
  }
  float spec[3] = {0.f, 0.f, 0.f};
  if (S.light_kind == 0) {
    for (int k = 0; k < 3; ++k) C.Nn[k] = interp3(b0, b1, b2, G.Nv[0][k], G.Nv[1][k], G.Nv[2][k]);
    normalize3(C.Nn, C.nh, C.nlen, C.nden);
    for (int k = 0; k < 3; ++k) C.l[k] = S.light_loc[k] - C.P[k];
    normalize3(C.l, C.lh, C.llen, C.lden);
    C.cosd = dot3(C.nh, C.lh);
    const float angle = C.cosd > 0.0f ? C.cosd : 0.0f;
    const float* cc = S.cam_centers + (int64_t)n * S.cam_center_stride;
    for (int k = 0; k < 3; ++k) C.v[k] = cc[k] - C.P[k];
    normalize3(C.v, C.vh, C.vlen, C.vden);
    for (int k = 0; k < 3; ++k) C.r[k] = -C.lh[k] + 2.0f * (C.cosd * C.nh[k]);
    C.vr = dot3(C.vh, C.r);
    C.as = (C.vr > 0.0f ? C.vr : 0.0f) * (C.cosd > 0.0f ? 1.0f : 0.0f);
    const float spow = fpow(C.as, S.shininess);
    for (int k = 0; k < 3; ++k) {
      C.diff[k] = S.mat_diff[k] * (S.light_diff[k] * angle);
      spec[k] = S.mat_spec[k] * (S.light_spec[k] * spow);
    }
  } else {
    for (int k = 0; k < 3; ++k) C.diff[k] = 0.0f;
  }
  for (int k = 0; k < 3; ++k) col[k] = (C.amb[k] + C.diff[k]) * C.texel[k] + spec[k];
}

// Backward of phong_fwd given the colour gradient gcol: gradients w.r.t. the barycentrics (gb),
// the interpolated world point (gP), the interpolated (unnormalised) normal (gNn), the texel
// (gtex) and the interpolated uv (guv; UV textures).
MR_DEV void phong_bwd(const ShadeParams& S, const PixGeom& G, const PhongCache& C, const float gcol[3], float gb[3],
                      float gP[3], float gNn[3], float gtex[3], float guv[2]) {
  MR_FP_FAST
  for (int k = 0; k < 3; ++k) {
    gtex[k] = gcol[k] * (C.amb[k] + C.diff[k]);
    gP[k] = gNn[k] = 0.0f;
  }
  if (S.light_kind == 0) {
    float gangle = 0.0f, gspow = 0.0f;
    for (int k = 0; k < 3; ++k) {
      gangle += gcol[k] * C.texel[k] * S.mat_diff[k] * S.light_diff[k];
      gspow += gcol[k] * S.mat_spec[k] * S.light_spec[k];
    }
    const float gas = (C.as > 0.0f) ? gspow * S.shininess * fpow(C.as, S.shininess - 1.0f) : 0.0f;
    const float gvr = (C.vr > 0.0f && C.cosd > 0.0f) ? gas : 0.0f;
    float gvh[3], gr[3], glh[3], gnh[3];
    for (int k = 0; k < 3; ++k) {
      gvh[k] = gvr * C.r[k];
      gr[k] = gvr * C.vh[k];
    }
    float gcos = 2.0f * dot3(gr, C.nh);
    for (int k = 0; k < 3; ++k) {
      glh[k] = -gr[k];
      gnh[k] = 2.0f * C.cosd * gr[k];
    }
    gcos += (C.cosd > 0.0f) ? gangle : 0.0f;
    for (int k = 0; k < 3; ++k) {
      gnh[k] += gcos * C.lh[k];
      glh[k] += gcos * C.nh[k];
    }
    float gl[3], gvv[3];
    normalize3_bwd(C.Nn, C.nlen, C.nden, gnh, gNn);
    normalize3_bwd(C.l, C.llen, C.lden, glh, gl);
    normalize3_bwd(C.v, C.vlen, C.vden, gvh, gvv);
    for (int k = 0; k < 3; ++k) gP[k] = -gl[k] - gvv[k];
  }
  guv[0] = guv[1] = 0.0f;
  for (int c = 0; c < 3; ++c) {
    gb[c] = dot3(G.X[c], gP);
    if (S.light_kind == 0) gb[c] += dot3(G.Nv[c], gNn);
  }
  if (S.tex_kind == 2) {
    tex_sample_bwd(S, C.tap, gtex, guv[0], guv[1]);
    for (int c = 0; c < 3; ++c) gb[c] += G.uv[c][0] * guv[0] + G.uv[c][1] * guv[1];
  } else if (S.tex_kind == 1) {
    for (int c = 0; c < 3; ++c) gb[c] += dot3(G.col[c], gtex);
  }
}

// Gradient of the bilinear texel w.r.t. the (flipped, RGBA-padded) map: the four taps' weights
// times gtex, added into gmap (Ht, Wt, 4) with float atomics (taps outside the map carry none).
MR_DEV void tex_map_bwd(const ShadeParams& S, const TexTap& t, const float gtex[3], float* __restrict__ gmap) {
  const float x1 = (float)(t.x0 + 1), y1 = (float)(t.y0 + 1), x0 = (float)t.x0, y0 = (float)t.y0;
  const float w[4] = {(x1 - t.ix) * (y1 - t.iy), (t.ix - x0) * (y1 - t.iy), (x1 - t.ix) * (t.iy - y0),
                      (t.ix - x0) * (t.iy - y0)};
  const int xs[4] = {t.x0, t.x0 + 1, t.x0, t.x0 + 1}, ys[4] = {t.y0, t.y0, t.y0 + 1, t.y0 + 1};
  for (int q = 0; q < 4; ++q) {
    if (xs[q] < 0 || ys[q] < 0 || xs[q] >= S.tex_w || ys[q] >= S.tex_h || w[q] == 0.0f) continue;
    float* dst = gmap + 4 * ((int64_t)(S.tex_h - 1 - ys[q]) * S.tex_w + xs[q]);  // torch.flip(maps, [H])
    for (int c = 0; c < 3; ++c)
      if (gtex[c] != 0.0f) atomicAdd(dst + c, w[q] * gtex[c]);
  }
}
