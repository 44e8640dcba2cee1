// mi355r — K-deep soft shading over stored fragments (forward and analytic backward).
// Part of the single translation unit mr_raster.hip (included there, in this order).
#pragma once

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
  int sorted;  // MR_FRAG_SORTED: each pixel's empty slots follow its filled ones (loops stop at the first)
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
      if (!m && P.sorted) break;  // the later masked slots repeat this one's z_inv: none is greater
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
    if (f < 0) {  // masked: prob 0, factor 1, weight 0
      if (P.sorted) break;
      continue;
    }
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
    if (P.sorted && __ballot(f >= 0) == 0ull) break;  // every lane past its last fragment (uniform)
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
            row[col_pos<ACC>(c, q)] = b[c] * gP[q];
            row[col_nrm<ACC>(c, q)] = b[c] * gNn[q];
            if (ACC == 27) row[col_rgb<ACC>(c, q)] = b[c] * gtex[q];
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
      if (P.g_zbuf) P.g_zbuf[base + k] = 0.0f;
      if (P.g_dists) P.g_dists[base + k] = 0.0f;
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
            row[col_pos<ACC>(c, q)] = b[c] * gP[q];
            row[col_nrm<ACC>(c, q)] = b[c] * gNn[q];
            if (ACC == 27) row[col_rgb<ACC>(c, q)] = b[c] * gtex[q];
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
      if (P.g_zbuf) P.g_zbuf[base + k] = gz;
      P.g_dists[base + k] = gd;
      if (P.g_bary) {
        P.g_bary[3 * (base + k)] = gb[0];
        P.g_bary[3 * (base + k) + 1] = gb[1];
        P.g_bary[3 * (base + k) + 2] = gb[2];
      }
    }
    // (empty slots: their zero gradients were written by coalesced fills before the launch; written
    // here one lane per pixel they were K-strided 4-B stores, most of this kernel's time at large K)
    if (!P.sil && S.light_kind == 0) seg_scatter<ACC>(key, row, P.gface, lrow[wave], lkey[wave]);
    else if (ACC == 27 && !P.sil) seg_scatter<ACC>(key, row, P.gface, lrow[wave], lkey[wave]);
  }
}

// Backward of the fused soft silhouette over the flat fragment array (coalesced, balanced: a chunk of
// MR_SIL_CHUNK fragments per workgroup iteration whatever the tile it came from; one wave per slot ran each
// heavy tile's ~3k fragments serially), the blend's derivative (k_frag_shade_bwd's silhouette branch: the
// distance gradient) chained straight into the rasterizer's backward (raster_bwd_fragment with zero depth /
// barycentric gradients) — no fragment gradient tensors; face_verts gradients summed per chunk in an LDS
// hash (a chunk's fragments come from one or two tiles), flushed with one global atomic per face component.
#define MR_SIL_CHUNK 1024
struct SilBwdParams {
  RasterBwdParams R;
  int T, TX;
  float isig;
  const int* ctr;
  const int* stile;
  const int4* sent;
  const float4* spix;
  const float* grad_rgba;
};
__global__ void __launch_bounds__(256) k_sil_bwd(SilBwdParams P) {
  __shared__ LdsAcc<9> L;
  const int ne = P.ctr[CTR_SENT];
  const int64_t HW = (int64_t)P.R.H * P.R.W;
#pragma unroll 1
  for (int c0 = blockIdx.x * MR_SIL_CHUNK; c0 < ne; c0 += gridDim.x * MR_SIL_CHUNK) {  // uniform
    acc_init(L);
    __syncthreads();
    const int c1 = min(c0 + MR_SIL_CHUNK, ne);
#pragma unroll 1
    for (int e = c0 + (int)threadIdx.x; e < c1; e += 256) {
      const int4 en = P.sent[e];
      const int s = en.w;
      const int gt = P.stile[s];
      const int n = gt / P.T, t = gt - n * P.T;
      const int ty = t / P.TX, tx = t - ty * P.TX;
      const int pl = en.z & 255, k = en.z >> 8;
      const int px = tx * MR_TS + (pl & 7), py = ty * MR_TS + (pl >> 3);
      const float4 inf = P.spix[(int64_t)s * 64 + pl];
      const float alpha_nz = inf.x;
      const int nzero = __float_as_int(inf.y), kzero = __float_as_int(inf.z);
      const float d = __int_as_float(en.y);
      const float g_alpha = -P.grad_rgba[4 * (n * HW + (int64_t)py * P.R.W + px) + 3];  // A = 1 - alpha
      const float prob = frag_prob(d, P.isig);
      const float one_m = 1.0f - prob;
      const float others = nzero == 0 ? alpha_nz * frcp(one_m) : (nzero == 1 && kzero == k ? alpha_nz : 0.0f);
      const float g_prob = g_alpha * (-others);
      float sp_, sq_;
      sigmoid2((-d) * P.isig, sp_, sq_);
      const float gd = -((g_prob * (sp_ * sq_)) * P.isig);
      const float gb0[3] = {0.0f, 0.0f, 0.0f};
      float g[3][3];
      raster_bwd_fragment_v(P.R, px, py, en.x, 0.0f, gb0, gd, g);
      acc_add<9>(L, P.R.gfv, en.x, &g[0][0]);
    }
    __syncthreads();
    acc_flush(L, P.R.gfv);
    __syncthreads();
  }
}
