// mi355r — Fused pose-optimiser loss (forward partial sums, final reduction, backward).
// Part of the single translation unit mr_raster.hip (included there, in this order).
#pragma once

// ---------------------------------------------------------------------------
// Fused pose-optimiser loss (camera_pose_optimizer.py:257-276 Model.calc_loss):
//   sil_loss   = L1Loss()(silhouette, mask)               mean over all pixels
//   hloss      = HuberLoss(delta)(depth[mask], depth_ref[mask])   mean over the masked pixels
//   color_loss = MSELoss()(color, rgb_ref)                mean over all pixels x 3
//   total      = sil_loss + hloss + w_color * color_loss
// Forward: per-block partial sums (fixed-order wave / block reductions), then one block sums the
// partials in a fixed order (deterministic). Backward: the elementwise gradients of the three
// means, scaled by the device scalar dL/dtotal (no host read).
// ---------------------------------------------------------------------------
struct PoseLossParams {
  const float* depth;
  const float* sil;
  int64_t sil_stride;  // 1, or 4: channel 3 of an RGBA image (sil points at element 3)
  const float* rgb;
  int64_t rgb_stride;  // floats between consecutive pixels' colours (3, or 4 for an RGBA view)
  const uint8_t* mask;
  const float* depth_ref;
  const float* rgb_ref;  // (npix, 3)
  int64_t npix;
  float delta, w_color;
};
#define MR_LOSS_BLOCKS 2048

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

// out[0] = total; terms[0..2] = the three terms (out + 1 for the 4-float output of mr_pose_loss_forward);
// count = the masked pixels (the backward's Huber divisor). 1024 threads, each summing the block partials
// i, i + 1024, ... in order with four partials' loads in flight, then a fixed tree: deterministic.
__global__ void __launch_bounds__(1024) k_pose_loss_final(PoseLossParams P, const float* __restrict__ part,
                                                          const int* __restrict__ pcnt, int nb, float* __restrict__ out,
                                                          float* __restrict__ terms, int64_t* __restrict__ count) {
  __shared__ float sm[3][16];
  __shared__ long long sn[16];
  float a = 0.0f, b = 0.0f, c = 0.0f;
  long long n = 0;
#pragma unroll 1
  for (int i0 = threadIdx.x; i0 < nb; i0 += 4 * 1024) {
    float pa[4], pb[4], pc[4];
    int pn[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 1024 < nb ? i0 + u * 1024 : i0;
      pa[u] = part[3 * i];
      pb[u] = part[3 * i + 1];
      pc[u] = part[3 * i + 2];
      pn[u] = pcnt[i];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * 1024 < nb) {
        a += pa[u];
        b += pb[u];
        c += pc[u];
        n += pn[u];
      }
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    c += __shfl_xor(c, o, 64);
    n += __shfl_xor(n, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[0][w] = a;
    sm[1][w] = b;
    sm[2][w] = c;
    sn[w] = n;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float ta = 0.0f, tb = 0.0f, tc = 0.0f;
    long long tn = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
      ta += sm[0][k];
      tb += sm[1][k];
      tc += sm[2][k];
      tn += sn[k];
    }
    const float l1 = ta / (float)P.npix;
    const float hl = tb / (float)tn;  // an empty mask gives NaN, as torch's mean of nothing
    const float ms = tc / (float)(3 * P.npix);
    out[0] = (l1 + hl) + P.w_color * ms;
    terms[0] = l1;
    terms[1] = hl;
    terms[2] = ms;
    *count = tn;
  }
}

__global__ void __launch_bounds__(256) k_pose_loss_bwd(PoseLossParams P, const float* __restrict__ g_total,
                                                       const int64_t* __restrict__ count, float* __restrict__ g_depth,
                                                       float* __restrict__ g_sil, float* __restrict__ g_rgb) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= P.npix) return;
  const float g = g_total ? *g_total : 1.0f;  // NULL: dL/dtotal = 1 (mr_pose_loss_forward_grad's fallback)
  const bool m = P.mask[i] != 0;
  const float e = P.sil[i * P.sil_stride] - (m ? 1.0f : 0.0f);
  const float gs = g * ((e > 0.0f ? 1.0f : (e < 0.0f ? -1.0f : 0.0f)) / (float)P.npix);
  // an RGBA silhouette's gradient is the whole (npix, 4) image's: zero RGB, one 16-B store per pixel
  if (P.sil_stride == 4) ((float4*)g_sil)[i] = make_float4(0.0f, 0.0f, 0.0f, gs);
  else g_sil[i] = gs;
  g_depth[i] = m ? g * (huber_grad(P.depth[i] - P.depth_ref[i], P.delta) / (float)*count) : 0.0f;
  const float s = P.w_color * (2.0f / (float)(3 * P.npix));
  const float* c = P.rgb + i * P.rgb_stride;
  const float* r = P.rgb_ref + 3 * i;
  const float g0 = g * (s * (c[0] - r[0])), g1 = g * (s * (c[1] - r[1])), g2 = g * (s * (c[2] - r[2]));
  if (P.rgb_stride == 4) {
    ((float4*)g_rgb)[i] = make_float4(g0, g1, g2, 0.0f);
  } else {
    g_rgb[3 * i] = g0;
    g_rgb[3 * i + 1] = g1;
    g_rgb[3 * i + 2] = g2;
  }
}

// The forward with the gradients (mr_pose_loss_forward_grad): the loss is linear in dL/dtotal, so
// the gradients for dL/dtotal = 1 are written while the forward reads its inputs, and the backward only
// rescales them when dL/dtotal != 1 (k_pose_loss_scale) — one pass over the ~53 B/pixel of inputs
// instead of two. Same formulas (and operation order) as k_pose_loss_bwd with g = 1, and its access
// pattern: a wave's 64 lanes on 64 consecutive pixels (a 16-B strided RGBA channel read is one 1-KB span
// per load instruction; four adjacent pixels per lane measured 339 us, their 64-B lane strides touching
// 4x the cache lines per instruction), four such pixels per thread with all their loads issued first.
// The masked-pixel count
// the Huber gradient divides by comes first (k_mask_count: per-block counts, summed in a fixed order by
// every block of this kernel).
__global__ void __launch_bounds__(256) k_mask_count(const uint8_t* __restrict__ mask, int64_t npix, int* __restrict__ pcnt) {
  __shared__ float sm[4];
  int cnt = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < npix; i += (int64_t)gridDim.x * 256) cnt += mask[i] != 0;
  const float n = block_sum_256((float)cnt, sm);  // exact: < 2^24 per block
  if (threadIdx.x == 0) pcnt[blockIdx.x] = (int)n;
}
// the masked-pixel total of k_mask_count's nb partials, in a fixed order (one 256-thread block)
__global__ void __launch_bounds__(256) k_mask_total(const int* __restrict__ pcnt, int nb, int64_t* __restrict__ tot) {
  __shared__ long long sn[4];
  long long n = 0;
  for (int i = threadIdx.x; i < nb; i += 256) n += pcnt[i];
  for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
  if ((threadIdx.x & 63) == 0) sn[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) *tot = ((sn[0] + sn[1]) + sn[2]) + sn[3];
}

MR_DEV float sgnf(float e) { return e > 0.0f ? 1.0f : (e < 0.0f ? -1.0f : 0.0f); }

// Four pixels per thread (a workgroup's 1024 consecutive pixels, each load instruction lane-contiguous),
// one launch over the image (GRAD: also the gradients for dL/dtotal = 1); per-workgroup partial sums for
// k_pose_loss_final, reduced with DPP (fixed order). (A grid-stride loop over 2048 workgroups took 323-384
// us for the 16.7M-pixel C3 batch: it issues each iteration's loads after the previous iteration's
// stores; one pixel per thread with __shfl_xor block sums 295 us.)
#define MR_LOSS_PPT 4
template <bool GRAD>
__global__ void __launch_bounds__(256) k_pose_loss_fused(PoseLossParams P, const int64_t* __restrict__ mtot,
                                                         float* __restrict__ part, int* __restrict__ pcnt,
                                                         float* __restrict__ g_depth, float* __restrict__ g_sil,
                                                         float* __restrict__ g_rgb) {
  __shared__ float sm[4][4];
  const float* __restrict__ depth = P.depth;
  const float* __restrict__ dref = P.depth_ref;
  const float* __restrict__ sil = P.sil;
  const float* __restrict__ rgb = P.rgb;
  const float* __restrict__ rref = P.rgb_ref;
  const uint8_t* __restrict__ mask = P.mask;
  const int64_t i0 = (int64_t)blockIdx.x * (256 * MR_LOSS_PPT) + threadIdx.x;
  bool m[MR_LOSS_PPT], ok[MR_LOSS_PPT];
  float sv[MR_LOSS_PPT], dd[MR_LOSS_PPT], e[MR_LOSS_PPT][3];
#pragma unroll
  for (int u = 0; u < MR_LOSS_PPT; ++u) {  // every load first
    const int64_t i = i0 + u * 256;
    ok[u] = i < P.npix;
    const int64_t k = ok[u] ? i : 0;
    m[u] = mask[k] != 0;
    sv[u] = sil[k * P.sil_stride];
    dd[u] = depth[k] - dref[k];
    const float* c = rgb + k * P.rgb_stride;
    const float* r = rref + 3 * k;
    e[u][0] = c[0] - r[0];
    e[u][1] = c[1] - r[1];
    e[u][2] = c[2] - r[2];
  }
  float l1 = 0.0f, h = 0.0f, mse = 0.0f, cnt = 0.0f;
  const float cs = P.w_color * (2.0f / (float)(3 * P.npix));
#pragma unroll
  for (int u = 0; u < MR_LOSS_PPT; ++u) {
    if (!ok[u]) continue;
    const int64_t i = i0 + u * 256;
    const float es = sv[u] - (m[u] ? 1.0f : 0.0f);
    l1 += fabsf(es);
    if (m[u]) {
      h += huber_val(dd[u], P.delta);
      cnt += 1.0f;
    }
    mse += (e[u][0] * e[u][0] + e[u][1] * e[u][1]) + e[u][2] * e[u][2];
    if (GRAD) {
      const float gs = 1.0f * (sgnf(es) / (float)P.npix);
      if (P.sil_stride == 4) ((float4*)g_sil)[i] = make_float4(0.0f, 0.0f, 0.0f, gs);
      else g_sil[i] = gs;
      g_depth[i] = m[u] ? 1.0f * (huber_grad(dd[u], P.delta) / (float)*mtot) : 0.0f;
      if (P.rgb_stride == 4) {
        ((float4*)g_rgb)[i] = make_float4(cs * e[u][0], cs * e[u][1], cs * e[u][2], 0.0f);
      } else {
        g_rgb[3 * i] = cs * e[u][0];
        g_rgb[3 * i + 1] = cs * e[u][1];
        g_rgb[3 * i + 2] = cs * e[u][2];
      }
    }
  }
  const int w = threadIdx.x >> 6;
  l1 = wave_sum_f(l1);
  h = wave_sum_f(h);
  mse = wave_sum_f(mse);
  cnt = wave_sum_f(cnt);  // exact: <= 256 per wave
  if ((threadIdx.x & 63) == 0) {
    sm[0][w] = l1;
    sm[1][w] = h;
    sm[2][w] = mse;
    sm[3][w] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x] = ((sm[0][0] + sm[0][1]) + sm[0][2]) + sm[0][3];
    part[3 * blockIdx.x + 1] = ((sm[1][0] + sm[1][1]) + sm[1][2]) + sm[1][3];
    part[3 * blockIdx.x + 2] = ((sm[2][0] + sm[2][1]) + sm[2][2]) + sm[2][3];
    pcnt[blockIdx.x] = (int)(((sm[3][0] + sm[3][1]) + sm[3][2]) + sm[3][3]);
  }
}

// dL/dtotal != 1: the forward's gradients (written for dL/dtotal = 1) times dL/dtotal, in place (the
// grid reads the device scalar and returns when it is 1 — the optimiser's loss.backward()).
__global__ void __launch_bounds__(256) k_pose_loss_scale(const float* __restrict__ g_total, int64_t nd, int64_t ns,
                                                         int64_t nc, float* __restrict__ gd, float* __restrict__ gs,
                                                         float* __restrict__ gc) {
  const float g = *g_total;
  if (g == 1.0f) return;
  const int64_t G = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nd; i += G) gd[i] = g * gd[i];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < ns; i += G) gs[i] = g * gs[i];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nc; i += G) gc[i] = g * gc[i];
}

// upstream quaternion_to_matrix, one thread per quaternion (torch's elementwise operation order, no
// contraction: bitwise the torch formula of transforms.quaternion_to_matrix).
__global__ void __launch_bounds__(256) k_quat_to_matrix(const float* __restrict__ q, int64_t qs, int64_t N,
                                                        float* __restrict__ R) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const float r = q[n * qs], i = q[n * qs + 1], j = q[n * qs + 2], k = q[n * qs + 3];
  const float two_s = 2.0f / (((r * r + i * i) + j * j) + k * k);
  float* o = R + 9 * n;
  o[0] = 1.0f - two_s * (j * j + k * k);
  o[1] = two_s * (i * j - k * r);
  o[2] = two_s * (i * k + j * r);
  o[3] = two_s * (i * j + k * r);
  o[4] = 1.0f - two_s * (i * i + k * k);
  o[5] = two_s * (j * k - i * r);
  o[6] = two_s * (i * k - j * r);
  o[7] = two_s * (j * k + i * r);
  o[8] = 1.0f - two_s * (i * i + j * j);
}

// Its backward: R_ab = [a == b] + two_s * M_ab(q) with M quadratic in q and two_s = 2 / |q|^2, so
// dL/dq = two_s * sum_ab G_ab dM_ab/dq - (two_s^2 (sum_ab G_ab M_ab)) q.
__global__ void __launch_bounds__(256) k_quat_to_matrix_bwd(const float* __restrict__ q, int64_t qs,
                                                            const float* __restrict__ gR, int64_t N,
                                                            float* __restrict__ gq) {
  const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const float r = q[n * qs], i = q[n * qs + 1], j = q[n * qs + 2], k = q[n * qs + 3];
  const float two_s = 2.0f / (((r * r + i * i) + j * j) + k * k);
  const float* G = gR + 9 * n;
  // M (R = I + two_s M): diagonal -(..), off-diagonal products
  const float M[9] = {-(j * j + k * k), i * j - k * r, i * k + j * r,
                      i * j + k * r, -(i * i + k * k), j * k - i * r,
                      i * k - j * r, j * k + i * r, -(i * i + j * j)};
  float gm = 0.0f;
  for (int a = 0; a < 9; ++a) gm += G[a] * M[a];
  // sum_ab G_ab dM_ab / d(r, i, j, k)
  const float dr = (-k * G[1] + j * G[2] + k * G[3] - i * G[5] - j * G[6] + i * G[7]);
  const float di = (j * G[1] + k * G[2] + j * G[3] - 2.0f * i * G[4] - r * G[5] + k * G[6] + r * G[7] - 2.0f * i * G[8]);
  const float dj = (-2.0f * j * G[0] + i * G[1] + r * G[2] + i * G[3] + k * G[5] - r * G[6] + k * G[7] - 2.0f * j * G[8]);
  const float dk = (-2.0f * k * G[0] - r * G[1] + i * G[2] + r * G[3] - 2.0f * k * G[4] + j * G[5] + i * G[6] + j * G[7]);
  const float c = two_s * two_s * gm;  // d two_s / dq = -two_s^2 q
  gq[4 * n] = two_s * dr - c * r;
  gq[4 * n + 1] = two_s * di - c * i;
  gq[4 * n + 2] = two_s * dj - c * j;
  gq[4 * n + 3] = two_s * dk - c * k;
}
