// mi355r — Backward: the modular rasterizer backward (k_raster_bwd_slots) and the fused render
// backward (k_bwd_fused) with its segmented per-face reduction and per-slot R/T partials.
// Part of the single translation unit mr_raster.hip (included there, in this order).
#pragma once

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
MR_DEV void raster_bwd_fragment_v(const RasterBwdParams& P, int px, int py, int64_t f, float gzp, const float (&gb)[3],
                                  float gdp, float (&g)[3][3]);
MR_DEV void raster_bwd_fragment(const RasterBwdParams& P, int px, int py, int64_t pix, int64_t f, float (&g)[3][3]) {
  // an upstream gradient PyTorch passed as None arrives as NULL: zero
  const float gb[3] = {P.gb ? P.gb[3 * pix] : 0.0f, P.gb ? P.gb[3 * pix + 1] : 0.0f, P.gb ? P.gb[3 * pix + 2] : 0.0f};
  const float gzp = P.gz ? P.gz[pix] : 0.0f, gdp = P.gd ? P.gd[pix] : 0.0f;
  raster_bwd_fragment_v(P, px, py, f, gzp, gb, gdp, g);
}
// The same from the fragment's upstream gradients given as values (gz, gb, gd).
MR_DEV void raster_bwd_fragment_v(const RasterBwdParams& P, int px, int py, int64_t f, float gzp, const float (&gb)[3],
                                  float gdp, float (&g)[3][3]) {
  FaceRec r;
  const float* v = P.fv + 9 * f;
  r.x0 = v[0]; r.y0 = v[1]; r.z0 = v[2];
  r.x1 = v[3]; r.y1 = v[4]; r.z1 = v[5];
  r.x2 = v[6]; r.y2 = v[7]; r.z2 = v[8];
  r.area = (float)((double)edge_fn(r.x2, r.y2, r.x0, r.y0, r.x1, r.y1) + MR_KEPS_D);
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
// Sum of v over the wave in a fixed order: DPP butterflies inside each 16-lane row (quad xor 1, quad
// xor 2, half-row mirror, row mirror), then the four row sums in lane order. Uniform result; no LDS
// round trips (a __shfl_xor tree is six dependent ds_bpermute per value).
MR_DEV float wave_sum_f(float v) {
  v += dppf<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
  v += dppf<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
  v += dppf<0x141, 0xf>(v);  // row_half_mirror
  v += dppf<0x140, 0xf>(v);  // row_mirror
  const int b = __builtin_bit_cast(int, v);
  return ((__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)) +
           __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32))) +
         __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48));
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
  // seg_incl_sum's six steps, each only when some lane's run reaches that far back (uniform
  // branches; a skipped step would have kept every lane's value): runs are mostly shorter than a
  // tile row, so the two cross-row steps and the 8-lane step usually drop out (same sums, bitwise)
  const int r = lane & 15;
  float sh;
  if (__ballot(d >= 1)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x111, 0xf>(v[i]); v[i] = d >= 1 ? sh : v[i]; }
  }
  if (__ballot(d >= 2)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x112, 0xf>(v[i]); v[i] = d >= 2 ? sh : v[i]; }
  }
  if (__ballot(d >= 4)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x114, 0xf>(v[i]); v[i] = d >= 4 ? sh : v[i]; }
  }
  if (__ballot(d >= 8)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x118, 0xf>(v[i]); v[i] = d >= 8 ? sh : v[i]; }
  }
  if (__ballot(d > r)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x142, 0xa>(v[i]); v[i] = d > r ? sh : v[i]; }
  }
  if (__ballot(d > lane - 32)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x143, 0xc>(v[i]); v[i] = d > lane - 32 ? sh : v[i]; }
  }
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
  // element j = 64 i + lane of the flattened rows: row r = j / ACC, column c = j % ACC, advanced by
  // 64 = q ACC + m per block instead of divided out; 32-bit element offsets (F * ACC < 2^30, checked
  // on the host) keep the atomics' address in the scalar base + 32-bit vector offset form
  constexpr int q = 64 / ACC, m = 64 - q * ACC;
  int r = lane / ACC, c = lane - r * ACC;
#pragma unroll
  for (int i = 0; i < ACC; ++i) {
    if (64 * i < tot) {
      const int j = 64 * i + lane;
      if (j < tot) {
        const float x = lrow[j];
        if (x != 0.0f) atomicAdd(dst + ((uint32_t)lkey[r] * (uint32_t)ACC + (uint32_t)c), x);
      }
    }
    c += m;
    const bool wrap = c >= ACC;
    c = wrap ? c - ACC : c;
    r += wrap ? q + 1 : q;
    __builtin_amdgcn_sched_barrier(0);  // one row block at a time (no hoisting: register peak)
  }
  wave_lds_sync();
}
template <int ACC>
MR_DEV void seg_scatter(int key, float (&v)[ACC], float* __restrict__ dst, float* lrow, int* lkey) {
  seg_flush<ACC>(seg_stage<ACC>(key, v, lrow, lkey), dst, lrow, lkey);
}

// The slot's 12 R/T partial sums (gR[0..8], gT[0..2] summed over the wave) by a reduce-scatter (gfx950 lane
// swaps): v_permlane32_swap pairs value 2i's upper
// half-wave with value 2i+1's lower half, so one add leaves value 2i's 32 partial sums in lanes 0-31 and
// 2i+1's in lanes 32-63 (6 swaps + 6 adds for 12 values); v_permlane16_swap does the same inside each
// half for pairs of those vectors (3 + 3), leaving 4 values per vector, one per 16-lane row; four DPP
// butterfly steps per vector (quad xor 1, xor 2, half-row mirror, row mirror) finish every row's sum in
// all its lanes. 30 VALU instead of rt_partial's ~100 (12 six-step scans + readlanes + selects). Fixed
// order: deterministic (a view's R/T gradient sums these rows in slot order, k_rt_vgrad_a). o[j] row r holds
// value RT_VALUE(j, r). Uniform call (full EXEC). Round 5's twelve scans: 61.3 -> 58.3 us per launch
// (profiles/r6d_ab.txt).
// gfx950 v_permlane32_swap / v_permlane16_swap as inline asm: lanes 32-63 of x trade with lanes 0-31 of y
// (x = {x.lo, y.lo}, y = {x.hi, y.hi}); the 16-lane form trades x's odd rows with y's even rows. (The
// compiler's builtins returned a pair whose two halves it treated as one register when both feed one add:
// v_add_f32 v4, v4, v4 after the swap — tools/micro/rt_swap.hip.) The s_nop covers the VALU-write ->
// swap-read hazard the compiler cannot see through the asm.
MR_DEV void lane_swap32(float& x, float& y) { asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y)); }
MR_DEV void lane_swap16(float& x, float& y) { asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y)); }
#define RT_VALUE(j, r) (4 * (j) + (((r) & 1) << 1) + ((r) >> 1))
MR_DEV void rt_partial_swap(const float (&gR)[9], const float (&gT)[3], float (&o)[3]) {
  float h[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float a = 2 * i < 9 ? gR[2 * i] : gT[2 * i - 9];
    const float b = 2 * i + 1 < 9 ? gR[2 * i + 1] : gT[2 * i + 1 - 9];
    float x = a, y = b;
    lane_swap32(x, y);
    h[i] = x + y;
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float x = h[2 * j], y = h[2 * j + 1];
    lane_swap16(x, y);
    float v = x + y;
    v += dppf<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
    v += dppf<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
    v += dppf<0x141, 0xf>(v);  // row_half_mirror
    v += dppf<0x140, 0xf>(v);  // row_mirror
    o[j] = v;
  }
}
// Store rt_partial_swap's sums as the slot's 12-float partial row (lanes 0, 16, 32, 48 of each vector).
MR_DEV void rt_store_swap(float* __restrict__ dst, const float (&o)[3], int lane) {
  if ((lane & 15) == 0) {
    const int r = lane >> 4;
#pragma unroll
    for (int j = 0; j < 3; ++j) dst[RT_VALUE(j, r)] = o[j];
  }
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
// float4s per pixel of the half-1 -> half-2 hand-off: gz, gsd, gb[3], gP[3], gNn[3] (+ gtex[3] with vertex
// colours); the barycentrics stay in the forward fragment's registers
#define MR_BWD_REC(ACC) ((ACC) == 27 ? 4 : 3)
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
  // per-face gradient totals (F, ACC): 9 position rows, 9 normal rows [, 9 vertex-colour rows], in
  // fixed point (gfix, 64-bit integer atomics: order-independent, deterministic) plus the float
  // remainder gface of the rare component >= MR_FIX_MAX
  unsigned long long* gfix;
  float* gface;
  int* fflag;      // ctr + CTR_FLT: set when a float remainder is written
  float* rt_part;  // (slots, 12) per-slot R/T partial sums
  const float4* frec;  // (slots, 64) the forward's fragments (k_shade<1>): b0, b1, b2, signed dist (pixel order)
  const int* sgrp;     // (slots, 64) the slot's winners grouped by record (k_shade<1>)
  const uint8_t* sgpix; // (slots, 64) the tile pixel of each grouped position
};

// seg_stage for the fused backward: key = record id (runs are whole (tile, record) groups after
// sort_slot_pixels), face = the record's face (the accumulator row every view's records add into).
// The run totals are staged in LDS with their face.
template <int ACC>
MR_DEV int seg_stage_face(int key, int face, float (&v)[ACC], float* lrow, int* lkey) {
  const int lane = threadIdx.x & 63;
  const int prev = dpp_wave_shr1(key, -2);
  const bool head = lane == 0 || key != prev;
  const int d = lane - wave_incl_max(head ? lane : 0);
  const int r = lane & 15;
  float sh;
  if (__ballot(d >= 1)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x111, 0xf>(v[i]); v[i] = d >= 1 ? sh : v[i]; }
  }
  if (__ballot(d >= 2)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x112, 0xf>(v[i]); v[i] = d >= 2 ? sh : v[i]; }
  }
  if (__ballot(d >= 4)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x114, 0xf>(v[i]); v[i] = d >= 4 ? sh : v[i]; }
  }
  if (__ballot(d >= 8)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x118, 0xf>(v[i]); v[i] = d >= 8 ? sh : v[i]; }
  }
  if (__ballot(d > r)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x142, 0xa>(v[i]); v[i] = d > r ? sh : v[i]; }
  }
  if (__ballot(d > lane - 32)) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) { sh = v[i] + dppf<0x143, 0xc>(v[i]); v[i] = d > lane - 32 ? sh : v[i]; }
  }
  const int next = dpp_wave_shl1(key, -2);
  const bool emit = (lane == 63 || key != next) && key >= 0;
  const unsigned long long m = __ballot(emit);
  if (emit) {
    const int slot = __popcll(m & ((1ull << lane) - 1ull));
    lkey[slot] = face;
#pragma unroll
    for (int i = 0; i < ACC; ++i) lrow[slot * ACC + i] = v[i];
  }
  wave_lds_sync();
  return __popcll(m);
}
// seg_flush for the fused backward: each nonzero run component is added into its face's fixed-point
// total with a 64-bit integer atomic (order-independent: the totals are deterministic), lanes covering
// consecutive components of consecutive runs; a component of magnitude >= MR_FIX_MAX takes a float
// atomic into the face's float row. Straight-line, as seg_flush.
template <int ACC, int STRIDE = ACC>
MR_DEV void seg_flush_fix(int nt, unsigned long long* __restrict__ gfix, float* __restrict__ gface, const float* lrow,
                          const int* lkey, int* __restrict__ fflag) {
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int tot = nt * ACC;
  constexpr int qd = 64 / ACC, m = 64 - qd * ACC;
  int r = lane / ACC, c = lane - r * ACC;
#pragma unroll
  for (int i = 0; i < ACC; ++i) {
    if (64 * i < tot) {
      const int j = 64 * i + lane;
      if (j < tot) {
        const float x = lrow[j];
        // a geometry-only run (ACC = 9 position values) into an ACC-wide row: value 3 corner + k -> col_pos
        const int cc = (ACC == 9 && STRIDE == 27) ? (c / 3) * 6 + (c - (c / 3) * 3) : c;
        const uint32_t e = (uint32_t)lkey[r] * (uint32_t)STRIDE + (uint32_t)cc;
        if (fabsf(x) < MR_FIX_MAX) {
          if (x != 0.0f) atomicAdd(gfix + e, (unsigned long long)fix_of(x));
        } else {
          atomicAdd(gface + e, x);
          *fflag = 1;  // (the gathers then read the remainder rows)
        }
      }
    }
    c += m;
    const bool wrap = c >= ACC;
    c = wrap ? c - ACC : c;
    r += wrap ? qd + 1 : qd;
    __builtin_amdgcn_sched_barrier(0);
  }
  wave_lds_sync();
}

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
template <int SPEC = 0>
MR_DEV void bwd_slot_inputs(const RenderBwdParams& P, int slot, int gt, int f, int lane, FaceRec& r, float g[5],
                             float4& fr) {
  int n, px, py;
  slot_pixel(P, gt, lane, n, px, py);
  const int64_t pix = n * (int64_t)P.H * P.W + (int64_t)py * P.W + px;
  r = load_rec(P.recs, f < 0 ? 0 : f);
  fr = P.frec[(int64_t)slot * 64 + lane];
  const float* pD = P.gD ? P.gD + pix : g_zero4;
  const float* pS = P.gS ? P.gS + ((!SPEC && P.sil_rgba) ? 4 * pix + 3 : pix) : g_zero4;
  const float* pC = P.gRGB ? P.gRGB + pix * (SPEC ? 3 : P.rgb_ch) : g_zero4;
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
// Three waves per SIMD (<= 168 VGPRs): the sort / row staging pushed the kernel past 168, to two
// waves; capped at three it keeps no VGPR spills (a few SGPRs) and measured 75 -> 64 us per launch
// (render step 223k -> 232k frames/s, profiles/r4f_bands_ab.txt). Not the CLIP instantiation: its
// clip chain rule would spill ~60 VGPRs under the cap.
#ifndef MR_BWD_ATTR
#define MR_BWD_ATTR __attribute__((amdgpu_waves_per_eu(GEO ? (CLIP ? 2 : 4) : (CLIP ? 1 : 3))))
#endif
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

// GEO: no RGB gradient arrived (a depth and / or silhouette render's backward: camera_pose_optimizer.py:244,
// :248): the blends' backward reduces to d/dz (relu) and d/dsdist (the silhouette sigmoid) — the Phong,
// texture and barycentric terms are zero — so half 1 is skipped and the two values are computed in half 2,
// bitwise those the full path gives with a zero RGB gradient; only the 9 position columns of each face row
// are non-zero (NV = 9 values per run instead of ACC, added into the ACC-wide rows).
// Experiment builds only (-DMR_XP_BWD_STAMP, tools/bwd_stamps.py): per wave, the global clock at start /
// end, its slot count and the shader-clock cycles spent per phase of the slot loop (readable through
// mr_xp_bwd_stamps). Reads of the clock counters only.
#ifdef MR_XP_BWD_STAMP
#define MR_XP_WAVES 16384
__device__ unsigned long long g_bwd_stamp[MR_XP_WAVES * 8];
#define XP_CLK() __builtin_amdgcn_s_memtime()
#define XP_DECL unsigned long long xp_acc[5] = {0, 0, 0, 0, 0}, xp_t = 0, xp_rt0 = __builtin_amdgcn_s_memrealtime(); int xp_n = 0;
#define XP_MARK(i) do { const unsigned long long xp_c = XP_CLK(); if ((i) >= 0) xp_acc[(i) < 0 ? 0 : (i)] += xp_c - xp_t; xp_t = xp_c; } while (0)
#define XP_COUNT() (++xp_n)
#define XP_STORE() do { const unsigned long long xp_rt1 = __builtin_amdgcn_s_memrealtime(); \
    const int xp_w = (int)(blockIdx.x * 4 + (threadIdx.x >> 6)); const int xp_l = threadIdx.x & 63; \
    if (xp_w < MR_XP_WAVES && xp_l < 8) { unsigned long long xp_v = xp_l == 0 ? xp_rt0 : xp_l == 1 ? xp_rt1 : xp_l == 2 ? (unsigned long long)xp_n : xp_acc[0]; \
      xp_v = xp_l == 4 ? xp_acc[1] : xp_l == 5 ? xp_acc[2] : xp_l == 6 ? xp_acc[3] : xp_l == 7 ? xp_acc[4] : xp_v; \
      g_bwd_stamp[(size_t)xp_w * 8 + xp_l] = xp_v; } } while (0)
#else
#define XP_DECL
#define XP_MARK(i) do { } while (0)
#define XP_COUNT() do { } while (0)
#define XP_STORE() do { } while (0)
#endif

// The face of slot pixel record f (-1: face 0, an unconditional load's address) in view n.
MR_DEV uint32_t bwd_face(const RenderBwdParams& P, int f, int n) {
  return f >= 0 ? (uint32_t)(rec_orig(f, P.NF) - n * P.F) : 0u;
}

// SPEC 1 (the drop-in Phong render's case, chosen on the host): UV map with an 8-bit copy, point light, 3-channel
// RGB, relu depth, plain silhouette: the shading's runtime switches become compile-time constants.
template <int ACC, bool CLIP, bool GEO = false, int SPEC = 0>
__global__ void __launch_bounds__(256) MR_BWD_ATTR k_bwd_fused(RenderBwdParams P0) {
  constexpr int NV = GEO ? 9 : ACC;  // values per face row this kernel adds
  const RenderBwdParams& P = P0;
  __shared__ float lrow[4][64 * NV];
  __shared__ int lkey[4][64];
  constexpr int NREC = GEO ? 1 : MR_BWD_REC(ACC);
  __shared__ float4 lrec[4][NREC][64];
  const bool lut = GEO ? false : stage_tex_lut(P.S);  // the u8 texture table in LDS
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nslots = P.ctr[CTR_SLOTS];
  if (nslots <= 0) return;  // no covered tile: the prefetches below would read unwritten winners
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
  // lane -> (record f, tile pixel p) of the slot, grouped by record by the forward (k_shade<1>: sgrp, sgpix)
  int gt_c = P.stile[sc + lz], f_c = P.sgrp[(int64_t)sc * 64 + lane], p_c = P.sgpix[(int64_t)sc * 64 + lane];
  sc = min(s + G, slast);
  int sl_n = sc;
  int gt_n = P.stile[sc + lz], f_n = P.sgrp[(int64_t)sc * 64 + lane], p_n = P.sgpix[(int64_t)sc * 64 + lane];
  FaceRec r_c;
  float g_c[5];
  float4 fr_c;
  bwd_slot_inputs<SPEC>(P, sl_c, __builtin_amdgcn_readfirstlane(gt_c), f_c, p_c, r_c, g_c, fr_c);
  int nt_prev = -1, s_prev = 0;  // the previous slot's staged runs (-1: none yet)
  float rt_prev[3] = {0.0f, 0.0f, 0.0f};  // the previous slot's R/T sums (rt_partial_swap)
#define RT_STORE(slot) rt_store_swap(P.rt_part + (int64_t)(slot) * 12, rt_prev, lane)
  XP_DECL
  XP_MARK(-1);
  for (; s < send; s += G) {
    const RenderBwdParams& P = kernarg_params<RenderBwdParams>();  // see kernarg_params
    XP_COUNT();
    const int gt = __builtin_amdgcn_readfirstlane(gt_c), f = f_c, p = p_c;
    const FaceRec r = r_c;
    const float4 frag = fr_c;
    float gin[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) gin[i] = g_c[i];
    int n, px, py;
    slot_pixel(P, gt, p, n, px, py);
    XP_MARK(0);  // loop top
    // ---- half 1: blends / Phong / texture backward -> lrec
    if (!GEO && f >= 0) {
      PixGeom Gm;
      load_geom(P.srec, bwd_face(P, f, n), Gm);
      const float gD = gin[0], gS = gin[1];
      float gC[3] = {gin[2], gin[3], gin[4]};
      const float gA = (!SPEC && P.gRGB && P.rgb_ch == 4) ? g_alpha(P, gt, p) : 0.0f;
      FragEval e;
      float4 o[NREC];
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
        shade_fwd<SPEC>(P.S, n, true, Gm, e.b0, e.b1, e.b2, e.pz, e.sdist, so, C, lut);
        ShadeGrad SG;
        shade_bwd<SPEC>(P.S, Gm, e.b0, e.b1, e.b2, e.pz, C, gD, gS, gC, gA, SG, lut);
        o[0] = make_float4(SG.gz, SG.gsd, SG.gb[0], SG.gb[1]);
        o[1] = make_float4(SG.gb[2], SG.gP[0], SG.gP[1], SG.gP[2]);
        o[2] = make_float4(SG.gNn[0], SG.gNn[1], SG.gNn[2], SG.gtex[0]);
        if (NREC > 3) o[NREC - 1] = make_float4(SG.gtex[1], SG.gtex[2], 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < NREC; ++k) lrec[wave][GEO ? 0 : k][lane] = o[k];
    }
    if (!GEO) wave_lds_sync();
    XP_MARK(1);  // half 1
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
    // The next slots' inputs (slot s + G's records, fragments and upstream gradients; slot s + 2G's tile and
    // grouped winners), issued only now, after this slot's ShadeRec / texel loads and world corners: a
    // load's wait (vmcnt, in-order retirement) also waits for every vector-memory op issued before it, so
    // issued at the loop top (round 5) they put the next slots' HBM gradient reads in front of this slot's
    // ShadeRec wait (54.8 -> 52.6-53.4 us, profiles/r6i_latepf_ab.txt).
    gt_c = gt_n;
    f_c = f_n;
    p_c = p_n;
    sl_c = sl_n;
    bwd_slot_inputs<SPEC>(P, sl_c, __builtin_amdgcn_readfirstlane(gt_c), f_c, p_c, r_c, g_c, fr_c);
    sc = min(s + 2 * G, slast);
    sl_n = sc;
    gt_n = P.stile[sc + lz];
    f_n = P.sgrp[(int64_t)sc * 64 + lane];
    p_n = P.sgpix[(int64_t)sc * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);
    // previous slot's face rows and R/T partials, deferred to here (see above): the loads of
    // half 1 and the corners above are already in flight or consumed
    if (nt_prev >= 0) {
      seg_flush_fix<NV, ACC>(nt_prev, P.gfix, P.gface, lrow[wave], lkey[wave], P.fflag);
      RT_STORE(s_prev);
    }
    XP_MARK(2);  // corners + the next slots' prefetches + the previous slot's flush
    __builtin_amdgcn_sched_barrier(0);
    float gR[9], gT[3];
#pragma unroll
    for (int i = 0; i < 9; ++i) gR[i] = 0.0f;
#pragma unroll
    for (int i = 0; i < 3; ++i) gT[i] = 0.0f;
    float row[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) row[k] = 0.0f;
    int key = -1;
    if (f >= 0) {
      const float X[3][3] = {{w0.x, w0.y, w0.z}, {w0.w, w1.x, w1.y}, {w1.z, w1.w, w2.x}};
      float4 a0, a1, a2, a3;
      if (GEO) {
        // shade_fwd / shade_bwd's depth and silhouette terms (the same operations; the RGB terms vanish)
        const float pz = (CLIP && (r.flags & FR_CLIP))
                             ? [&] { FragEval es; eval_face(r, col_ndc(px, P.H, P.W), row_ndc(py, P.H, P.W), P.bbox_pad,
                                                            P.blur, P.persp, P.clipb, es); return es.pz; }()
                             : (frag.x * r.z0 + frag.y * r.z1) + frag.z * r.z2;
        float ps, qs;
        sigmoid2((-frag.w) * P.S.inv_sigma_sil, ps, qs);
        const float gz = (P.S.zbuf_mode || pz > 0.0f) ? 0.0f + gin[0] : 0.0f;
        const float gx = gin[1] * (ps * qs);
        const float gsd = 0.0f + -(gx * P.S.inv_sigma_sil);
        a0 = make_float4(gz, gsd, 0.f, 0.f);
        a1 = a2 = a3 = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        a0 = lrec[wave][0][lane];
        a1 = lrec[wave][1][lane];
        a2 = lrec[wave][2][lane];
        a3 = NREC > 3 ? lrec[wave][NREC - 1][lane] : make_float4(0.f, 0.f, 0.f, 0.f);
      }

      const float gb[3] = {a0.z, a0.w, a1.x};
      const float gP[3] = {a1.y, a1.z, a1.w};
      const float gNn[3] = {a2.x, a2.y, a2.z};
      const float b[3] = {frag.x, frag.y, frag.z};  // (the values half 1 shaded with)
      const float gt3[3] = {a2.w, a3.x, a3.y};
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
          if (GEO) {
            row[3 * c + k] = gX[k];  // (positions only; seg_flush_fix places them in the ACC-wide row)
          } else {
            row[col_pos<ACC>(c, k)] = b[c] * gP[k] + gX[k];
            row[col_nrm<ACC>(c, k)] = b[c] * gNn[k];
            if (ACC == 27) row[col_rgb<ACC>(c, k)] = b[c] * gt3[k];
          }
        }
      }
    }
    XP_MARK(3);  // raster + projection backward
    nt_prev = seg_stage_face<NV>(f >= 0 ? f : -1, key, row, lrow[wave], lkey[wave]);
    rt_partial_swap(gR, gT, rt_prev);
    s_prev = s;
    XP_MARK(4);  // segmented scan + R/T wave sums
  }
  if (nt_prev >= 0) {
    seg_flush_fix<NV, ACC>(nt_prev, P.gfix, P.gface, lrow[wave], lkey[wave], P.fflag);
    RT_STORE(s_prev);
  }
#undef RT_STORE
  XP_STORE();
}

// grad_views[n] = sum of the partial rows of view n's slots (fixed order: deterministic).
// out (N,12) PyTorch3D-frame R/T grads, or (gRcv, gtcv) non-null: the same grads written
// straight in the OpenCV frame (k_view_grads_to_opencv's chain rule, saving its launch).
// vslot holds (first slot, count) of each (view, band) range: N * bands firsts, then the counts.
// NT threads per workgroup (256, or 1024 inside k_rt_vgrad_a/b: four times the rows in flight).
template <int NT = 256>
MR_DEV void rt_reduce_view(const float* __restrict__ part, const int* __restrict__ vslot, int N, int bands,
                           float* __restrict__ out, float* __restrict__ gRcv, float* __restrict__ gtcv, int n) {
  constexpr int NW = NT / 64;
  __shared__ float sm[12][NW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // each thread sums whole 48-B partial rows (three 16-B loads in flight together instead of 12
  // dependent passes over the rows); per component the order is the same as a per-component loop
  float acc[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) acc[i] = 0.0f;
  // the view's slots in tile order: its bands' ranges concatenated (band b holds tile rows above band b+1's).
  // Thread t sums the slots t, t + NT, ... of that sequence in that order, whatever the band split — the
  // result does not depend on how many bands (i.e. on the batch size: a view's gradient is bitwise the same
  // in any batch). Four positions' rows are loaded together (a single-view batch has thousands of slots:
  // one dependent load per 256 slots made k_rt_reduce 24 us at C5), then added in sequence order.
  __shared__ int bfirst[MR_BANDS_MAX], bcount[MR_BANDS_MAX], bpre[MR_BANDS_MAX + 1];
  if ((int)threadIdx.x < bands) {  // the bands' ranges, loaded in parallel
    bfirst[threadIdx.x] = vslot[n * bands + threadIdx.x];
    bcount[threadIdx.x] = vslot[N * bands + n * bands + threadIdx.x];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int b = 0; b < bands; ++b) {
      bpre[b] = tot;
      tot += bcount[b];
    }
    bpre[bands] = tot;
  }
  __syncthreads();
  const int total = bpre[bands];
  auto slot_at = [&](int p) {  // sequence position -> slot: the last band starting at or before p (binary search:
    int lo = 0, hi = bands - 1;  // a walk advanced ~15 of C5's 64 bands per 1024 positions, one LDS read each)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (bpre[mid] <= p) lo = mid;
      else hi = mid - 1;
    }
    return bfirst[lo] + (p - bpre[lo]);
  };
#pragma unroll 1
  for (int p0 = threadIdx.x; p0 < total; p0 += 4 * NT) {
    float4 r[4][3];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + u * NT < total ? p0 + u * NT : total - 1;
      const float4* q = (const float4*)(part + (int64_t)slot_at(p) * 12);
      r[u][0] = q[0];
      r[u][1] = q[1];
      r[u][2] = q[2];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (p0 + u * NT >= total) break;
      const float4 a = r[u][0], c4 = r[u][1], c = r[u][2];
      acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
      acc[4] += c4.x; acc[5] += c4.y; acc[6] += c4.z; acc[7] += c4.w;
      acc[8] += c.x; acc[9] += c.y; acc[10] += c.z; acc[11] += c.w;
    }
  }
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    for (int o = 32; o > 0; o >>= 1) acc[i] += __shfl_xor(acc[i], o, 64);
    if (lane == 0) sm[i][wave] = acc[i];
  }
  __syncthreads();
  const int i = threadIdx.x;
  if (i >= 12) return;
  float v = sm[i][0];
#pragma unroll
  for (int k = 1; k < NW; ++k) v += sm[i][k];  // ((w0 + w1) + w2) + ...
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
                                                   int N, int bands, float* __restrict__ out, float* __restrict__ gRcv,
                                                   float* __restrict__ gtcv) {
  rt_reduce_view(part, vslot, N, bands, out, gRcv, gtcv, blockIdx.x);
}
