// mi355r — K > 1 raster (PyTorch3D faces_per_pixel > 1): the pair-enumerating register-list kernel
// (K <= 64) and the LDS insertion-list kernel (K <= 128).
// Part of the single translation unit mr_raster.hip (included there, in this order).
#pragma once

// K > 1 (modular path, PyTorch3D faces_per_pixel): one wave per non-empty tile, one pixel per
// lane. The tile's faces are staged 64 at a time in the wave's LDS (one record per lane, then
// read as broadcasts) and each lane keeps the K smallest packed (z, face) keys of its pixel in
// an ascending per-lane LDS list (insertion; lane-strided so the 64 lanes hit 64 banks). The
// K smallest keys are exactly the CPU's K nearest with the earlier face winning depth ties,
// already in output order (RasterizeMeshesNaiveCpu keeps the K smallest, then sorts).
// LDS per wave: K * 512 B of keys + 4.25 KB of staged records.
#define MR_KMAX 128
MR_DEV size_t rk_wave_bytes(int K) { return (size_t)K * 64 * 8 + 64 * sizeof(FaceRec) + 64 * sizeof(int); }
__global__ void __launch_bounds__(256) k_raster_k(FwdParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char rk_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wpg = blockDim.x >> 6;
  const int K = P.K;
  unsigned char* base = rk_lds + (size_t)wave * rk_wave_bytes(K);
  unsigned long long* q = (unsigned long long*)base + lane;  // q[k * 64]
  FaceRec* rs = (FaceRec*)(base + (size_t)K * 64 * 8);
  int* ids = (int*)(rs + 64);
  const int nslots = P.ctr[CTR_SLOTS];
  const float pad = P.bbox_pad, blur = P.blur;
  const bool persp = P.persp != 0, clipb = P.clipb != 0;
  const bool fast_ok = !(blur > 0.0f);
  const int H = P.H, W = P.W;
  const int64_t HW = (int64_t)H * W;
#pragma unroll 1
  for (int s = blockIdx.x * wpg + wave; s < nslots; s += gridDim.x * wpg) {
    const int gt = P.stile[s];
    const int n = gt / P.T, t = gt - n * P.T;
    const int ty = t / P.TX, tx = t - ty * P.TX;
    const int px = tx * MR_TS + (lane & 7), py = ty * MR_TS + (lane >> 3);
    const bool in_img = px < W && py < H;
    const float xf = col_ndc(in_img ? px : 0, H, W), yf = row_ndc(in_img ? py : 0, H, W);
    const int cc = P.cnt[gt], ex = P.start[gt];
    const int64_t vb = P.vbase[n];
    // the scan's overflow rule: scan the whole view
    const bool ovf = vb + ex + cc > P.list_cap || (P.mfpb > 0 && cc > P.mfpb);
    const int64_t vfirst = P.view_first ? P.view_first[n] : (int64_t)n * P.F;
    const int64_t vcnt = P.view_count ? P.view_count[n] : P.F;
    const int count = ovf ? (int)(vcnt < 0x7fffffffll ? vcnt : 0x7fffffffll) : cc;
    int nq = 0;
#pragma unroll 1
    for (int eb = 0; eb < count; eb += 64) {
      const int e = eb + lane;
      if (e < count) {
        const int id = ovf ? (int)(vfirst + e) : P.list[vb + ex + e];
        rs[lane] = P.recs[id];
        ids[lane] = id;
      }
      wave_lds_sync();
      const int m = count - eb < 64 ? count - eb : 64;
#pragma unroll 1
      for (int j = 0; j < m; ++j) {
        const FaceRec r = rs[j];
        const int id = ids[j];
        float pz;
        int cid = id;
        bool keep = false;
        if (in_img && (r.flags & FR_PAIR)) {
          // a split face: the pair's candidate is inserted from its own entry (both entries are
          // listed for every pixel either can keep), or from the first triangle's entry when an
          // overflow unit scans the view's records (second triangles are not scanned there)
          keep = pair_keep(P.recs, P.NF, id, r, xf, yf, pad, blur, persp, clipb, cid, pz) &&
                 (cid == id || (ovf && id < P.NF));
        } else if (in_img && (r.flags & FR_VALID)) {
          keep = frag_keep(r, xf, yf, pad, blur, persp, clipb, fast_ok && (r.flags & FR_FAST), pz);
        }
        if (keep) {
          const unsigned long long key = frag_key(pz, (int)rec_code(cid, P.NF));
          if (key < MR_KEY_EMPTY && (nq < K || key < q[(nq - 1) * 64])) {
            int i = nq < K ? nq : K - 1;
            while (i > 0 && q[(i - 1) * 64] > key) {
              q[i * 64] = q[(i - 1) * 64];
              --i;
            }
            q[i * 64] = key;
            nq += nq < K ? 1 : 0;
          }
        }
      }
      wave_lds_sync();
    }
    if (!in_img) continue;
    const int64_t pix = (n * HW + (int64_t)py * W + px) * K;
#pragma unroll 1
    for (int k = 0; k < K; ++k) {
      int64_t f = -1;
      float z = -1.0f, d = -1.0f, b0 = -1.0f, b1 = -1.0f, b2 = -1.0f;
      if (k < nq) {
        const int id = code_rec((unsigned)(q[k * 64] & 0xffffffffull), P.NF);
        const FaceRec r = P.recs[id];
        FragEval ev;
        eval_face(r, xf, yf, pad, blur, persp, clipb, ev);  // kept by construction
        if (r.flags & FR_CLIP) clip_unconvert(P.crec[id], ev.b0, ev.b1, ev.b2, ev.b0, ev.b1, ev.b2);
        f = rec_orig(id, P.NF); z = ev.pz; d = ev.sdist; b0 = ev.b0; b1 = ev.b1; b2 = ev.b2;
      }
      P.p2f[pix + k] = f;
      P.zbuf[pix + k] = z;
      P.dists[pix + k] = d;
      P.bary[3 * (pix + k) + 0] = b0;
      P.bary[3 * (pix + k) + 1] = b1;
      P.bary[3 * (pix + k) + 2] = b2;
    }
  }
}

// K <= 64 (PyTorch3D faces_per_pixel > 1): one wave per non-empty tile, each lane keeping its pixel's
// K nearest (z, face) keys in REGISTERS (KP >= K slots, ascending; a shift-insert whose KP steps are
// independent selects, shifted out through slot 0 so the array is never dynamically indexed). The
// keys are evaluated over (face, pixel) PAIRS: as in k_tile_raster, each lane clips one list entry's
// padded bbox to the tile, a DPP prefix numbers the pairs and a pass evaluates 64 of them exactly
// (frag_keep / pair_keep, one per lane) — with blur a face of the deform workload covers ~a quarter
// of the tile, and evaluating every listed face at all 64 pixels (the previous kernel) ran 4x the
// exact tests. A kept candidate goes to its PIXEL's LDS bucket; the buckets drain into the register
// lists when the fullest has less than MR_KP_ROOM slots left and at the end of the tile, so a list
// takes one insert per candidate of its pixel (~4 of K = 50 on the deform workload), not one per
// listed face, and a drain whose lists will all hold <= 8 / 16 / 32 keys runs that many shift steps
// instead of KP. A pass is limited to the entries whose candidates the buckets can still take (an
// entry adds at most one candidate per pixel). The K nearest keys do not depend on the insertion
// order: the fragments are bitwise those of the face-at-a-time kernel (deform workload: 2.22 ms
// (two waves per tile, every face at every pixel) -> see DESIGN.md for this kernel's numbers).
#ifndef MR_KP_BC
#define MR_KP_BC 20  // 20 KB of LDS per wave with the stage and the depth-order permutation: 8 waves per CU (24: 7, 1.75 per SIMD; 1192-1206 -> 1150-1169 us at K = 50, profiles/r5m_soft_bucket_ab.txt)
#endif
// Shift-insert of key into the first NS positions of the ascending list q (positions >= NS are
// empty for every lane of the wave and stay so: no lane holds more than NS keys).
template <int KP, int NS>
MR_DEV void insert_ns(unsigned long long (&q)[KP], unsigned long long key) {
  if (__ballot(key < q[NS - 1]) != 0ull) {
    bool ltk = key < q[NS - 1];
#pragma unroll
    for (int k = NS - 1; k > 0; --k) {
      const bool ltp = key < q[k - 1];
      q[k] = ltk ? (ltp ? q[k - 1] : key) : q[k];
      ltk = ltp;
    }
    q[0] = ltk ? key : q[0];
  }
}

#ifndef MR_KP_ROOM
#define MR_KP_ROOM 8  // drain the buckets once the fullest one has less room than this (12 with 24-deep buckets; 10 -> 8: 1157-1169 -> 1125-1139 us, profiles/r5n_soft_room_ab.txt)
#endif
#ifndef MR_KP_SORT
#define MR_KP_SORT 2048  // tiles of 65 .. MR_KP_SORT listed faces are walked in depth order (0: never)
#endif
#define MR_KP_ZBINS 256
struct KpStage {
  StageRecs rec;
  int id[64];
  int meta[64];
  int mark[64];
  int bcnt[64];
  unsigned long long cmask[64];
  unsigned long long thr[64];  // per pixel: its list's last key once full (else EMPTY), set at each drain
  unsigned long long bucket[MR_KP_BC][64];
};
static_assert(MR_KP_SORT <= 65536 && sizeof(KpStage::bucket) >= sizeof(int) * (MR_KP_SORT + MR_KP_ZBINS),
              "the depth sort's scratch lives in the bucket array");

// Depth order of a tile's list (entries list[base .. base + count)): perm[i] = the entry to walk i-th,
// by a counting sort of the faces' nearest vertex depth into MR_KP_ZBINS bins over the tile's range
// (order inside a bin: arbitrary). The K nearest keys do not depend on the walk order, so this only
// changes how much work they take: walked near-to-far, each pixel's list holds its final keys after
// its first few dozen candidates and the full list's last key (S.thr) then keeps the farther
// candidates out of the buckets — the drains' shift-inserts, ~40 % of the kernel on the deform
// workload, run about once per kept key instead of once per candidate. The bucket array is the
// sort's scratch (the bins' counts and each entry's (bin, rank)); only perm (u16) persists.
MR_DEV void kp_depth_order(const FwdParams& P, KpStage& S, unsigned short* perm, int64_t base, int count, int lane) {
  float* zs = (float*)&S.bucket[0][0];  // count floats, then the bins
  int* zb = (int*)zs;
  int* bins = (int*)zs + MR_KP_SORT;
  float lo = INFINITY, hi = -INFINITY;
#pragma unroll 1
  for (int e = lane; e < count; e += 64) {
    const float* f = (const float*)(P.recs + P.list[base + e]);
    const float z = fminf(fminf(f[2], f[5]), f[8]);  // z0, z1, z2
    zs[e] = z;
    lo = fminf(lo, z);
    hi = fmaxf(hi, z);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o, 64));
    hi = fmaxf(hi, __shfl_xor(hi, o, 64));
  }
  const float span = hi - lo;
  const float scale = span > 0.0f && span < INFINITY ? (float)MR_KP_ZBINS / span : 0.0f;
#pragma unroll
  for (int k = 0; k < MR_KP_ZBINS / 64; ++k) bins[k * 64 + lane] = 0;
  wave_lds_sync();
#pragma unroll 1
  for (int e = lane; e < count; e += 64) {
    const float t = (zs[e] - lo) * scale;
    const int b = t >= 0.0f ? min((int)t, MR_KP_ZBINS - 1) : 0;  // (NaN: bin 0)
    zb[e] = (b << 16) | atomicAdd(&bins[b], 1);
  }
  wave_lds_sync();
  int c[MR_KP_ZBINS / 64], run = 0;  // lane owns bins [4 lane, 4 lane + 4): exclusive prefix
#pragma unroll
  for (int k = 0; k < MR_KP_ZBINS / 64; ++k) {
    c[k] = run;
    run += bins[lane * (MR_KP_ZBINS / 64) + k];
  }
  const int off = wave_incl_sum(run) - run;
  wave_lds_sync();
#pragma unroll
  for (int k = 0; k < MR_KP_ZBINS / 64; ++k) bins[lane * (MR_KP_ZBINS / 64) + k] = off + c[k];
  wave_lds_sync();
#pragma unroll 1
  for (int e = lane; e < count; e += 64) {
    const int v = zb[e];
    perm[bins[v >> 16] + (v & 0xffff)] = (unsigned short)e;
  }
  wave_lds_sync();
}

// SIL: the fused soft silhouette (mr_soft_silhouette_forward): instead of writing the K fragment
// slots, each pixel's sorted list is blended (sigmoid_alpha_blend, as k_frag_shade_fwd over the stored
// fragments, same operations in the same order) into rgba, and the tile's fragments are kept compactly
// for the backward: {packed face, signed distance, lane | k << 8, slot} per fragment in one flat array (each
// slot's run lane-major, a pixel's fragments consecutive, at an offset from one atomic per wave; the total in
// ctr[CTR_SENT]), and per tile pixel the blend's
// {product of the non-zero (1 - p) factors, number of zero factors, index of the last zero factor}.
template <int KP, bool SIL = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_raster_kp(FwdParams P) {
  __shared__ KpStage S;
  __shared__ unsigned short perm[MR_KP_SORT > 0 ? MR_KP_SORT : 1];
  const int lane = threadIdx.x;
  if ((int)blockIdx.x >= P.ctr[CTR_SLOTS]) return;
  const int s = P.sorder ? P.sorder[blockIdx.x] : (int)blockIdx.x;
  const int K = P.K;
  const float pad = P.bbox_pad, blur = P.blur;
  const bool persp = P.persp != 0, clipb = P.clipb != 0;
  const bool fast_ok = !(blur > 0.0f);
  const int H = P.H, W = P.W;
  const int64_t HW = (int64_t)H * W;
  const int gt = P.stile[s];
  const int n = gt / P.T, t = gt - n * P.T;
  const int ty = t / P.TX, tx = t - ty * P.TX;
  const int x0 = tx * MR_TS, y0 = ty * MR_TS;
  const int px = x0 + (lane & 7), py = y0 + (lane >> 3);
  const bool in_img = px < W && py < H;
  const int cc = P.cnt[gt], ex = P.start[gt];
  const int64_t vb = P.vbase[n];
  const bool ovf = vb + ex + cc > P.list_cap || (P.mfpb > 0 && cc > P.mfpb);
  const int64_t vfirst = P.view_first ? P.view_first[n] : (int64_t)n * P.F;
  const int64_t vcnt = P.view_count ? P.view_count[n] : P.F;
  const int count = ovf ? (int)(vcnt < 0x7fffffffll ? vcnt : 0x7fffffffll) : cc;
  const int xe = min(x0 + MR_TS, W) - 1, ye = min(y0 + MR_TS, H) - 1;  // the tile's last pixels inside the image
  const bool zsorted = MR_KP_SORT > 0 && !ovf && count > 64 && count <= MR_KP_SORT;
  if (zsorted) {
    kp_depth_order(P, S, perm, vb + ex, count, lane);
    if (lane == 0) atomicAdd(&P.ctr[CTR_ZWALK], 1);  // tiles walked near-to-far (mr_workspace_stats out[4])
  }
  unsigned long long q[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) q[k] = MR_KEY_EMPTY;
  auto insert = [&](unsigned long long key) {
    if (__ballot(key < q[KP - 1]) != 0ull) {
      bool ltk = key < q[KP - 1];
#pragma unroll
      for (int k = KP - 1; k > 0; --k) {
        const bool ltp = key < q[k - 1];
        q[k] = ltk ? (ltp ? q[k - 1] : key) : q[k];
        ltk = ltp;
      }
      q[0] = ltk ? key : q[0];
    }
  };
  S.bcnt[lane] = 0;
  S.mark[lane] = -1;
  S.thr[lane] = MR_KEY_EMPTY;
  int mb = 0;  // the fullest bucket's fill (uniform)
  int lc = 0;  // keys in this lane's list
  // Drain: every bucket's keys into its lane's list. The lists' fill after the drain is known before
  // it (all keys are distinct, so none is dropped until a list holds KP): when no lane will hold more
  // than NS keys, only the first NS positions can change and the shift runs NS steps, not KP
  // (most lists hold a few keys: the full KP-step shift was ~half of the kernel).
  auto drain = [&]() {
    wave_lds_sync();
    const int c = S.bcnt[lane];
    const int mc = __builtin_amdgcn_readlane(wave_incl_max(c), 63);
    lc = min(lc + c, KP);
    const int need = __builtin_amdgcn_readlane(wave_incl_max(lc), 63);
    if (need <= 8 && KP > 8) {
#pragma unroll 1
      for (int i = 0; i < mc; ++i) insert_ns<KP, (KP > 8 ? 8 : KP)>(q, i < c ? S.bucket[i][lane] : MR_KEY_EMPTY);
    } else if (need <= 16 && KP > 16) {
#pragma unroll 1
      for (int i = 0; i < mc; ++i) insert_ns<KP, (KP > 16 ? 16 : KP)>(q, i < c ? S.bucket[i][lane] : MR_KEY_EMPTY);
    } else if (need <= 32 && KP > 32) {
#pragma unroll 1
      for (int i = 0; i < mc; ++i) insert_ns<KP, (KP > 32 ? 32 : KP)>(q, i < c ? S.bucket[i][lane] : MR_KEY_EMPTY);
    } else {
#pragma unroll 1
      for (int i = 0; i < mc; ++i) insert(i < c ? S.bucket[i][lane] : MR_KEY_EMPTY);
    }
    S.bcnt[lane] = 0;
    S.thr[lane] = lc >= KP ? q[KP - 1] : MR_KEY_EMPTY;  // a full list rejects every key above its last
    wave_lds_sync();
    mb = 0;
  };
#pragma unroll 1
  for (int eb = 0; eb < count; eb += 64) {
    const int e = eb + lane;
    unsigned long long cmask = 0;
    if (e < count) {
      const int id = ovf ? (int)(vfirst + e) : P.list[vb + ex + (zsorted ? (int)perm[e] : e)];
      const FaceRec r = load_rec(P.recs, id);
      // candidate pixels: the record's padded bbox; an overflow unit scans only first triangles of
      // split faces, so there it covers both triangles of the pair (as k_tile_raster)
      float bx0 = r.xmin, bx1 = r.xmax, by0 = r.ymin, by1 = r.ymax;
      bool bvalid = (r.flags & FR_VALID) != 0;
      if (ovf && (r.flags & FR_PAIR) && id < P.NF) {
        const FaceRec ro = load_rec(P.recs, P.NF + id);
        if (ro.flags & FR_VALID) {
          bx0 = bvalid ? smin(bx0, ro.xmin) : ro.xmin;
          bx1 = bvalid ? smax(bx1, ro.xmax) : ro.xmax;
          by0 = bvalid ? smin(by0, ro.ymin) : ro.ymin;
          by1 = bvalid ? smax(by1, ro.ymax) : ro.ymax;
          bvalid = true;
        }
      }
      int cx0, cx1, cy0, cy1;
      ndc_range_to_pix(bx0 - pad, bx1 + pad, W, H, cx0, cx1);
      ndc_range_to_pix(by0 - pad, by1 + pad, H, W, cy0, cy1);
      cx0 = max(cx0, x0);
      cx1 = min(cx1, xe);
      cy0 = max(cy0, y0);
      cy1 = min(cy1, ye);
      if (bvalid && cx0 <= cx1 && cy0 <= cy1) cmask = rect_mask(cx0 - x0, cx1 - x0, cy0 - y0, cy1 - y0);
      stage_rec_put(S.rec, lane, r);
      S.id[lane] = id;
    }
    const int np = __popcll(cmask);
    const int pincl = wave_incl_sum(np);
    const int pexcl = pincl - np;
    const int NP = __builtin_amdgcn_readlane(pincl, 63);
    S.meta[lane] = pexcl;
    S.cmask[lane] = cmask;
#pragma unroll 1
    for (int pb = 0; pb < NP;) {
      if (mb > MR_KP_BC - MR_KP_ROOM) drain();
      // the entry straddling pb, and the first entry past what the buckets can still take
      const int first = 63 - __builtin_clzll(__ballot(np > 0 && pexcl <= pb));
      const int lim = first + (MR_KP_BC - mb);
      const int pend = min(pb + 64, lim < 64 ? __builtin_amdgcn_readlane(pexcl, lim) : NP);
      wave_lds_sync();
      if (np > 0 && pexcl > pb && pexcl < pend) S.mark[pexcl - pb] = lane;
      wave_lds_sync();
      int m = S.mark[lane];
      S.mark[lane] = -1;
      if (lane == 0) m = first;
      m = wave_incl_max(m);
      const int qq = pb + lane;
      if (qq < pend) {
        const int p = kth_bit(S.cmask[m], qq - S.meta[m]);
        const FaceRec r = stage_rec_get(S.rec, m);
        const int id = S.id[m];
        const float xf = col_ndc(x0 + (p & 7), H, W), yf = row_ndc(y0 + (p >> 3), H, W);
        float pz = 0.0f;
        int cid = id;
        bool keep = false;
        if (r.flags & FR_PAIR) {  // the split face's two triangles as one candidate (pair rule)
          keep = pair_keep(P.recs, P.NF, id, r, xf, yf, pad, blur, persp, clipb, cid, pz) &&
                 (cid == id || (ovf && id < P.NF));
          keep = keep && frag_key(pz, (int)rec_code(cid, P.NF)) < S.thr[p];
        } else if (r.flags & FR_VALID) {
          // the depth key first: a key the pixel's full list rejects skips the point-triangle distance
          // (most of the late candidates of a near-to-far walk)
          bool inside = false;
          keep = frag_depth(r, xf, yf, pad, persp, clipb, fast_ok && (r.flags & FR_FAST), pz, inside) &&
                 frag_key(pz, (int)rec_code(cid, P.NF)) < S.thr[p] &&
                 (inside || (blur > 0.0f && !(pt_tri_dist(xf, yf, r) >= blur)));
        }
        const unsigned long long key = frag_key(pz, (int)rec_code(cid, P.NF));
        if (keep) {  // (keys a full list would reject do not enter the buckets)
          const int pos = atomicAdd(&S.bcnt[p], 1);
          S.bucket[pos][p] = key;
        }
      }
      pb = pend;
      wave_lds_sync();
      mb = __builtin_amdgcn_readlane(wave_incl_max(S.bcnt[lane]), 63);  // the fullest bucket
    }
    wave_lds_sync();  // the stage is rewritten by the next batch
  }
  drain();
  if (SIL) {
    const float xf = col_ndc(in_img ? px : 0, H, W), yf = row_ndc(in_img ? py : 0, H, W);
    const int cnt = in_img ? min(lc, K) : 0;
    const int incl = wave_incl_sum(cnt);
    int base = 0;
    if (lane == 63) base = atomicAdd(&P.ctr[CTR_SENT], incl);  // the slot's run of the flat fragment array
    base = __builtin_amdgcn_readlane(base, 63);
    int4* ent = P.sent + base + (incl - cnt);
    float alpha_nz = 1.0f;
    int nzero = 0, kzero = -1;
    // the keys leave the list through q[0]; the next key's record is loaded while this one is evaluated
    // (unconditional load of record 0 for an empty key: a guarded load would be waited on at once)
    unsigned long long key_n = q[0];
    FaceRec r_n = load_rec(P.recs, key_n < MR_KEY_EMPTY ? code_rec((unsigned)(key_n & 0xffffffffull), P.NF) : 0);
#pragma unroll 1
    for (int k = 0; k < K; ++k) {
      if (__ballot(key_n < MR_KEY_EMPTY) == 0ull) break;
      const unsigned long long key = key_n;
      const FaceRec r = r_n;
#pragma unroll
      for (int i = 0; i + 1 < KP; ++i) q[i] = q[i + 1];
      q[KP - 1] = MR_KEY_EMPTY;
      key_n = q[0];
      r_n = load_rec(P.recs, key_n < MR_KEY_EMPTY ? code_rec((unsigned)(key_n & 0xffffffffull), P.NF) : 0);
      if (!in_img || !(key < MR_KEY_EMPTY)) continue;
      const int id = code_rec((unsigned)(key & 0xffffffffull), P.NF);
      FragEval ev;
      eval_face(r, xf, yf, pad, blur, persp, clipb, ev);  // kept by construction
      const float prob = frag_prob(ev.sdist, P.isig);
      const float one_m = 1.0f - prob;
      if (one_m == 0.0f) {
        ++nzero;
        kzero = k;
      } else {
        alpha_nz *= one_m;
      }
      ent[k] = make_int4(rec_orig(id, P.NF), __float_as_int(ev.sdist), lane | (k << 8), s);
    }
    if (in_img) {
      const int64_t q4 = n * HW + (int64_t)py * W + px;
      const float alpha = nzero ? 0.0f : alpha_nz;
      ((float4*)P.sil)[q4] = make_float4(1.0f, 1.0f, 1.0f, 1.0f - alpha);
    }
    P.spix[(int64_t)s * 64 + lane] = make_float4(alpha_nz, __int_as_float(nzero), __int_as_float(kzero), 0.0f);
    return;
  }
  if (!in_img) return;
  const int64_t pix = (n * HW + (int64_t)py * W + px) * K;
  const float xf = col_ndc(px, H, W), yf = row_ndc(py, H, W);
  // only the filled slots (k_fill wrote the background of every slot); keys shifted out through q[0]
  // (constant indices only: the array stays in registers)
  unsigned long long key_n = q[0];  // (the next key's record in flight, as in the SIL tail above)
  FaceRec r_n = load_rec(P.recs, key_n < MR_KEY_EMPTY ? code_rec((unsigned)(key_n & 0xffffffffull), P.NF) : 0);
#pragma unroll 1
  for (int k = 0; k < K; ++k) {
    if (__ballot(key_n < MR_KEY_EMPTY) == 0ull) break;
    const unsigned long long key = key_n;
    const FaceRec r = r_n;
#pragma unroll
    for (int i = 0; i + 1 < KP; ++i) q[i] = q[i + 1];
    q[KP - 1] = MR_KEY_EMPTY;
    key_n = q[0];
    r_n = load_rec(P.recs, key_n < MR_KEY_EMPTY ? code_rec((unsigned)(key_n & 0xffffffffull), P.NF) : 0);
    if (!(key < MR_KEY_EMPTY)) continue;
    const int id = code_rec((unsigned)(key & 0xffffffffull), P.NF);
    FragEval ev;
    eval_face(r, xf, yf, pad, blur, persp, clipb, ev);  // kept by construction
    if (r.flags & FR_CLIP) clip_unconvert(P.crec[id], ev.b0, ev.b1, ev.b2, ev.b0, ev.b1, ev.b2);
    P.p2f[pix + k] = rec_orig(id, P.NF);
    P.zbuf[pix + k] = ev.pz;
    P.dists[pix + k] = ev.sdist;
    P.bary[3 * (pix + k) + 0] = ev.b0;
    P.bary[3 * (pix + k) + 1] = ev.b1;
    P.bary[3 * (pix + k) + 2] = ev.b2;
  }
}

// Slot order for k_raster_kp, heaviest tile lists first (longest-processing-time-first over the wave slots):
// a counting sort of the slots by list length (buckets of 4 entries, descending; order inside a bucket
// arbitrary — every tile's result is independent of when it runs). One workgroup.
#ifndef MR_KP_ORDER
#define MR_KP_ORDER 1
#endif
#define MR_ORDER_BINS 2048
__global__ void __launch_bounds__(1024) k_slot_order(const int* __restrict__ ctr, const int* __restrict__ stile,
                                                     const int* __restrict__ cnt, int* __restrict__ order) {
  __shared__ int hist[MR_ORDER_BINS];
  __shared__ int part[16];
  const int t = threadIdx.x, n = ctr[CTR_SLOTS];
  for (int i = t; i < MR_ORDER_BINS; i += 1024) hist[i] = 0;
  __syncthreads();
  for (int s = t; s < n; s += 1024) atomicAdd(&hist[MR_ORDER_BINS - 1 - min(cnt[stile[s]] >> 2, MR_ORDER_BINS - 1)], 1);
  __syncthreads();
  // exclusive scan over the (descending) bins: two per thread
  const int a = hist[2 * t], b = hist[2 * t + 1];
  int tot;
  const int incl = block_incl_sum(a + b, part, tot);
  __syncthreads();
  hist[2 * t] = incl - (a + b);
  hist[2 * t + 1] = incl - b;
  __syncthreads();
  for (int s = t; s < n; s += 1024)
    order[atomicAdd(&hist[MR_ORDER_BINS - 1 - min(cnt[stile[s]] >> 2, MR_ORDER_BINS - 1)], 1)] = s;
}

template <int KP, bool SIL = false>
static void launch_raster_kr(const FwdParams& P, int64_t slots_cap, hipStream_t st) {
  if (slots_cap >= (1ll << 31)) return;
  MR_TIMED(KID_RASTER_K, st, (k_raster_kp<KP, SIL><<<(unsigned)slots_cap, 64, 0, st>>>(P)));  // one wave per tile
}
// The fused soft silhouette's raster (K <= 64, register lists).
// The heaviest tile lists first: one wave per tile and more tiles than wave slots, so the waves that start
// last set the kernel's tail; started first, the long lists overlap the many short ones (LPT order).
static void slot_order(FwdParams& P, hipStream_t st) {
  if (!MR_KP_ORDER || !P.sorder_ws) return;
  k_slot_order<<<1, 1024, 0, st>>>(P.ctr, P.stile, P.cnt, P.sorder_ws);
  P.sorder = P.sorder_ws;
}
static void launch_raster_sil(FwdParams P, const BinGeom& g, int64_t N, hipStream_t st) {
  slot_order(P, st);
  const int K = P.K;
  const int64_t sc = N * (int64_t)g.T;
  if (K <= 4) launch_raster_kr<4, true>(P, sc, st);
  else if (K <= 8) launch_raster_kr<8, true>(P, sc, st);
  else if (K <= 16) launch_raster_kr<16, true>(P, sc, st);
  else if (K <= 32) launch_raster_kr<32, true>(P, sc, st);
  else if (K <= 50) launch_raster_kr<50, true>(P, sc, st);
  else launch_raster_kr<64, true>(P, sc, st);
}


static int launch_raster_k(FwdParams P, const BinGeom& g, int64_t N, hipStream_t st) {
  static int fgrid = 0;
  if (!fgrid) fgrid = resident_grid(k_fill<0, 3>, 256, 8);
  MR_TIMED(KID_FILL_FRAG, st, (k_fill<0, 3><<<fgrid, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_fill");
  const int K = P.K;
  if (K <= 64) {  // keys in registers (k_raster_kr)
    slot_order(P, st);
    const int64_t sc = N * (int64_t)g.T;
    if (K <= 4) launch_raster_kr<4>(P, sc, st);
    else if (K <= 8) launch_raster_kr<8>(P, sc, st);
    else if (K <= 16) launch_raster_kr<16>(P, sc, st);
    else if (K <= 32) launch_raster_kr<32>(P, sc, st);
    else if (K <= 50) launch_raster_kr<50>(P, sc, st);
    else launch_raster_kr<64>(P, sc, st);
    MR_CHECK_LAUNCH("k_raster_kr");
    return MR_OK;
  }
  const size_t wb = (size_t)K * 64 * 8 + 64 * sizeof(FaceRec) + 64 * sizeof(int);
  const int wpg = wb * 4 <= 65536 ? 4 : wb * 2 <= 65536 ? 2 : 1;
  const int64_t slots_cap = N * (int64_t)g.T;
  const int64_t want = (slots_cap + wpg - 1) / wpg;
  const int grid = (int)(want < 8192 ? want : 8192);
  MR_TIMED(KID_RASTER_K, st, (k_raster_k<<<grid, 64 * wpg, wb * wpg, st>>>(P)));
  MR_CHECK_LAUNCH("k_raster_k");
  return MR_OK;
}
