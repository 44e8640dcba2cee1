// mi355r — K = 1 raster: background fills, k_tile_raster (per-tile (z, face) keys), k_shade (covered
// pixels: PyTorch3D fragments or fused shading), persistent-grid sizing and the forward parameters.
// Part of the single translation unit mr_raster.hip (included there, in this order).
#pragma once

// ---------------------------------------------------------------------------
// 2. raster: per-tile depth keys (k_tile_raster), then a streaming resolve (k_resolve)
// ---------------------------------------------------------------------------
// Exact per-(pixel, face) decision and depth: eval_face's return value and pz, without
// the point-triangle distance unless blur > 0 and the pixel is outside. On the fast path
// (blur == 0, FR_FAST) the edge signs reject before any division: a pixel whose edge
// functions do not all carry the area's strict sign has some w_i <= 0, hence c_i <= 0
// (all z > 0), hence is not inside, hence eval_face rejects it too.
// Candidate pixels of one face in one 8x8 tile, as a 64-bit coverage mask (bit 8 * row + col,
// tile-local): the rectangle [rx0, rx1] x [ry0, ry1] (the face's padded bbox clipped to the
// tile), narrowed on the fast path to the columns of each row whose centre can pass the
// edge-sign test. Every pixel frag_keep keeps is in the mask; a few columns within 0.02 px of an
// edge are extra (frag_keep rejects them exactly).
// Edge E_i(p) = (px - ax)(by - ay) - (py - ay)(bx - ax), kept iff s E_i > 0 (s = sign of the
// area). On row py this is linear in px: A (px - ax) > g with A = s dy, g = s dx (py - ay), i.e.
// px > T (A > 0) or px < T (A < 0), T = ax + g / A. Columns run right to left in NDC (tile column
// c of NDC x: c = C0 - x C1), so px > T is c < c(T) and px < T is c > c(T). g is lowered by a
// slack of 2 tol, tol bounding the float rounding of the edge function evaluated in frag_keep
// and of this threshold; a horizontal edge (A = 0) is the limit A -> +0 (all or no columns).
struct TileCols {
  float C0, C1;  // tile column of an NDC x: c = C0 - x * C1
  float omax;    // bound on |NDC| of any pixel centre
};
MR_DEV TileCols tile_cols(int x0, int H, int W) {
  TileCols t;
  t.C1 = W > H ? 0.5f * (float)H : 0.5f * (float)W;
  t.C0 = 0.5f * (float)W - 0.5f - (float)x0;
  t.omax = (float)max(W, H) / (float)min(W, H);
  return t;
}
MR_DEV unsigned long long rect_mask(int rx0, int rx1, int ry0, int ry1) {
  const unsigned long long row = (2ull << rx1) - (1ull << rx0);
  const unsigned long long rows = (0x0101010101010101ull >> (8 * (7 - ry1))) & (~0ull << (8 * ry0));
  return row * rows;
}
MR_DEV unsigned long long tri_mask(const FaceRec& r, const float* ys, int rx0, int rx1, int ry0, int ry1,
                                   const TileCols& tc) {
  const float s = r.area > 0.0f ? 1.0f : -1.0f;
  float Gx[3], K[3], rA[3], ax[3], sC1[3], sC0[3];
  bool up[3];  // A > 0 (or = 0): the edge bounds the columns from above
  const float vx[3] = {r.x0, r.x1, r.x2}, vy[3] = {r.y0, r.y1, r.y2};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int a = (i + 1) % 3, b = (i + 2) % 3;  // E_0 = E(p, v1, v2), E_1 = E(p, v2, v0), E_2 = E(p, v0, v1)
    const float dx = vx[b] - vx[a], dy = vy[b] - vy[a];
    const float A = s * dy;
    const float tol = 1e-6f * (fabsf(dx) + fabsf(dy)) * (tc.omax + fabsf(vx[a]) + fabsf(vy[a]));
    Gx[i] = s * dx;
    K[i] = Gx[i] * vy[a] + 2.0f * tol;  // g - 2 tol = Gx py - K
    up[i] = A >= 0.0f;
    rA[i] = A != 0.0f ? __builtin_amdgcn_rcpf(A) : 1e30f;
    ax[i] = vx[a];
    // sigma c(T) + eps, sigma = +1 (up) / -1: floor of it bounds hi (up) or -lo
    sC1[i] = up[i] ? -tc.C1 : tc.C1;
    sC0[i] = (up[i] ? tc.C0 : -tc.C0) + 0.02f;
  }
  unsigned long long m = 0;
#pragma unroll
  for (int ry = 0; ry < MR_TS; ++ry) {
    if (ry < ry0 || ry > ry1) continue;
    const float py = ys[ry];
    int hi = rx1, lo = rx0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float T = fmaf(fmaf(Gx[i], py, -K[i]), rA[i], ax[i]);
      const float v = __builtin_amdgcn_fmed3f(fmaf(T, sC1[i], sC0[i]), -10.0f, 10.0f);  // NaN -> -10: no column
      const int h = (int)floorf(v);
      if (up[i]) hi = min(hi, h);
      else lo = max(lo, -h);
    }
    if (lo <= hi) m |= ((2ull << hi) - (1ull << lo)) << (8 * ry);
  }
  return m;
}

// The k-th (from 0) set bit of m (k < popcount(m)).
MR_DEV int kth_bit(unsigned long long m, int k) {
  const unsigned lo = (unsigned)m;
  const int clo = __popc(lo);
  const bool hi = k >= clo;
  unsigned x = hi ? (unsigned)(m >> 32) : lo;
  int pos = hi ? 32 : 0;
  k = hi ? k - clo : k;
#pragma unroll
  for (int sh = 16; sh >= 1; sh >>= 1) {
    const int c = __popc(x & ((1u << sh) - 1u));
    const bool go = k >= c;
    x = go ? x >> sh : x;
    k = go ? k - c : k;
    pos = go ? pos + sh : pos;
  }
  return pos;
}

MR_DEV bool frag_keep(const FaceRec& r, float x, float y, float pad, float blur, bool persp, bool clipb,
                      bool fast, float& pz) {
  if (x > r.xmax + pad || x < r.xmin - pad || y > r.ymax + pad || y < r.ymin - pad) return false;
  const float e0 = edge_fn(x, y, r.x1, r.y1, r.x2, r.y2);
  const float e1 = edge_fn(x, y, r.x2, r.y2, r.x0, r.y0);
  const float e2 = edge_fn(x, y, r.x0, r.y0, r.x1, r.y1);
  if (fast) {
    const bool inp = (e0 > 0.0f) & (e1 > 0.0f) & (e2 > 0.0f);
    const bool inn = (e0 < 0.0f) & (e1 < 0.0f) & (e2 < 0.0f);
    if (!(r.area > 0.0f ? inp : inn)) return false;
  }
  const float w0 = e0 / r.area, w1 = e1 / r.area, w2 = e2 / r.area;
  float c0, c1, c2, b0, b1, b2;
  if (persp) persp_fwd(w0, w1, w2, r.z0, r.z1, r.z2, c0, c1, c2);
  else { c0 = w0; c1 = w1; c2 = w2; }
  if (clipb) clip_fwd(c0, c1, c2, b0, b1, b2);
  else { b0 = c0; b1 = c1; b2 = c2; }
  pz = b0 * r.z0 + b1 * r.z1 + b2 * r.z2;
  if (pz < 0.0f) return false;
  const bool inside = c0 > 0.0f && c1 > 0.0f && c2 > 0.0f;
  if (!inside) {
    if (!(blur > 0.0f)) return false;
    if (pt_tri_dist(x, y, r) >= blur) return false;
  }
  return true;
}

// frag_keep split in two for callers that can reject on the depth key first (k_raster_kp): the part
// up to the depth (bbox, edge signs, divisions, pz >= 0), with the inside flag; the caller then keeps
// the fragment iff inside || (blur > 0 && !(pt_tri_dist >= blur)) — frag_keep's decision exactly.
MR_DEV bool frag_depth(const FaceRec& r, float x, float y, float pad, bool persp, bool clipb, bool fast, float& pz,
                       bool& inside) {
  if (x > r.xmax + pad || x < r.xmin - pad || y > r.ymax + pad || y < r.ymin - pad) return false;
  const float e0 = edge_fn(x, y, r.x1, r.y1, r.x2, r.y2);
  const float e1 = edge_fn(x, y, r.x2, r.y2, r.x0, r.y0);
  const float e2 = edge_fn(x, y, r.x0, r.y0, r.x1, r.y1);
  if (fast) {
    const bool inp = (e0 > 0.0f) & (e1 > 0.0f) & (e2 > 0.0f);
    const bool inn = (e0 < 0.0f) & (e1 < 0.0f) & (e2 < 0.0f);
    if (!(r.area > 0.0f ? inp : inn)) return false;
  }
  const float w0 = e0 / r.area, w1 = e1 / r.area, w2 = e2 / r.area;
  float c0, c1, c2, b0, b1, b2;
  if (persp) persp_fwd(w0, w1, w2, r.z0, r.z1, r.z2, c0, c1, c2);
  else { c0 = w0; c1 = w1; c2 = w2; }
  if (clipb) clip_fwd(c0, c1, c2, b0, b1, b2);
  else { b0 = c0; b1 = c1; b2 = c2; }
  pz = b0 * r.z0 + b1 * r.z1 + b2 * r.z2;
  if (pz < 0.0f) return false;
  inside = c0 > 0.0f && c1 > 0.0f && c2 > 0.0f;
  return true;
}

#define MR_NONE 0x7fffffff  // "no face" sentinel, larger than any face code

// Sort code of a record id: upstream's clipped packed order puts the two triangles of a split
// face at consecutive ids in place of the face, so the (z, face) tie order is by (face instance,
// triangle): code = 2 * rid (+1 for the second triangle, record NF + rid). Requires NF < 2^30.
MR_DEV unsigned rec_code(int id, int64_t NF) {
  return id < NF ? 2u * (unsigned)id : 2u * (unsigned)(id - NF) + 1u;
}
MR_DEV int code_rec(unsigned code, int64_t NF) {
  return (code & 1u) ? (int)(NF + (code >> 1)) : (int)(code >> 1);
}
// The original face instance (pix_to_face) of a record id.
MR_DEV int rec_orig(int id, int64_t NF) { return id >= NF ? (int)(id - NF) : id; }

// A split face's two triangles at one pixel (upstream clipped_faces_neighbor_idx rule, for the
// pair as one candidate): if both are kept the second replaces the first iff its distance to the
// pixel is smaller than the first's |signed distance|; else whichever is kept. Returns the record
// id and depth of the candidate.
MR_DEV bool pair_keep(const FaceRec* __restrict__ recs, int64_t NF, int id, const FaceRec& r, float x, float y,
                      float pad, float blur, bool persp, bool clipb, int& cid, float& pz);
// The pixels of one lane's tile rectangle for a split face's triangle (k_tile_raster, rare path;
// out of line so that its registers do not weigh on the pixel-pair loop).
// A wave's staged face records (one per entry lane), structure-of-arrays: field i of record m at
// rec[i][m]. (Measured against 80-B padded array-of-structures records read with ds_read_b128: no gain,
// profiles/r4f_bands_ab.txt.)
struct StageRecs {
  float rec[16][64];
};
MR_DEV void stage_rec_put(StageRecs& S, int lane, const FaceRec& r) {
  const float* f = (const float*)&r;
#pragma unroll
  for (int i = 0; i < 16; ++i) S.rec[i][lane] = f[i];
}
MR_DEV FaceRec stage_rec_get(const StageRecs& S, int m) {
  FaceRec r;
  float* f = (float*)&r;
#pragma unroll
  for (int i = 0; i < 16; ++i) f[i] = S.rec[i][m];
  return r;
}
__attribute__((noinline)) __device__ void raster_pair_rect(const FaceRec* __restrict__ recs, int64_t NF,
                                                           const StageRecs& srec, const int* sid, const float* xs,
                                                           const float* ys, unsigned long long* key, int lane,
                                                           int prect, float pad, float blur, bool persp, bool clipb);
MR_DEV bool pair_keep(const FaceRec* __restrict__ recs, int64_t NF, int id, const FaceRec& r, float x, float y,
                      float pad, float blur, bool persp, bool clipb, int& cid, float& pz) {
  const bool second = id >= NF;
  const int oid = second ? (int)(id - NF) : (int)(id + NF);
  const FaceRec ro = recs[oid];
  const FaceRec& r1 = second ? ro : r;
  const FaceRec& r2 = second ? r : ro;
  const int id1 = second ? oid : id, id2 = second ? id : oid;
  FragEval e1, e2;
  const bool k1 = (r1.flags & FR_VALID) && eval_face(r1, x, y, pad, blur, persp, clipb, e1);
  const bool k2 = (r2.flags & FR_VALID) && eval_face(r2, x, y, pad, blur, persp, clipb, e2);
  if (k1 && k2) {
    const bool use2 = fabsf(e2.sdist) < fabsf(e1.sdist);
    cid = use2 ? id2 : id1;
    pz = use2 ? e2.pz : e1.pz;
    return true;
  }
  if (k1 || k2) {
    cid = k1 ? id1 : id2;
    pz = k1 ? e1.pz : e2.pz;
    return true;
  }
  return false;
}

// (z, face) packed so that unsigned order == frag_less order on the depths that are ever
// kept (pz >= 0; -0 folds onto +0, which the CPU compares equal). The empty key sorts
// after every kept fragment, +inf depth included.
MR_DEV unsigned long long frag_key(float z, int f) {
  const unsigned zb = z == 0.0f ? 0u : __float_as_uint(z);
  return ((unsigned long long)zb << 32) | (unsigned)f;
}

// Everything the forward kernels read and write (geometry, work lists, outputs).
struct FwdParams {
  int N, H, W, TX, T, K;
  float blur, bbox_pad;
  int persp, clipb;
  const int64_t* view_first;  // NULL: shared mode (overflow units scan faces n*F ..)
  int64_t F;                  // faces per view in shared mode (record id = n*F + face)
  int64_t NF;                 // face instances: the second triangle of a split face is record NF + rid
  const ClipRec* crec;        // conversions of clipped records (flag FR_CLIP)
  const FaceRec* recs;
  const int* list;
  const int4* units;
  const int64_t* view_count;  // modular mode: faces per view (overflow tiles scan them all)
  const int* cnt;             // per-tile entries, start inside the view, view bases (K > 1)
  const int* start;
  const int* vbase;
  int64_t list_cap;
  int mfpb;
  int fill;  // k_tile_raster also writes the background
  int emit_frag;  // MODE 0, W % 4 == 0, cnt per tile: k_tile_raster writes each listed tile's 64 fragments
                  // itself and its background chunks skip the listed tiles (no k_shade<0> launch)
  int fill_first;  // ... from this chunk on: the chunks before it were written by k_bin_view<MODE, CH>
  int* ctr;
  unsigned long long* tkey;
  int* tdone;
  int* sface;       // (slots, 64) winning face record per tile pixel or -1
  const int* stile; // (slots) view * T + tile
  // MODE 0 outputs (PyTorch3D Fragments, K = 1)
  int64_t* p2f;
  float* zbuf;
  float* bary;
  float* dists;
  // MODE 1 outputs
  ShadeParams S;
  const ShadeRec* srec;
  int out_flags;
  float* depth;
  float* sil;
  float* rgb;
  int32_t* p2f32;  // optional
  float4* frec;    // MODE 1: the winners' fragments for the backward (slot-major, 64 per slot, tile-pixel order)
  int* sgrp;       // MODE 1: (slots, 64) the winners grouped by record (sort_slot_pixels), for the backward
  uint8_t* sgpix;  // MODE 1: (slots, 64) the tile pixel of each grouped position
  // fused soft silhouette (k_raster_kp<KP, true>): sil = rgba (N,H,W,4); the compact fragments per slot
  float isig;
  int4* sent;
  float4* spix;
  const int* sorder;  // k_raster_kp: workgroup -> slot (k_slot_order), NULL: slot = workgroup
  int* sorder_ws;     // the workspace's order array (RasterWS::sorder)
  int4* units_ws2;    // RasterWS::units2 (k_unit_order's output)
};

// One wave's LDS: the batch of up to 64 entries of its unit and the tile's 64 keys (5.4 KB).
// Face records of the unit's entries, structure-of-arrays: field i of entry m at rec[i][m]. The
// pair passes read the records of up to 64 different entries at once; an array of 64-B records
// put entries 4 apart on the same LDS bank (bank conflicts on every record read), the field
// arrays put distinct entries on distinct banks.
struct WaveStage {
  StageRecs rec;
  int id[64];
  int meta[64];  // index of the entry's first candidate pixel
  int mark[64];  // pass-local: candidate slot -> entry lane that starts there
  unsigned long long key[64];
  unsigned long long cmask[64];  // the entry's candidate pixels (bit 8 * row + col)
  float xs[MR_TS], ys[MR_TS];
};

// Background values of every output (view-independent: a pixel without a face has zero
// blend weight, so depth = relu(-1) = 0, silhouette = 0, rgb = background, alpha = 0).
struct Bg {
  float d, s, c[4];
};
template <int MODE>
MR_DEV Bg background(const FwdParams& P) {
  Bg b;
  b.d = b.s = -1.0f;
  b.c[0] = b.c[1] = b.c[2] = b.c[3] = -1.0f;
  if (MODE == 1) {
    PixGeom G;
    ShadeOut o;
    ShadeCache C;
    shade_fwd(P.S, 0, false, G, 0.f, 0.f, 0.f, 0.f, 0.f, o, C);
    b.d = o.depth;
    b.s = o.sil;
    b.c[0] = o.rgb[0]; b.c[1] = o.rgb[1]; b.c[2] = o.rgb[2]; b.c[3] = o.alpha;
  }
  return b;
}

// Background of one 64-lane chunk of view n: 4 pixels per lane and 16-B vector stores when
// W % 4 == 0 (every row then starts 16-B aligned; PyTorch3D fragments lane-contiguous), else one
// pixel per lane.
template <int MODE, int CH>
MR_DEV void fill_chunk(const FwdParams& P, const Bg& b, int n, int c, bool vec) {
  const int lane = threadIdx.x & 63;
  const int64_t HW = (int64_t)P.H * P.W * (MODE == 0 ? P.K : 1);  // MODE 0: every entry is -1
  if (MODE == 0 && vec) {
    const int64_t q0 = (int64_t)c * 64;  // first quad of the chunk inside the view
    const int nq = (int)min((int64_t)64, HW / 4 - q0);
    if (nq <= 0) return;
    const int64_t pix = (int64_t)n * HW + 4 * q0;
    const float4 m1 = make_float4(-1.f, -1.f, -1.f, -1.f);
    const longlong2 l1 = make_longlong2(-1ll, -1ll);
    fill_words<2>((longlong2*)(P.p2f + pix), nq, lane, l1);
    fill_words<1>((float4*)(P.zbuf + pix), nq, lane, m1);
    fill_words<1>((float4*)(P.dists + pix), nq, lane, m1);
    fill_words<3>((float4*)(P.bary + pix * 3), nq, lane, m1);
  } else if (vec) {
    const int64_t g = (int64_t)c * 64 + lane;
    if (g >= HW / 4) return;
    const int64_t pix = (int64_t)n * HW + 4 * g;
    if (MODE == 0) {
      const float4 m1 = make_float4(-1.f, -1.f, -1.f, -1.f);
      longlong2* q = (longlong2*)(P.p2f + pix);
      q[0] = make_longlong2(-1ll, -1ll);
      q[1] = make_longlong2(-1ll, -1ll);
      *(float4*)(P.zbuf + pix) = m1;
      *(float4*)(P.dists + pix) = m1;
      float4* q3 = (float4*)(P.bary + pix * 3);
      q3[0] = m1; q3[1] = m1; q3[2] = m1;
    } else {
      if (P.out_flags & MR_OUT_DEPTH) *(float4*)(P.depth + pix) = make_float4(b.d, b.d, b.d, b.d);
      if (P.out_flags & MR_OUT_SIL) {
        if (P.out_flags & MR_OUT_SIL_RGBA) {
          float4* q = (float4*)(P.sil + pix * 4);
          const float4 v = make_float4(1.0f, 1.0f, 1.0f, b.s);
          q[0] = v; q[1] = v; q[2] = v; q[3] = v;
        } else {
          *(float4*)(P.sil + pix) = make_float4(b.s, b.s, b.s, b.s);
        }
      }
      if (P.p2f32) *(int4*)(P.p2f32 + pix) = make_int4(-1, -1, -1, -1);
      if (P.out_flags & MR_OUT_RGB) {
        float4* q = (float4*)(P.rgb + pix * CH);
        if (CH == 4) {
          const float4 v = make_float4(b.c[0], b.c[1], b.c[2], b.c[3]);
          q[0] = v; q[1] = v; q[2] = v; q[3] = v;
        } else {
          // 4 pixels x 3 channels = 3 aligned 16-B stores. Opaque copies keep the compiler from
          // re-splitting the period-3 pattern into four unaligned 12-B stores.
          float r0 = b.c[0], g0 = b.c[1], b0 = b.c[2], r1 = r0, g1 = g0, b1 = b0, r2 = r0, g2 = g0, b2 = b0;
          asm volatile("" : "+v"(r1), "+v"(g1), "+v"(b1), "+v"(r2), "+v"(g2), "+v"(b2));
          q[0] = make_float4(r0, g0, b0, r1);
          q[1] = make_float4(g1, b1, r2, g2);
          q[2] = make_float4(b2, r0, g0, b0);
        }
      }
    }
  } else {
    const int64_t i = (int64_t)c * 64 + lane;
    if (i >= HW) return;
    const int64_t q = (int64_t)n * HW + i;
    if (MODE == 0) {
      P.p2f[q] = -1ll;
      P.zbuf[q] = -1.0f;
      P.dists[q] = -1.0f;
      for (int k = 0; k < 3; ++k) P.bary[q * 3 + k] = -1.0f;
    } else {
      if (P.out_flags & MR_OUT_DEPTH) P.depth[q] = b.d;
      if (P.out_flags & MR_OUT_SIL) {
        if (P.out_flags & MR_OUT_SIL_RGBA) *(float4*)(P.sil + q * 4) = make_float4(1.0f, 1.0f, 1.0f, b.s);
        else P.sil[q] = b.s;
      }
      if (P.p2f32) P.p2f32[q] = -1;
      if (P.out_flags & MR_OUT_RGB)
        for (int k = 0; k < CH; ++k) P.rgb[q * CH + k] = b.c[k];
    }
  }
}

// PyTorch3D fragment background of one chunk (view n, 64 pixel quads, W % 4 == 0) outside the
// listed tiles (emit_frag: k_tile_raster writes every pixel of a listed tile when it resolves the
// tile, so neither write can land after the other on the same pixel). A quad never straddles a
// tile (quads start at multiples of 4 pixels, tiles at multiples of 8), and each 16-B word of
// every array belongs to one quad (p2f: 2 words per quad, zbuf / dists: 1, bary: 3).
MR_DEV void fill_frag_unlisted(const FwdParams& P, int n, int c) {
  const int lane = threadIdx.x & 63;
  const int64_t HW = (int64_t)P.H * P.W;
  const int64_t q0 = (int64_t)c * 64;
  const int nq = (int)min((int64_t)64, HW / 4 - q0);
  if (nq <= 0) return;
  bool listed = false;
  if (lane < nq) {
    const int p0 = (int)(4 * q0);  // the chunk's first pixel (uniform: one division per chunk)
    int y = p0 / P.W, x = p0 - y * P.W + 4 * lane;
    while (x >= P.W) {  // (one step at most when W >= 256)
      x -= P.W;
      ++y;
    }
    listed = P.cnt[(int64_t)n * P.T + (y >> 3) * P.TX + (x >> 3)] > 0;
  }
  const unsigned long long lm = __ballot(listed);
  const int64_t pix = (int64_t)n * HW + 4 * q0;
  const float4 m1 = make_float4(-1.f, -1.f, -1.f, -1.f);
  longlong2* p2 = (longlong2*)(P.p2f + pix);
  float4* pz = (float4*)(P.zbuf + pix);
  float4* pd = (float4*)(P.dists + pix);
  float4* pb = (float4*)(P.bary + pix * 3);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int j = k * 64 + lane;
    if (j < 2 * nq && !((lm >> (j >> 1)) & 1ull)) p2[j] = make_longlong2(-1ll, -1ll);
  }
  if (lane < nq && !((lm >> lane) & 1ull)) {
    pz[lane] = m1;
    pd[lane] = m1;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int j = k * 64 + lane;
    if (j < 3 * nq && !((lm >> (j / 3)) & 1ull)) pb[j] = m1;
  }
}

// Persistent grid of independent waves (4 per workgroup, no workgroup barriers): wave g
// takes units g, g + G, ... of the list k_bin_scan emitted (G = resident waves). Per unit:
//  (1) one entry per lane: load its face record, clip the face's padded pixel bbox to the
//      tile (<= 64 pixels);
//  (2) a DPP prefix sum over the rectangle sizes numbers the (face, pixel) pairs, and the
//      wave evaluates 64 pairs per pass exactly (frag_keep), one per lane — a ~3-pixel
//      face costs ~3 lanes, not a wave;
//  (3) kept fragments meet in a per-pixel ds_min_u64 on the packed (z, face) key, which is
//      order-independent and equals the CPU's "strictly nearer, earlier face wins";
//  (4) a tile that is a single unit writes its 64 winners (face record or -1) to its slot
//      of sface straight from LDS; units sharing a tile merge their keys with global u64
//      atomicMin, and the last of them to finish (an atomic count-down) reads the merged
//      keys back with returning atomics and writes the slot.
// The background of every pixel (k_shade later overwrites the covered ones) is written by
// the same waves, a share of 64-lane chunks after each unit: the stores stream to HBM while
// the raster work, which is latency-bound, leaves it idle. (Measured: a separate fill kernel
// on a forked stream overlapping binning was slower in the graph-replayed step, and the
// raster's time barely drops without the fill.) k_fill is the stand-alone version, used
// before k_raster_k (K > 1).
// The fused render's background of one 64-quad chunk with lane-contiguous stores (one 1-KB burst per
// store instruction, as the fragment background): the stand-alone fill of mr_render_reshade. (Inside
// k_tile_raster the per-lane layout of fill_chunk measured faster: its stores interleave with the raster.)
MR_DEV void fill_chunk_render_lc(const FwdParams& P, const Bg& b, int n, int c, int CH) {
  const int lane = threadIdx.x & 63;
  const int64_t HW = (int64_t)P.H * P.W;
  const int64_t q0 = (int64_t)c * 64;
  const int nq = (int)min((int64_t)64, HW / 4 - q0);
  if (nq <= 0) return;
  const int64_t pix = (int64_t)n * HW + 4 * q0;
  if (P.out_flags & MR_OUT_DEPTH) fill_words<1>((float4*)(P.depth + pix), nq, lane, make_float4(b.d, b.d, b.d, b.d));
  if (P.out_flags & MR_OUT_SIL) {
    if (P.out_flags & MR_OUT_SIL_RGBA) fill_words<4>((float4*)(P.sil + pix * 4), nq, lane, make_float4(1.0f, 1.0f, 1.0f, b.s));
    else fill_words<1>((float4*)(P.sil + pix), nq, lane, make_float4(b.s, b.s, b.s, b.s));
  }
  if (P.p2f32) fill_words<1>((int4*)(P.p2f32 + pix), nq, lane, make_int4(-1, -1, -1, -1));
  if (P.out_flags & MR_OUT_RGB) {
    float4* q = (float4*)(P.rgb + pix * CH);
    if (CH == 4) {
      fill_words<4>(q, nq, lane, make_float4(b.c[0], b.c[1], b.c[2], b.c[3]));
    } else {  // period-3 pattern: word j of the chunk holds channels (4 j .. 4 j + 3) mod 3
      const float4 w0 = make_float4(b.c[0], b.c[1], b.c[2], b.c[0]);
      const float4 w1 = make_float4(b.c[1], b.c[2], b.c[0], b.c[1]);
      const float4 w2 = make_float4(b.c[2], b.c[0], b.c[1], b.c[2]);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int j = k * 64 + lane;
        if (j < 3 * nq) q[j] = (j % 3) == 0 ? w0 : (j % 3) == 1 ? w1 : w2;
      }
    }
  }
}

template <int MODE, int CH>
__global__ void __launch_bounds__(256) k_fill(FwdParams P) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), G = gridDim.x * 4;
  const bool vec = (P.W & 3) == 0;
  const int64_t HW = (int64_t)P.H * P.W * (MODE == 0 ? P.K : 1);
  const int cpv = (int)(vec ? (HW / 4 + 63) / 64 : (HW + 63) / 64);
  const int nchunks = P.N * cpv;
  const Bg bg = background<MODE>(P);
#pragma unroll 1
  for (int c = gw; c < nchunks; c += G) {
    if (MODE == 1 && vec) fill_chunk_render_lc(P, bg, c / cpv, c - (c / cpv) * cpv, CH);
    else fill_chunk<MODE, CH>(P, bg, c / cpv, c - (c / cpv) * cpv, vec);
  }
}


// The per-view binning with background workgroups: one 1024-thread workgroup per view leaves
// most CUs idle, so workgroups past the views (and the ShadeRec ones) stream the background of
// the first F.fill_first chunks (view-major) while the views bin; k_tile_raster writes the rest.
// The background does not depend on the raster (k_shade overwrites the covered pixels later).
// Experiment builds only (-DMR_XP_BV_STAMP, tools/binview_stamps.py): per workgroup of the last launch, the
// global clock when its first wave starts and when its last wave ends, its role (0 binning, 1 ShadeRec,
// 2 background) and a binning workgroup's phase ends (BV_PH). Reads of the clock counters only; vector stores.
#ifdef MR_XP_BV_STAMP
#define MR_XP_BV_WGS 4096
__device__ unsigned long long g_bv_stamp[MR_XP_BV_WGS * 8];
#endif
template <int MODE, int CH>
__global__ void __launch_bounds__(1024) k_bin_view(ViewBinParams P, FwdParams F) {
#ifdef MR_XP_BV_STAMP
  const unsigned long long xp_t0 = __builtin_amdgcn_s_memrealtime();
  const int xp_role = (int)blockIdx.x < P.nviews * P.bands ? 0 : (int)blockIdx.x < P.nviews * P.bands + P.nsrec_wg ? 1 : 2;
  struct XpEnd {
    unsigned long long t0;
    int role;
    __device__ ~XpEnd() {
      __syncthreads();
      const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
      const int i = (int)threadIdx.x;
      if (blockIdx.x < MR_XP_BV_WGS && i < 8)
        g_bv_stamp[(size_t)blockIdx.x * 8 + i] = i == 0 ? t0 : i == 1 ? t1 : i == 2 ? (unsigned long long)role
                                               : role == 0 ? g_bv_ph[i - 3] : 0ull;
    }
  } xp_end{xp_t0, xp_role};
#endif
  const int b = (int)blockIdx.x - P.nviews * P.bands - P.nsrec_wg;
  if (b < 0) {
    bin_view_body(P);
    return;
  }
  const int nbw = ((int)gridDim.x - P.nviews * P.bands - P.nsrec_wg) * 16;  // background waves
  const bool vec = (F.W & 3) == 0;
  const int64_t HW = (int64_t)F.H * F.W * (MODE == 0 ? F.K : 1);
  const int cpv = (int)(vec ? (HW / 4 + 63) / 64 : (HW + 63) / 64);
  const Bg bg = background<MODE>(F);
  const int c0 = b * 16 + (int)(threadIdx.x >> 6);
  const int gn = nbw / cpv, gc = nbw - gn * cpv;
  int cn = c0 / cpv, cc = c0 - cn * cpv;
#pragma unroll 1
  for (int c = c0; c < F.fill_first; c += nbw) {
    fill_chunk<MODE, CH>(F, bg, cn, cc, vec);
    cn += gn;
    cc += gc;
    if (cc >= cpv) { cc -= cpv; ++cn; }
  }
}

__attribute__((noinline)) __device__ void raster_pair_rect(const FaceRec* __restrict__ recs, int64_t NF,
                                                           const StageRecs& srec, const int* sid, const float* xs,
                                                           const float* ys, unsigned long long* key, int lane,
                                                           int prect, float pad, float blur, bool persp, bool clipb) {
  const FaceRec r = stage_rec_get(srec, lane);
  const int id = sid[lane];
  for (int yy = (prect >> 6) & 7; yy <= ((prect >> 9) & 7); ++yy)
    for (int xx = prect & 7; xx <= ((prect >> 3) & 7); ++xx) {
      float pz;
      int cid;
      if (pair_keep(recs, NF, id, r, xs[xx], ys[yy], pad, blur, persp, clipb, cid, pz))
        atomicMin(&key[yy * MR_TS + xx], frag_key(pz, (int)rec_code(cid, NF)));
    }
}

// CLIP: near-plane clipping on (split faces may be present); the CLIP = false instantiation
// carries none of their code, so the common launch keeps its register budget.
#ifndef MR_TR_BGFIRST_FRAG
#define MR_TR_BGFIRST_FRAG 4
#endif
#ifndef MR_RASTER_WAVES
#define MR_RASTER_WAVES 4  // waves / SIMD: 5 -> <= 96 VGPRs, 4 -> <= 128
#endif
template <int MODE, int CH, bool CLIP>
__global__ void __launch_bounds__(256, MR_RASTER_WAVES) k_tile_raster(FwdParams P) {
  __shared__ WaveStage stage[4];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  WaveStage& S = stage[wave];
  const int nunits = P.ctr[CTR_UNITS];
  const float pad = P.bbox_pad, blur = P.blur;
  const bool persp = P.persp != 0, clipb = P.clipb != 0;
  const bool fast_ok = !(blur > 0.0f);
  const int H = P.H, W = P.W;
  // background chunks of this wave: c = gw, gw + G, ... < N * cpv, written after its units (the
  // waves that finish their raster work early stream the background while the others still run;
  // chunks interleaved with the units measured 3 us slower, all chunks before them 20 us slower)
  const int gw = blockIdx.x * 4 + wave, G = gridDim.x * 4;
  const bool vec = (W & 3) == 0;
  const int64_t HW = (int64_t)H * W * (MODE == 0 ? P.K : 1);
  const int cpv = (int)(vec ? (HW / 4 + 63) / 64 : (HW + 63) / 64);
  const int nchunks = P.fill ? P.N * cpv : 0;
  // XCD-aware unit partition: workgroups are dispatched round-robin over the 8 XCDs, so
  // blockIdx % 8 names this wave's XCD; each XCD's waves take a contiguous eighth of the
  // (view-major) units, which keeps the face records they gather in that XCD's L2.
  const int parts = (gridDim.x & 7) == 0 ? 8 : 1;
  const int jw = (blockIdx.x / parts) * 4 + wave, Gp = (gridDim.x / parts) * 4;
  const int Cp = (nunits + parts - 1) / parts;
  const int ub = (blockIdx.x % parts) * Cp, ue = ub + Cp < nunits ? ub + Cp : nunits;
  const Bg bg = background<MODE>(P);
  int chunk = P.fill_first + gw;
  // the wave's background chunks c = chunk, chunk + G, ... (view, chunk) stepped incrementally: no
  // integer division per chunk
  auto background_chunks = [&]() {
    const int gn = G / cpv, gc = G - gn * cpv;
    int cn = chunk / cpv, cc = chunk - cn * cpv;
    if (MODE == 0 && P.emit_frag) {
#pragma unroll 1
      for (; chunk < nchunks; chunk += G) {
        fill_frag_unlisted(P, cn, cc);
        cn += gn;
        cc += gc;
        if (cc >= cpv) { cc -= cpv; ++cn; }
      }
    } else {
#pragma unroll 1
      for (; chunk < nchunks; chunk += G) {
        fill_chunk<MODE, CH>(P, bg, cn, cc, vec);
        cn += gn;
        cc += gc;
        if (cc >= cpv) { cc -= cpv; ++cn; }
      }
    }
  };
  // Fragments (K = 1): one wave in MR_TR_BGFIRST_FRAG (alternating over workgroups, so each SIMD holds
  // both kinds) streams its background first, overlapping the other waves' latency-bound raster
  // (alone: units 59 us, background 53 us, together 92; one in 4 first: 89, one in 2: 94 — the
  // fused render loses 2-3 % with either, profiles/r4y_bgfirst_ab.txt)
  if (MODE == 0 && MR_TR_BGFIRST_FRAG > 0 &&
      (blockIdx.x + wave) % (MR_TR_BGFIRST_FRAG > 0 ? MR_TR_BGFIRST_FRAG : 1) == 0)
    background_chunks();
  // Software pipeline over the wave's units u, u + Gp, u + 2Gp, ...: while unit u is
  // rasterised, the face records of u + Gp, the list entries of u + 2Gp and the unit record of
  // u + 3Gp are in flight (unit records are wave-uniform scalar loads). Each link of the
  // unit -> list entry -> record chain so gets a whole unit of work to land in, and a unit
  // starts with its records in registers. (Overflow units fetch their records in the batch.)
  // The prefetches are unconditional loads of clamped (valid) indices whose results are only
  // used when the unit / entry exists (guarded loads become branches whose phi copies wait on
  // the load at once), and the unit records travel as per-lane copies made uniform where they
  // are consumed (a uniform load is otherwise scalarised: load + readfirstlane + wait at issue).
  const int lz = lane_zero();
  const int ulast = max(ue - 1, 0);
  int4 U1v = P.units[min(ub + jw, ulast) + lz];
  int4 U2v = P.units[min(ub + jw + Gp, ulast) + lz];
  int4 U3v = P.units[min(ub + jw + 2 * Gp, ulast) + lz];
  int id1 = P.list[(ub + jw < ue && U1v.y >= 0 && lane < U1v.z) ? U1v.y + lane : 0];
  int id2 = P.list[(ub + jw + Gp < ue && U2v.y >= 0 && lane < U2v.z) ? U2v.y + lane : 0];
  FaceRec r1 = load_rec(P.recs, (ub + jw < ue && U1v.y >= 0 && lane < U1v.z) ? id1 : 0);
#pragma unroll 1
  for (int u = ub + jw; u < ue; u += Gp) {
    const int4 U = make_int4(__builtin_amdgcn_readfirstlane(U1v.x), __builtin_amdgcn_readfirstlane(U1v.y),
                             __builtin_amdgcn_readfirstlane(U1v.z), __builtin_amdgcn_readfirstlane(U1v.w));
    const int id0 = id1;
    const int n = U.x / P.T, t = U.x - n * P.T;
    const int ty = t / P.TX, tx = t - ty * P.TX;
    const int x0 = tx * MR_TS, y0 = ty * MR_TS;
    const TileCols tc = tile_cols(x0, H, W);
    if (lane < MR_TS) S.xs[lane] = col_ndc(x0 + lane < W ? x0 + lane : W - 1, H, W);
    else if (lane < 2 * MR_TS) S.ys[lane - MR_TS] = row_ndc(y0 + lane - MR_TS < H ? y0 + lane - MR_TS : H - 1, H, W);
    S.key[lane] = MR_KEY_EMPTY;
    S.mark[lane] = -1;
    const bool ovf = U.y < 0;
    wave_lds_sync();
#pragma unroll 1
    for (int eb = 0; eb < U.z; eb += 64) {
      const int e = eb + lane;
      int prect = 0;
      unsigned long long cmask = 0;
      if (e < U.z) {
        int id;
        FaceRec r;
        if (ovf) {  // (the view's first record loaded here: a load hoisted to the unit's start is waited on there)
          const int64_t vfirst = P.view_first ? P.view_first[n] : (int64_t)n * P.F;
          id = (int)(vfirst + e);
          r = P.recs[id];
        } else {  // a listed unit has <= 64 entries: its records are already here
          id = id0;
          r = r1;
        }
        // pixel rectangle: the record's padded bbox; an overflow unit scans only first triangles
        // of split faces, so there it covers both triangles of the pair
        float bx0 = r.xmin, bx1 = r.xmax, by0 = r.ymin, by1 = r.ymax;
        bool bvalid = (r.flags & FR_VALID) != 0;
        if (CLIP && ovf && (r.flags & FR_PAIR)) {
          const FaceRec ro = P.recs[P.NF + id];
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
        cx0 = cx0 > x0 ? cx0 : x0;
        cx1 = cx1 < x0 + MR_TS - 1 ? cx1 : x0 + MR_TS - 1;
        cy0 = cy0 > y0 ? cy0 : y0;
        cy1 = cy1 < y0 + MR_TS - 1 ? cy1 : y0 + MR_TS - 1;
        if (bvalid && cx0 <= cx1 && cy0 <= cy1) {
          if (CLIP && (r.flags & FR_PAIR)) {  // a split face's triangle: its own per-lane loop after the passes
            prect = 0x1000 | (cx0 - x0) | ((cx1 - x0) << 3) | ((cy0 - y0) << 6) | ((cy1 - y0) << 9);
          } else {
            const int rx0 = cx0 - x0, rx1 = cx1 - x0, ry0 = cy0 - y0, ry1 = cy1 - y0;
            // coverage rows from the edges (fast path; coordinates small enough that the
            // threshold arithmetic stays finite), else the whole rectangle
            const bool tm = fast_ok && (r.flags & FR_FAST) &&
                            fmaxf(fmaxf(fabsf(r.xmin), fabsf(r.xmax)), fmaxf(fabsf(r.ymin), fabsf(r.ymax))) < 1e12f;
            cmask = tm ? tri_mask(r, S.ys, rx0, rx1, ry0, ry1, tc) : rect_mask(rx0, rx1, ry0, ry1);
          }
        }
        stage_rec_put(S.rec, lane, r);
        S.id[lane] = id;
      }
      if (eb == 0) {  // advance the pipeline (after this unit's records are consumed)
        r1 = load_rec(P.recs, (u + Gp < ue && U2v.y >= 0 && lane < U2v.z) ? id2 : 0);
        id1 = id2;
        U1v = U2v;
        id2 = P.list[(u + 2 * Gp < ue && U3v.y >= 0 && lane < U3v.z) ? U3v.y + lane : 0];
        U2v = U3v;
        U3v = P.units[min(u + 3 * Gp, ulast) + lz];
      }
      // candidate numbering: a DPP prefix sum over the masks' popcounts
      const int np = __popcll(cmask);
      const int pincl = wave_incl_sum(np);
      const int pexcl = pincl - np;
      const int NP = __builtin_amdgcn_readlane(pincl, 63);
      S.meta[lane] = pexcl;
      S.cmask[lane] = cmask;
      // 64 candidates per pass, one per lane, each evaluated exactly (frag_keep: bbox, edge
      // signs, divisions, perspective correction, depth) and merged into the tile's keys
#pragma unroll 1
      for (int pb = 0; pb < NP; pb += 64) {
        wave_lds_sync();
        // the entry starting inside this pass marks its first slot; slot 0 belongs to the
        // entry straddling pb (the last non-empty entry starting at or before it)
        if (np > 0 && pexcl > pb && pexcl < pb + 64) S.mark[pexcl - pb] = lane;
        const unsigned long long own = __ballot(np > 0 && pexcl <= pb);
        const int straddle = 63 - __builtin_clzll(own);
        wave_lds_sync();
        int m = S.mark[lane];
        S.mark[lane] = -1;
        if (lane == 0) m = straddle;
        m = wave_incl_max(m);
        const int q = pb + lane;
        if (q < NP) {
          const int p = kth_bit(S.cmask[m], q - S.meta[m]);
          const int sx = p & 7, sy = p >> 3;
          const FaceRec r = stage_rec_get(S.rec, m);
          float pz;
          if (frag_keep(r, S.xs[sx], S.ys[sy], pad, blur, persp, clipb, fast_ok && (r.flags & FR_FAST), pz))
            atomicMin(&S.key[p], frag_key(pz, CLIP ? (int)rec_code(S.id[m], P.NF) : 2 * S.id[m]));
        }
      }
      if (CLIP && __builtin_expect(__ballot(prect != 0) != 0ull, 0)) {
        // near-plane split faces (rare): each such lane walks its rectangle, resolving the pair
        if (prect) raster_pair_rect(P.recs, P.NF, S.rec, S.id, S.xs, S.ys, S.key, lane, prect, pad, blur, persp, clipb);
      }
      wave_lds_sync();  // the stage is rewritten by the next batch
    }
    unsigned long long k = S.key[lane];
    const int slot = U.w & 0x7fffffff;
    bool emit = true;
    if (U.w < 0) {  // tile shared by several units
      unsigned long long* dst = P.tkey + (int64_t)slot * 64 + lane;
      // Device-scope atomics are performed at the memory side (never cached in an XCD's L2),
      // so agent atomics on both sides hand the keys over: this wave's 64 atomicMin are
      // acknowledged (vmcnt) before its count-down, and the last unit reads the merged keys
      // with returning atomics issued after it observed the count-down reach it.
      atomicMin(dst, k);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int left = 0;
      if (lane == 0) left = __hip_atomic_fetch_add(&P.tdone[slot], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      left = __builtin_amdgcn_readfirstlane(left);
      emit = left == 0;  // the last unit of the tile
      if (emit) k = atomicMin(dst, MR_KEY_EMPTY);
    }
    if (emit) {
      const unsigned code = (unsigned)(k & 0xffffffffull);
      const int px = x0 + (lane & 7), py = y0 + (lane >> 3);
      const bool hit = code != MR_NONE && px < W && py < H;
      const int rid = hit ? (CLIP ? code_rec(code, P.NF) : (int)(code >> 1)) : -1;
      if (MODE == 0 && P.emit_frag) {
        // the tile's fragments (k_shade<0>'s work): the winner's exact evaluation, or the background
        if (px < W && py < H) {
          const int64_t q = (int64_t)n * H * W + (int64_t)py * W + px;
          int64_t f = -1;
          float z = -1.0f, d = -1.0f, b0 = -1.0f, b1 = -1.0f, b2 = -1.0f;
          if (hit) {
            const FaceRec r = load_rec(P.recs, rid);
            FragEval ev;
            eval_face(r, S.xs[lane & 7], S.ys[lane >> 3], pad, blur, persp, clipb, ev);  // kept by construction
            if (r.flags & FR_CLIP) clip_unconvert(P.crec[rid], ev.b0, ev.b1, ev.b2, ev.b0, ev.b1, ev.b2);
            f = rec_orig(rid, P.NF); z = ev.pz; d = ev.sdist; b0 = ev.b0; b1 = ev.b1; b2 = ev.b2;
          }
          P.p2f[q] = f;
          P.zbuf[q] = z;
          P.dists[q] = d;
          P.bary[3 * q + 0] = b0;
          P.bary[3 * q + 1] = b1;
          P.bary[3 * q + 2] = b2;
        }
      } else {
        P.sface[(int64_t)slot * 64 + lane] = rid;
      }
    }
    wave_lds_sync();
  }
  background_chunks();
}

// Per-face shading records of the shared mesh (one thread per face).
__global__ void __launch_bounds__(256) k_shade_rec(ShadeParams S, int64_t F, ShadeRec* __restrict__ out) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  ShadeRec R;
  make_shade_rec(S, (uint32_t)f, R);
  out[f] = R;
}

MR_DEV void vertex_normal(const float* __restrict__ verts, const int32_t* __restrict__ faces,
                          const int32_t* __restrict__ ptr, const int32_t* __restrict__ adj, int64_t v,
                          float* __restrict__ vn, float* __restrict__ vraw);

// The fused forward's first kernel: blocks [0, vb) compute the vertex normals (one thread per
// vertex, as k_vertex_normals; vb = 0 when the caller passed them), the rest zero `nzero` ints
// (per-tile counts, view totals, work counters) with coalesced stores — one launch instead of a
// normals launch + a memset. The ShadeRecs, which need the normals, are packed by extra blocks
// of the binning fill launch (k_bin_fill_world row N).
__global__ void __launch_bounds__(256) k_setup_zero(const float* __restrict__ verts, int64_t V,
                                                    const int32_t* __restrict__ faces, const int32_t* __restrict__ ptr,
                                                    const int32_t* __restrict__ adj, float* __restrict__ vn,
                                                    float* __restrict__ vraw, int64_t vb, int* __restrict__ zero,
                                                    int64_t nzero) {
  if ((int64_t)blockIdx.x < vb) {
    const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v < V) vertex_normal(verts, faces, ptr, adj, v, vn, vraw);
    return;
  }
  const int64_t base = ((int64_t)blockIdx.x - vb) * 1024;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    if (i < nzero) zero[i] = 0;
  }
}

// XCD-aware slot ranges: workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8
// names the XCD), so each XCD takes a contiguous eighth of the (view-major, tile-ordered) slots
// and its waves stride inside it. Horizontally / vertically adjacent tiles then run on the same
// XCD at about the same time and share that XCD's L2 lines (the 128-B lines of the per-pixel
// upstream gradients and outputs span two 8-pixel tile rows; a face record serves neighbouring
// tiles). Returns the wave's first slot, its stride and the range end.
MR_DEV void xcd_slot_range(int nslots, int wave, int& s0, int& step, int& end) {
  const int parts = (gridDim.x & 7) == 0 ? 8 : 1;
  const int per = (nslots + parts - 1) / parts;
  const int x = blockIdx.x % parts;
  const int b = x * per;
  end = b + per < nslots ? b + per : nslots;
  s0 = b + (int)(blockIdx.x / parts) * 4 + wave;
  step = (int)(gridDim.x / parts) * 4;
}

// Order the 64 pixels of a slot by winning record (groups in order of first appearance, pixels of a
// group in tile order): each (tile, record) then forms ONE run of consecutive lanes of the backward, so the per-face
// rows of a tile come out of one segmented scan, one row per (tile, record) — 13.5 instead of 28.7
// runs per tile on the bench workload — and can be written with plain stores. The loop runs once
// per distinct record of the tile (uniform, scalar bookkeeping). Returns the tile pixel this lane
// takes; f becomes that pixel's record.
MR_DEV int sort_slot_pixels(int& f, int lane, int* lperm) {
  unsigned long long rem = ~0ull;
  int pos = 0, base = 0;
  while (rem) {
    const int l = (int)__builtin_ctzll(rem);
    const int key = __builtin_amdgcn_readlane(f, l);
    const unsigned long long m = __ballot(f == key);
    const int below = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
    pos = f == key ? base + below : pos;
    base += __popcll(m);
    rem &= ~m;
  }
  lperm[pos] = lane;
  wave_lds_sync();
  const int src = lperm[lane];
  f = __builtin_amdgcn_ds_bpermute(src << 2, f);
  wave_lds_sync();  // lperm is rewritten for the next slot
  return src;
}

// Covered pixels: waves stride over the non-empty tiles' slots, one tile pixel per lane:
// recompute the winning fragment exactly, then write PyTorch3D fragments (M = 0) or shade
// (M = 1) over the background k_tile_raster wrote.
// MODE 1 (the fused render) also groups each slot's pixels by winning record (sort_slot_pixels) and
// writes the grouping (sgrp, sgpix) beside the fragments (frec, tile-pixel order): the backward then reads
// its lanes' pixels pre-grouped instead of sorting every slot again (round 5 sorted in k_bwd_fused).
template <int MODE, int CH>
__global__ void __launch_bounds__(256) k_shade(FwdParams P) {
  __shared__ int lperm[MODE == 1 ? 4 : 1][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nslots = P.ctr[CTR_SLOTS];
  if (nslots <= 0) return;  // no covered tile: the prefetches below would read unwritten winners
  const int64_t HW = (int64_t)P.H * P.W;
  int s0, G, send;
  xcd_slot_range(nslots, wave, s0, G, send);
  // Two-deep pipeline: while slot s is processed, the winners' face records of slot s + G and
  // the tile and winners of slot s + 2G are in flight (unconditional loads of clamped indices;
  // the tile id as a per-lane copy made uniform at use — see k_bwd_fused).
  const int lz = lane_zero();
  const int slast = max(nslots - 1, 0);
  int sc = min(s0, slast);
  int gt_c = P.stile[sc + lz], f_c = P.sface[(int64_t)sc * 64 + lane];
  sc = min(s0 + G, slast);
  int gt_n = P.stile[sc + lz], f_n = P.sface[(int64_t)sc * 64 + lane];
  // lane -> tile pixel p_c (MODE 1: grouped by record; the record prefetch follows the grouped order)
  int p_c = MODE == 1 ? sort_slot_pixels(f_c, lane, lperm[wave]) : lane;
  FaceRec r_c = load_rec(P.recs, f_c < 0 ? 0 : f_c);
  for (int s = s0; s < send; s += G) {
    const int gt = __builtin_amdgcn_readfirstlane(gt_c);
    const int f = f_c, p = p_c;
    const FaceRec r = r_c;
    gt_c = gt_n;
    f_c = f_n;
    if (MODE == 1) p_c = sort_slot_pixels(f_c, lane, lperm[wave]);
    r_c = load_rec(P.recs, f_c < 0 ? 0 : f_c);
    sc = min(s + 2 * G, slast);
    gt_n = P.stile[sc + lz];
    f_n = P.sface[(int64_t)sc * 64 + lane];
    if (MODE == 1) {
      P.sgrp[(int64_t)s * 64 + lane] = f;
      P.sgpix[(int64_t)s * 64 + lane] = (uint8_t)p;
    }
    if (f < 0) continue;
    const int n = gt / P.T, t = gt - n * P.T;
    const int ty = t / P.TX, tx = t - ty * P.TX;
    const int px = tx * MR_TS + (p & 7), py = ty * MR_TS + (p >> 3);
    const int64_t q = n * HW + (int64_t)py * P.W + px;
    const int fo = rec_orig(f, P.NF);  // the original face instance
    PixGeom G;
    if (MODE == 1) load_geom(P.srec, (uint32_t)(fo - n * P.F), G);  // in parallel with the record
    FragEval ev;
    const bool hit = eval_face(r, col_ndc(px, P.H, P.W), row_ndc(py, P.H, P.W), P.bbox_pad, P.blur, P.persp,
                               P.clipb, ev);  // true by construction (same test that kept it)
    if (!hit) continue;
    if (r.flags & FR_CLIP) {  // near-plane sub-triangle: barycentrics of the original face
      const ClipRec cr = P.crec[f];
      clip_unconvert(cr, ev.b0, ev.b1, ev.b2, ev.b0, ev.b1, ev.b2);
    }
    if (MODE == 0) {
      P.p2f[q] = (int64_t)fo;
      P.zbuf[q] = ev.pz;
      P.dists[q] = ev.sdist;
      P.bary[3 * q + 0] = ev.b0;
      P.bary[3 * q + 1] = ev.b1;
      P.bary[3 * q + 2] = ev.b2;
    } else {
      // the fragment the backward shades again (its barycentrics must be these bits: they pick the
      // texel cell), so k_bwd_fused does not re-run eval_face's IEEE divisions
      P.frec[(int64_t)s * 64 + p] = make_float4(ev.b0, ev.b1, ev.b2, ev.sdist);  // (tile-pixel order)
      ShadeOut o;
      ShadeCache C;
      shade_fwd(P.S, n, true, G, ev.b0, ev.b1, ev.b2, ev.pz, ev.sdist, o, C);
      if (P.out_flags & MR_OUT_DEPTH) P.depth[q] = o.depth;
      if (P.out_flags & MR_OUT_SIL) {
        if (P.out_flags & MR_OUT_SIL_RGBA) *(float4*)(P.sil + q * 4) = make_float4(1.0f, 1.0f, 1.0f, o.sil);
        else P.sil[q] = o.sil;
      }
      if (P.out_flags & MR_OUT_RGB) {
        P.rgb[q * CH + 0] = o.rgb[0];
        P.rgb[q * CH + 1] = o.rgb[1];
        P.rgb[q * CH + 2] = o.rgb[2];
        if (CH == 4) P.rgb[q * CH + 3] = o.alpha;
      }
      if (P.p2f32) P.p2f32[q] = fo;
    }
  }
}

// The fused render's covered pixels (k_shade<1>'s work, one kernel of its own): group each slot's pixels by
// record (sgrp, sgpix for the backward), recompute the winner's fragment (frec), shade, write depth / silhouette /
// RGB. Each slot's stores are deferred into the next slot's iteration, after that slot's ShadeRec loads: a
// load's wait (vmcnt, in-order retirement) includes every store issued before it, so storing at the end of the
// iteration put the previous slot's ~1 KB of writes in front of each ShadeRec wait. SPEC 1: the shading's runtime
// switches as compile-time constants (UV map with an 8-bit copy, point light), outputs depth + silhouette + RGB.
template <int CH, int SPEC>
__global__ void __launch_bounds__(256) k_shade_render(FwdParams P) {
  __shared__ int lperm[4][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nslots = P.ctr[CTR_SLOTS];
  if (nslots <= 0) return;
  const int64_t HW = (int64_t)P.H * P.W;
  int s0, G, send;
  xcd_slot_range(nslots, wave, s0, G, send);
  const int lz = lane_zero();
  const int slast = max(nslots - 1, 0);
  int sc = min(s0, slast);
  int gt_c = P.stile[sc + lz], f_c = P.sface[(int64_t)sc * 64 + lane];
  sc = min(s0 + G, slast);
  int gt_n = P.stile[sc + lz], f_n = P.sface[(int64_t)sc * 64 + lane];
  int p_c = sort_slot_pixels(f_c, lane, lperm[wave]);
  FaceRec r_c = load_rec(P.recs, f_c < 0 ? 0 : f_c);
  const int of = SPEC ? (MR_OUT_DEPTH | MR_OUT_SIL | MR_OUT_RGB) : P.out_flags;
  // the previous slot's outputs, stored in this iteration
  int s_prev = -1, f_prev = -1, p_prev = 0, fo_prev = 0;
  bool w_prev = false;  // this lane covered a pixel of the previous slot
  int64_t q_prev = 0;
  float4 fr_prev = make_float4(0.f, 0.f, 0.f, 0.f);
  ShadeOut o_prev;
  o_prev.depth = o_prev.sil = o_prev.alpha = 0.f;
  o_prev.rgb[0] = o_prev.rgb[1] = o_prev.rgb[2] = 0.f;
  auto store_prev = [&]() {
    if (s_prev < 0) return;
    P.sgrp[(int64_t)s_prev * 64 + lane] = f_prev;
    P.sgpix[(int64_t)s_prev * 64 + lane] = (uint8_t)p_prev;
    if (w_prev) {
      P.frec[(int64_t)s_prev * 64 + p_prev] = fr_prev;  // (tile-pixel order)
      if (of & MR_OUT_DEPTH) P.depth[q_prev] = o_prev.depth;
      if (of & MR_OUT_SIL) {
        if (!SPEC && (of & MR_OUT_SIL_RGBA)) *(float4*)(P.sil + q_prev * 4) = make_float4(1.0f, 1.0f, 1.0f, o_prev.sil);
        else P.sil[q_prev] = o_prev.sil;
      }
      if (of & MR_OUT_RGB) {
        P.rgb[q_prev * CH + 0] = o_prev.rgb[0];
        P.rgb[q_prev * CH + 1] = o_prev.rgb[1];
        P.rgb[q_prev * CH + 2] = o_prev.rgb[2];
        if (CH == 4) P.rgb[q_prev * CH + 3] = o_prev.alpha;
      }
      if (!SPEC && P.p2f32) P.p2f32[q_prev] = fo_prev;
    }
  };
  for (int s = s0; s < send; s += G) {
    const int gt = __builtin_amdgcn_readfirstlane(gt_c);
    const int f = f_c, p = p_c;
    const FaceRec r = r_c;
    const int n = gt / P.T, t = gt - n * P.T;
    const int ty = t / P.TX, tx = t - ty * P.TX;
    const int px = tx * MR_TS + (p & 7), py = ty * MR_TS + (p >> 3);
    const int64_t q = n * HW + (int64_t)py * P.W + px;
    const int fo = f >= 0 ? (int)rec_orig(f, P.NF) : 0;  // the original face instance
    PixGeom Gm;
    load_geom(P.srec, f >= 0 ? (uint32_t)(fo - n * P.F) : 0u, Gm);  // first: its wait follows no store
    gt_c = gt_n;
    f_c = f_n;
    p_c = sort_slot_pixels(f_c, lane, lperm[wave]);
    r_c = load_rec(P.recs, f_c < 0 ? 0 : f_c);
    sc = min(s + 2 * G, slast);
    gt_n = P.stile[sc + lz];
    f_n = P.sface[(int64_t)sc * 64 + lane];
    store_prev();
    FragEval ev;
    const bool hit = f >= 0 && eval_face(r, col_ndc(px, P.H, P.W), row_ndc(py, P.H, P.W), P.bbox_pad, P.blur,
                                         P.persp, P.clipb, ev);  // true by construction when f >= 0
    ShadeOut o;
    o.depth = o.sil = o.alpha = 0.f;
    o.rgb[0] = o.rgb[1] = o.rgb[2] = 0.f;
    if (hit) {
      if (r.flags & FR_CLIP) {  // near-plane sub-triangle: barycentrics of the original face
        const ClipRec cr = P.crec[f];
        clip_unconvert(cr, ev.b0, ev.b1, ev.b2, ev.b0, ev.b1, ev.b2);
      }
      ShadeCache C;
      shade_fwd<SPEC>(P.S, n, true, Gm, ev.b0, ev.b1, ev.b2, ev.pz, ev.sdist, o, C);
    }
    s_prev = s;
    f_prev = f;
    p_prev = p;
    w_prev = hit;
    q_prev = q;
    fo_prev = fo;
    fr_prev = make_float4(ev.b0, ev.b1, ev.b2, ev.sdist);
    o_prev = o;
  }
  store_prev();
}

// Resident workgroups of a kernel on the current device (persistent grid size).
template <typename K>
static int resident_grid(K kernel, int threads, int fallback_per_cu) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0) != hipSuccess || per <= 0)
    per = fallback_per_cu;
  return cus * per;
}

// Static forward parameters from the settings; the workspace pointers from the carve.
static FwdParams make_fwd(const mr_raster_settings_t* s, const BinGeom& g, const RasterWS& w, int64_t N,
                          const int64_t* view_first, int64_t F, int64_t NF) {
  FwdParams P;
  memset(&P, 0, sizeof(P));
  P.N = (int)N; P.H = s->H; P.W = s->W; P.TX = g.TX; P.T = g.T; P.K = s->faces_per_pixel;
  P.blur = s->blur_radius;
  P.bbox_pad = sqrtf(s->blur_radius);
  P.persp = s->perspective_correct;
  P.clipb = s->clip_barycentric_coords;
  P.view_first = view_first; P.F = F; P.NF = NF; P.crec = w.crec;
  P.recs = w.recs; P.list = w.list; P.units = w.units; P.ctr = w.ctr; P.tkey = w.tkey;
  P.cnt = w.cnt; P.start = w.start; P.vbase = w.vbase; P.list_cap = g.list_cap; P.mfpb = g.mfpb;
  P.tdone = w.tdone; P.sface = w.sface; P.stile = w.stile;
  P.frec = w.frec;
  P.sgrp = w.sgrp;
  P.sgpix = w.sgpix;
  P.sorder_ws = w.sorder;
  P.units_ws2 = w.units2;
  return P;
}


// The raster's work units, heaviest first inside each of the 8 XCD ranges k_tile_raster partitions them into
// (its waves take units round-robin from their range, so a descending order deals every wave about the same
// load instead of leaving the slowest wave's random share to set the kernel's end; LPT order). Key: an
// overflow unit (every face of the view) first, then by entries, 64 down to 1; order inside a key arbitrary
// (the raster's result does not depend on the order its units run in). One workgroup per range.
#ifndef MR_UNIT_ORDER
#define MR_UNIT_ORDER 1
#endif
#ifndef MR_UNIT_ORDER_MIN_VIEWS
#define MR_UNIT_ORDER_MIN_VIEWS 16
#endif
MR_DEV int unit_key(const int4& U) { return U.y < 0 ? 0 : MR_UE + 1 - min(max(U.z, 1), MR_UE); }
__global__ void __launch_bounds__(1024) k_unit_order(const int4* __restrict__ units, const int* __restrict__ ctr,
                                                     int4* __restrict__ out) {
  __shared__ int hist[128];
  const int t = threadIdx.x, n = ctr[CTR_UNITS];
  const int per = (n + 7) / 8, b = (int)blockIdx.x * per, e = min(b + per, n);
  if (t < 128) hist[t] = 0;
  __syncthreads();
  for (int u = b + t; u < e; u += 1024) atomicAdd(&hist[unit_key(units[u])], 1);
  __syncthreads();
  if (t < 64) {  // exclusive scan of the 128 keys, two per lane, from the range's start
    const int x = hist[2 * t], y = hist[2 * t + 1];
    const int incl = wave_incl_sum(x + y);
    hist[2 * t] = b + incl - (x + y);
    hist[2 * t + 1] = b + incl - y;
  }
  __syncthreads();
  for (int u = b + t; u < e; u += 1024) {
    const int4 U = units[u];
    out[atomicAdd(&hist[unit_key(U)], 1)] = U;
  }
}

#ifndef MR_SHADE_RENDER
#define MR_SHADE_RENDER 1
#endif
// k_shade_render (the fused render's covered pixels), specialised when the shading and outputs are the drop-in
// Phong render's: UV map with an 8-bit copy, point light, depth + silhouette + RGB, no pix_to_face.
template <int CH>
static int launch_shade_render(const FwdParams& P, int64_t slots_cap, hipStream_t st) {
  static int g0 = 0, g1 = 0;
  if (!g0) g0 = resident_grid(k_shade_render<CH, 0>, 256, 4);
  if (!g1) g1 = resident_grid(k_shade_render<CH, 1>, 256, 4);
  const bool spec = CH == 3 && P.S.tex_kind == 2 && P.S.tex8 && P.S.light_kind == 0 && !P.S.zbuf_mode &&
                    !P.p2f32 && P.out_flags == (MR_OUT_DEPTH | MR_OUT_SIL | MR_OUT_RGB);
  const int gr = spec ? g1 : g0;
  int sg = (int)(slots_cap / 4 + 1 < gr ? slots_cap / 4 + 1 : gr);
  sg = (sg + 7) / 8 * 8;  // XCD-partitioned slot ranges
  if (spec) MR_TIMED(KID_SHADE_RENDER, st, (k_shade_render<CH, 1><<<sg, 256, 0, st>>>(P)));
  else MR_TIMED(KID_SHADE_RENDER, st, (k_shade_render<CH, 0><<<sg, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_shade_render");
  return MR_OK;
}

// Raster (+ background) then covered-pixel outputs; grids sized once per kernel instance.
template <int MODE, int CH>
static int launch_raster_and_shade(FwdParams P, const BinGeom& g, int64_t N, hipStream_t st, bool clip) {
  P.fill = 1;
  static int rgrid = 0, rgrid_c = 0, sgrid = 0;
  if (!rgrid) rgrid = resident_grid(k_tile_raster<MODE, CH, false>, 256, 7);
  if (!rgrid_c) rgrid_c = resident_grid(k_tile_raster<MODE, CH, true>, 256, 7);
  if (!sgrid) sgrid = resident_grid(k_shade<MODE, CH>, 256, 6);
  // (the fused render only: in the fragment pass the raster's time is its background stores, and the order's
  // launch cost more than it saved — fragments 421k -> 405-416k, render 300k -> 301-302k, profiles/r5_unit_order_ab.txt;
  // and only for batches of MR_UNIT_ORDER_MIN_VIEWS views or more: C5's single view rasters 0.3 us slower without it
  // and saves the 4.4-us launch, profiles/r6n_c5_ab.txt)
  if (MR_UNIT_ORDER && MODE == 1 && P.units_ws2 && N >= MR_UNIT_ORDER_MIN_VIEWS) {
    MR_TIMED(KID_UNIT_ORDER, st, (k_unit_order<<<8, 1024, 0, st>>>(P.units, P.ctr, P.units_ws2)));
    MR_CHECK_LAUNCH("k_unit_order");
    P.units = P.units_ws2;
  }
  if (clip) MR_TIMED(KID_TILE_RASTER, st, (k_tile_raster<MODE, CH, true><<<rgrid_c, 256, 0, st>>>(P)));
  else MR_TIMED(KID_TILE_RASTER, st, (k_tile_raster<MODE, CH, false><<<rgrid, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_tile_raster");
  if (MODE == 0 && P.emit_frag) return MR_OK;  // the raster wrote the listed tiles' fragments
  const int64_t slots_cap = N * (int64_t)g.T;
  if (MODE == 1 && MR_SHADE_RENDER) return launch_shade_render<CH>(P, slots_cap, st);
  int sg = (int)(slots_cap / 4 + 1 < sgrid ? slots_cap / 4 + 1 : sgrid);
  sg = (sg + 7) / 8 * 8;  // XCD-partitioned slot ranges
  MR_TIMED(MODE == 0 ? KID_SHADE_FRAG : KID_SHADE_RENDER, st, (k_shade<MODE, CH><<<sg, 256, 0, st>>>(P)));
  MR_CHECK_LAUNCH("k_shade");
  return MR_OK;
}
