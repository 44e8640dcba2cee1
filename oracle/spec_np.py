"""ORACLE — test infrastructure only.

Float64 NumPy restatement of the rasterizer forward, written
independently of oracle/raster_cpu.c, used to cross-check the C oracle on small
images: pix_to_face must agree wherever the float64 depth gap between the best two
candidates is not within float32 noise, and zbuf/bary/dists agree to ~1e-5.

Follows PyTorch3D RasterizeMeshesNaiveCpu: PixToNonSquareNdc pixel centres, bbox
reject, zero-area skip (|E(v0,v1,v2)| <= 1e-8), barycentrics E/(E(v2,v0,v1)+1e-8),
perspective correction, pz < 0 skip, inside = all bary > 0, blur test on the squared
point-triangle distance, K nearest by (z, face).
"""
from __future__ import annotations

import numpy as np

EPS = 1e-8


def pix_to_ndc(i, S1, S2):
    rng = 2.0 * S1 / S2 if S1 > S2 else 2.0
    off = rng / 2.0
    return -off + (rng * i + off) / S1


def _edge(p, a, b):
    return (p[..., 0] - a[0]) * (b[1] - a[1]) - (p[..., 1] - a[1]) * (b[0] - a[0])


def _seg_dist2(p, a, b):
    ab = b - a
    l2 = ab @ ab
    if l2 <= EPS:
        d = p - b
        return (d * d).sum(-1)
    t = np.clip(((p - a) @ ab) / l2, 0.0, 1.0)
    q = a + t[..., None] * ab
    d = p - q
    return (d * d).sum(-1)


def rasterize(face_verts, first, count, H, W, K=1, blur=0.0, persp=True):
    fv = np.asarray(face_verts, dtype=np.float64)
    N = len(first)
    p2f = -np.ones((N, H, W, K), np.int64)
    zbuf = -np.ones((N, H, W, K))
    bary = -np.ones((N, H, W, K, 3))
    dists = -np.ones((N, H, W, K))
    gap = np.full((N, H, W), np.inf)  # depth gap between the best two candidates (tie detector)
    ys = np.array([pix_to_ndc(H - 1 - yi, H, W) for yi in range(H)])
    xs = np.array([pix_to_ndc(W - 1 - xi, W, H) for xi in range(W)])
    P = np.stack(np.meshgrid(xs, ys), -1)  # (H,W,2): [...,0]=x, [...,1]=y
    pad = np.sqrt(blur)
    for n in range(N):
        cand_z = [[[] for _ in range(W)] for _ in range(H)]
        for f in range(int(first[n]), int(first[n] + count[n])):
            v = fv[f]
            v0, v1, v2 = v[0, :2], v[1, :2], v[2, :2]
            z = v[:, 2]
            area_f = _edge(v0, v1, v2)
            if abs(area_f) <= EPS or z.max() < 0:
                continue
            lo, hi = v[:, :2].min(0) - pad, v[:, :2].max(0) + pad
            m = (P[..., 0] >= lo[0]) & (P[..., 0] <= hi[0]) & (P[..., 1] >= lo[1]) & (P[..., 1] <= hi[1])
            if not m.any():
                continue
            area = _edge(v2, v0, v1) + EPS
            w = np.stack([_edge(P, v1, v2), _edge(P, v2, v0), _edge(P, v0, v1)], -1) / area
            if persp:
                top = np.stack([w[..., 0] * z[1] * z[2], w[..., 1] * z[0] * z[2], w[..., 2] * z[0] * z[1]], -1)
                w = top / np.maximum(top.sum(-1, keepdims=True), EPS)
            pz = (w * z).sum(-1)
            inside = (w > 0).all(-1)
            d2 = np.minimum(np.minimum(_seg_dist2(P, v0, v1), _seg_dist2(P, v0, v2)), _seg_dist2(P, v1, v2))
            keep = m & (pz >= 0) & (inside | (d2 < blur))
            for yi, xi in zip(*np.nonzero(keep)):
                cand_z[yi][xi].append((pz[yi, xi], f, -d2[yi, xi] if inside[yi, xi] else d2[yi, xi],
                                       w[yi, xi]))
        for yi in range(H):
            for xi in range(W):
                c = sorted(cand_z[yi][xi], key=lambda t: (t[0], t[1]))
                if len(c) >= 2:
                    gap[n, yi, xi] = c[1][0] - c[0][0]
                for k, (zz, f, d, w) in enumerate(c[:K]):
                    p2f[n, yi, xi, k] = f
                    zbuf[n, yi, xi, k] = zz
                    dists[n, yi, xi, k] = d
                    bary[n, yi, xi, k] = w
    return p2f, zbuf, bary, dists, gap
