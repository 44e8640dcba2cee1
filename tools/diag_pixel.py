#!/usr/bin/env python3
"""Diagnostic (GPU): find the pixels whose contribution to one vertex's gradient differs between the
fused GPU backward and the oracle (metric workload views 0 and 37, cow 512x512, UV texture).

For the faces around vertex V: every covered pixel of those faces gets its own run with the upstream
gradient of (depth, silhouette, rgb) kept at that pixel only; the GPU and oracle vertex gradients of V
are compared. Prints the pixels whose contributions differ by more than 1e-5.

    python tools/diag_pixel.py VERTEX [max_pixels]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tests.test_gpu_configs as C  # noqa: E402
from tests.helpers import canonical_views, mesh_arrays  # noqa: E402
from torch_renderer_amd import TexturesUV  # noqa: E402


def main():
    V = int(sys.argv[1])
    maxp = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    verts, faces, d = mesh_arrays("cow")
    img, vuv, fuv = C._uv_texture(d)
    H = W = 512
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, 64, H, W, dist=0.5)
    sel = [0, 37]
    R_cv, t_cv = R_cv[sel], t_cv[sel]
    tex = TexturesUV(maps=[img.to(C.DEV)], faces_uvs=[fuv.to(C.DEV)], verts_uvs=[vuv.to(C.DEV)])
    otex = ("uv", vuv, fuv, img)
    gD, gS, gC = C._upstream(2, H, W)
    out, _ = C._gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, None)
    p2f = out["pix_to_face32"].cpu().long()
    Fn = faces.shape[0]
    adj = set(int(f) for f in (faces == V).any(1).nonzero()[:, 0])
    local = torch.where(p2f >= 0, p2f % Fn, p2f)
    mask = torch.zeros_like(local, dtype=torch.bool)
    for f in adj:
        mask |= local == f
    pix = mask.nonzero()
    # pixels next to those (the silhouette's soft edge reaches neighbours of covered pixels)
    print(f"[pix] vertex {V}: faces {sorted(adj)}, {pix.shape[0]} covered pixels", flush=True)
    rows = []
    for k, (n, y, x) in enumerate(pix.tolist()[:maxp]):
        m = torch.zeros(2, H, W)
        m[n, y, x] = 1.0
        g = (gD * m, gS * m, gC * m[..., None])
        _, gg = C._gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, g, want_p2f=False)
        win = (max(y - 2, 0), min(y + 3, H), max(x - 2, 0), min(x + 3, W))
        _, r32 = C._oracle_views(verts, faces, R_cv, t_cv, K, H, W, otex, g, window=win)
        a, b = gg[0][V].cpu(), r32[0][V]
        dd = (a - b).abs().max().item()
        rows.append((dd, n, y, x, int(local[n, y, x]), a.tolist(), b.tolist()))
        if dd > 1e-5:
            print(f"[pix] view {n} y {y} x {x} face {int(local[n, y, x])}: gpu {a.tolist()} oracle {b.tolist()} "
                  f"diff {dd:.3e}", flush=True)
    rows.sort(reverse=True)
    print("[pix] top:", [(f"{r[0]:.2e}", r[1], r[2], r[3], r[4]) for r in rows[:8]], flush=True)


if __name__ == "__main__":
    main()
