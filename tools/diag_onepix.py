#!/usr/bin/env python3
"""Diagnostic (GPU): one pixel's contribution to one vertex's gradient, per output channel (depth,
silhouette, rgb), GPU fused backward vs oracle f32 vs its float64 shadow (metric workload views 0, 37).
    python tools/diag_onepix.py VERTEX VIEW Y X"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tests.test_gpu_configs as C  # noqa: E402
from tests.helpers import canonical_views, mesh_arrays  # noqa: E402
from torch_renderer_amd import TexturesUV, TexturesVertex  # noqa: E402


def main():
    V, n, y, x = (int(a) for a in sys.argv[1:5])
    verts, faces, d = mesh_arrays("cow")
    img, vuv, fuv = C._uv_texture(d)
    H = W = 512
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, 64, H, W, dist=0.5)
    sel = [0, 37]
    R_cv, t_cv = R_cv[sel], t_cv[sel]
    for texmode in ("uv", "white"):
        if texmode == "uv":
            tex = TexturesUV(maps=[img.to(C.DEV)], faces_uvs=[fuv.to(C.DEV)], verts_uvs=[vuv.to(C.DEV)])
            otex = ("uv", vuv, fuv, img)
        else:
            tex = TexturesVertex([torch.ones_like(verts).to(C.DEV)])
            otex = ("vertex", torch.ones_like(verts))
        gD, gS, gC = C._upstream(2, H, W)
        m = torch.zeros(2, H, W)
        m[n, y, x] = 1.0
        z = torch.zeros(2, H, W)
        win = (max(y - 2, 0), min(y + 3, H), max(x - 2, 0), min(x + 3, W))
        for nm, g in (("depth", (gD * m, z, z[..., None] * gC)), ("sil", (z, gS * m, z[..., None] * gC)),
                      ("rgb", (z, z, gC * m[..., None])), ("rgb-r", (z, z, gC * m[..., None] * torch.tensor([1., 0, 0]))),
                      ("rgb-g", (z, z, gC * m[..., None] * torch.tensor([0, 1., 0]))),
                      ("rgb-b", (z, z, gC * m[..., None] * torch.tensor([0, 0, 1.])))):
            _, gg = C._gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, g, want_p2f=False)
            _, r32 = C._oracle_views(verts, faces, R_cv, t_cv, K, H, W, otex, g, window=win)
            _, r64 = C._oracle_views(verts, faces, R_cv, t_cv, K, H, W, otex, g, window=win, precision="f64")
            print(f"[one] {texmode} {nm}: gpu {gg[0][V].cpu().tolist()} f32 {r32[0][V].tolist()} "
                  f"f64 {r64[0][V].tolist()}", flush=True)


if __name__ == "__main__":
    main()
