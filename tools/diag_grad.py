#!/usr/bin/env python3
"""Diagnostic (GPU): which output's gradient path carries the GPU's vertex-gradient deviation from
the oracle on the metric workload (cow, 512x512, views 0 and 37)? Runs the fused render backward with
only the depth, only the silhouette and only the RGB upstream gradient, and compares each with the
f32 oracle and its float64 shadow. Prints the worst entries."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import tests.test_gpu_configs as C  # noqa: E402
from tests.helpers import canonical_views, mesh_arrays  # noqa: E402
from torch_renderer_amd import TexturesUV, TexturesVertex  # noqa: E402


def main():
    verts, faces, d = mesh_arrays("cow")
    img, vuv, fuv = C._uv_texture(d)
    H = W = 512
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, 64, H, W, dist=0.5)
    sel = [0, 37]
    R_cv, t_cv = R_cv[sel], t_cv[sel]
    gD, gS, gC = C._upstream(2, H, W)
    z = (torch.zeros_like(gD), torch.zeros_like(gS), torch.zeros_like(gC))
    texmode = sys.argv[1] if len(sys.argv) > 1 else "uv"
    if texmode == "uv":
        tex = TexturesUV(maps=[img.to(C.DEV)], faces_uvs=[fuv.to(C.DEV)], verts_uvs=[vuv.to(C.DEV)])
        otex = ("uv", vuv, fuv, img)
    else:
        tex = TexturesVertex([torch.ones_like(verts).to(C.DEV)])
        otex = ("vertex", torch.ones_like(verts))
    for nm, grads in (("depth", (gD, z[1], z[2])), ("sil", (z[0], gS, z[2])), ("rgb", (z[0], z[1], gC))):
        _, gg = C._gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, grads)
        _, r32 = C._oracle_views(verts, faces, R_cv, t_cv, K, H, W, otex, grads)
        _, r64 = C._oracle_views(verts, faces, R_cv, t_cv, K, H, W, otex, grads, precision="f64")
        for k, lab in enumerate(("verts", "R_cv", "t_cv")):
            g = gg[k].cpu().double()
            a, b = r32[k].double(), r64[k].double()
            bar = 1e-4 * b.abs().clamp(min=1.0)
            eg, eo = (g - b).abs() / bar, (a - b).abs() / bar
            i = int(eg.reshape(-1).argmax())
            print(f"[diag] {texmode} {nm}-only grad {lab}: GPU vs f64 worst {eg.max():.2f} bar (oracle f32 vs f64 worst "
                  f"{eo.max():.2f}); #GPU>1 bar {int((eg > 1).sum())}, #oracle>1 bar {int((eo > 1).sum())}; worst at "
                  f"{tuple(int(x) for x in torch.unravel_index(torch.tensor(i), g.shape))}: gpu {g.reshape(-1)[i]:.6e} "
                  f"f32 {a.reshape(-1)[i]:.6e} f64 {b.reshape(-1)[i]:.6e}", flush=True)


if __name__ == "__main__":
    main()
