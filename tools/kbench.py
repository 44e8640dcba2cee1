"""Per-kernel timing of the raster/render kernels on the bench workload (HIP events via
the library's timing hooks). python tools/kbench.py [--views 64 --size 512 --mesh cow --iters 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from torch_renderer_amd import _lib, kernels as Kn  # noqa: E402
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.transforms import opencv_to_pytorch3d  # noqa: E402
from torch_renderer_amd.torch_renderer import texture_args  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=64)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--mesh", default="cow")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dist", type=float, default=0.5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    m = load_asset(a.mesh, device=dev)
    v, f = m.shared_verts(), m.shared_faces()
    H = W = a.size
    R_cv, t_cv, K = bench.canonical_views(v.cpu(), a.views, H, W, dist_m=a.dist)
    R, T = opencv_to_pytorch3d(R_cv, t_cv)
    s = min(H, W) / 2.0
    intr = torch.tensor([[K[0, 0] / s, 0.0, K[1, 1] / s, 0.0]]).expand(a.views, 4).contiguous().to(dev)
    R, T = R.to(dev), T.to(dev)
    fv = Kn.ProjectFaces.apply(v, R, T, f, intr)
    Fn = f.shape[0]
    first = torch.arange(a.views, device=dev) * Fn
    count = torch.full((a.views,), Fn, device=dev)
    tex, vcol = texture_args(m, True)
    cfg = Kn.ShadeConfig(H=H, W=W, want_p2f=True)
    vg = v.clone().requires_grad_(True)
    gD = torch.rand(a.views, H, W, device=dev)
    gS = torch.rand(a.views, H, W, device=dev)
    gC = torch.rand(a.views, H, W, 3, device=dev)

    def run():
        Kn.rasterize_meshes_fwd(fv, first, count, H, W)
        out = Kn.render_views(vg, R, T, f, intr, torch.zeros(1, 3, device=dev), cfg, tex)
        torch.autograd.backward([out["depth"], out["sil"], out["rgb"]], [gD, gS, gC])
        return out

    out = run()
    torch.cuda.synchronize()
    cov = (out["pix_to_face32"] >= 0).float().mean().item()
    _lib.timing_enable(True)
    for _ in range(a.iters):
        run()
    torch.cuda.synchronize()
    kt = _lib.timing_read()
    _lib.timing_enable(False)
    res = {k: round(t / n * 1e3, 2) for k, (n, t) in kt.items()}
    print(json.dumps({"mesh": a.mesh, "views": a.views, "size": H, "coverage": round(cov, 4), "avg_us": res}))


if __name__ == "__main__":
    main()
