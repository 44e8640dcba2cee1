"""Per-wave phase stamps of k_render_bwd from an MR_PROF build (s_memtime, core clock).
Build:  hipcc ... -DMR_PROF -o torch_renderer_amd/libmi355r_prof.so torch_renderer_amd/csrc/mr_raster.hip
Run:    python tools/phase_stamps.py  (bench workload: cow, 64 views, 512x512)"""
import ctypes
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ.setdefault("MI355R_LIB", os.path.join(ROOT, "torch_renderer_amd", "libmi355r_prof.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from torch_renderer_amd import _lib, kernels as Kn  # noqa: E402
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.torch_renderer import texture_args  # noqa: E402
from torch_renderer_amd.transforms import opencv_to_pytorch3d  # noqa: E402


def st(x):
    x = np.asarray(x, dtype=np.float64)
    return "n=0" if x.size == 0 else f"n={x.size} mean={x.mean():.0f} p50={np.percentile(x, 50):.0f} p90={np.percentile(x, 90):.0f} max={x.max():.0f}"


def main():
    L = _lib.load()
    L.mr_debug_set_prof.restype = ctypes.c_int32
    L.mr_debug_set_prof.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    m = load_asset("cow", device=dev)
    v, f = m.shared_verts(), m.shared_faces()
    H = W = 512
    N = 64
    R_cv, t_cv, K = bench.canonical_views(v.cpu(), N, H, W)
    R, T = opencv_to_pytorch3d(R_cv, t_cv)
    s = min(H, W) / 2.0
    intr = torch.tensor([[K[0, 0] / s, 0.0, K[1, 1] / s, 0.0]]).expand(N, 4).contiguous().to(dev)
    R, T = R.to(dev), T.to(dev)
    tex, _ = texture_args(m, True)
    cfg = Kn.ShadeConfig(H=H, W=W)
    vg = v.clone().requires_grad_(True)
    g = [torch.rand(N, H, W, device=dev), torch.rand(N, H, W, device=dev), torch.rand(N, H, W, 3, device=dev)]
    nw = 1 << 16
    buf = torch.zeros(nw * 8, dtype=torch.int64, device=dev)

    def run():
        out = Kn.render_views(vg, R, T, f, intr, torch.zeros(1, 3, device=dev), cfg, tex)
        torch.autograd.backward([out["depth"], out["sil"], out["rgb"]], g)

    run()
    torch.cuda.synchronize()
    _lib.check(L.mr_debug_set_prof(buf.data_ptr()))
    run()
    torch.cuda.synchronize()
    _lib.check(L.mr_debug_set_prof(None))
    p = buf.cpu().numpy().view(np.uint64).reshape(nw, 8).astype(np.float64)
    act = (p[:, 0] > 0) & (p[:, 1] > 0)
    p = p[act]
    print(f"active waves {act.sum()}")
    t0 = p[:, 0].min()
    print("start (cycles from first):", st(p[:, 0] - t0))
    print("end   (cycles from first):", st(p[:, 7] - t0))
    names = ["loads issued(0-1)", "eval+shade_fwd(1-2)", "shade_bwd(2-3)", "raster_bwd(3-4)", "project+rows(4-5)",
             "seg_scatter(5-6)", "rt_reduce(6-7)", "total(0-7)"]
    idx = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 7), (0, 7)]
    for nm, (i, j) in zip(names, idx):
        d = p[:, j] - p[:, i]
        print(f"  {nm:22s}", st(d[(p[:, j] > 0) & (p[:, i] > 0)]))


if __name__ == "__main__":
    main()
