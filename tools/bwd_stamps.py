"""Per-wave phase cycle sums of k_bwd_fused from an MR_PROF build (s_memtime, core clock).
Build:  hipcc ... -DMR_PROF -o exp/libmi355r_prof.so torch_renderer_amd/csrc/mr_raster.hip
Run:    python tools/bwd_stamps.py   (bench workload: cow, 64 views, 512x512, one fwd+bwd)
Phases per slot iteration: 0 wait for prefetched inputs + pipeline advance; 1 ShadeRec load +
eval_face; 2 shade_fwd (incl. texture taps); 3 shade_bwd; 4 LDS hand-off + ShadeRec corners;
5 raster + projection backward; 6 seg_scatter (+ the R/T store, not stamped separately)."""
import ctypes
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ.setdefault("MI355R_LIB", os.path.join(ROOT, "exp", "libmi355r_prof.so"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from torch_renderer_amd import _lib  # noqa: E402
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.structures import Meshes  # noqa: E402
from torch_renderer_amd.torch_renderer import DepthColorRender  # noqa: E402


def main():
    L = _lib.load()
    L.mr_debug_set_prof.restype = ctypes.c_int32
    L.mr_debug_set_prof.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    m = load_asset("cow", device=dev)
    H = W = 512
    N = 64
    R_cv, t_cv, K = bench.canonical_views(m.shared_verts().cpu(), N, H, W)
    R_cv, t_cv = R_cv.to(dev).requires_grad_(True), t_cv.to(dev).requires_grad_(True)
    v = m.shared_verts().clone().requires_grad_(True)
    mesh = Meshes([v], [m.shared_faces()], m.textures).extend(N)
    r = DepthColorRender(K.to(dev), (H, W), device=dev)
    g = [torch.rand(N, H, W, device=dev), torch.rand(N, H, W, device=dev), torch.rand(N, H, W, 3, device=dev)]
    nw = 1 << 16
    buf = torch.zeros(nw * 8, dtype=torch.int64, device=dev)

    def run():
        torch.autograd.backward(list(r.render(mesh, R_cv, t_cv)), g)

    run()
    torch.cuda.synchronize()
    _lib.check(L.mr_debug_set_prof(buf.data_ptr()))
    run()
    torch.cuda.synchronize()
    _lib.check(L.mr_debug_set_prof(None))
    p = buf.cpu().numpy().view(np.uint64).reshape(nw, 8).astype(np.float64)[32768:]
    act = p[:, 6] > 0
    p = p[act]
    print(f"active waves {act.sum()}, iterations per wave mean {p[:, 6].mean():.2f}")
    tot = p[:, 7].mean()
    names = ["0 wait inputs/advance", "1 ShadeRec+eval_face", "2 shade_fwd", "3 shade_bwd",
             "4 handoff+corners", "5 raster+proj bwd"]
    for i, nm in enumerate(names):
        print(f"  {nm:24s} mean/wave {p[:, i].mean():9.0f} cyc  ({p[:, i].mean() / tot * 100:5.1f}% of wave life)")
    rest = p[:, 7] - p[:, :6].sum(1)
    print(f"  {'6 seg_scatter+rt (rest)':24s} mean/wave {rest.mean():9.0f} cyc  ({rest.mean() / tot * 100:5.1f}%)")
    print(f"  wave lifetime mean {tot:.0f} cyc, max {p[:, 7].max():.0f}")


if __name__ == "__main__":
    main()
