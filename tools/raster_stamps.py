"""Per-wave phase cycles of k_tile_raster from an MR_PROF build (s_memtime deltas summed over
the wave's units). Build the prof library as in tools/phase_stamps.py, then run this on a GPU."""
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
    return "n=0" if x.size == 0 else f"mean={x.mean():.0f} p50={np.percentile(x, 50):.0f} p90={np.percentile(x, 90):.0f} max={x.max():.0f} sum={x.sum():.3g}"


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
    nw = 1 << 16
    buf = torch.zeros(nw * 8, dtype=torch.int64, device=dev)
    if len(sys.argv) > 1 and sys.argv[1] == "frag":  # the fragment pass (mr_rasterize_meshes_world)
        run = lambda: Kn.RasterizeMeshesWorld.apply(v, R.contiguous(), T.contiguous(), f, intr, N, H, W, 1, 0.0,  # noqa: E731
                                                    True, False, False, None)
    else:
        run = lambda: Kn.render_views(v, R, T, f, intr, torch.zeros(1, 3, device=dev), cfg, tex)  # noqa: E731
    run()
    torch.cuda.synchronize()
    _lib.check(L.mr_debug_set_prof(buf.data_ptr()))
    run()
    torch.cuda.synchronize()
    _lib.check(L.mr_debug_set_prof(None))
    p = buf.cpu().numpy().view(np.uint64).reshape(nw, 8).astype(np.float64)
    p = p[p[:, 7] == 1]
    print(f"waves {len(p)}; units/wave {st(p[:, 5] % 65536)}; passes/wave {st(p[:, 5] // 65536)}")
    for i, nm in enumerate(["load", "cheap", "emit", "fill", "exact", "", "total"]):
        if nm:
            print(f"  {nm:8s} cycles/wave {st(p[:, i])}")


if __name__ == "__main__":
    main()
