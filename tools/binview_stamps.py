"""Phase stamps of k_bin_view (MR_PROF build: python tools/build_variant.py prof -DMR_PROF; run
with MI355R_LIB=exp/prof.so) on the bench workload: per-workgroup s_memtime deltas."""
import ctypes
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from torch_renderer_amd import _lib, kernels as Kn  # noqa: E402
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.torch_renderer import texture_args  # noqa: E402
from torch_renderer_amd.transforms import opencv_to_pytorch3d  # noqa: E402


def main():
    L = _lib.load()
    L.mr_debug_set_prof.restype = ctypes.c_int32
    L.mr_debug_set_prof.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    mesh = sys.argv[1] if len(sys.argv) > 1 else "cow"
    H = W = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    m = load_asset(mesh, device=dev)
    v, f = m.shared_verts(), m.shared_faces()
    N = 64
    R_cv, t_cv, K = bench.canonical_views(v.cpu(), N, H, W, dist_m=bench.view_distance(mesh, v.cpu()))
    R, T = opencv_to_pytorch3d(R_cv, t_cv)
    s = min(H, W) / 2.0
    intr = torch.tensor([[K[0, 0] / s, 0.0, K[1, 1] / s, 0.0]]).expand(N, 4).contiguous().to(dev)
    R, T = R.to(dev), T.to(dev)
    tex, _ = texture_args(m, True) if m.textures is not None else (None, None)
    cfg = Kn.ShadeConfig(H=H, W=W)
    buf = torch.zeros(65536 * 8, dtype=torch.int64, device=dev)
    if len(sys.argv) > 3 and sys.argv[3] == "frag":  # the fragment pass (mr_rasterize_meshes_world)
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
    p = buf.cpu().numpy().view(np.uint64).reshape(-1, 8).astype(np.float64)[60000:60000 + N]
    p = p[p[:, 7] == 1]
    t0 = p[:, 0].min()
    print(f"workgroups {len(p)}; start spread {p[:, 0].max() - t0:.0f}; end {p[:, 5].max() - t0:.0f}")
    for i, nm in enumerate(["count", "scan", "atomics", "units", "fill"]):
        d = p[:, i + 1] - p[:, i]
        print(f"  {nm:8s} mean={d.mean():.0f} p50={np.percentile(d, 50):.0f} max={d.max():.0f}")


if __name__ == "__main__":
    main()
