"""Phase timing inside k_raster from an MR_PROF build (per-wave s_memtime stamps).
Build: hipcc ... -DMR_PROF -o torch_renderer_amd/libmi355r_prof.so torch_renderer_amd/csrc/mr_raster.hip
Run:   python tools/raster_phases.py [--mode 1 --views 64 --size 512 --dist 0.5]"""
import argparse
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


def stats(x):
    x = np.asarray(x, dtype=np.float64)
    if x.size == 0:
        return "n=0"
    return (f"n={x.size} mean={x.mean():.0f} p50={np.percentile(x, 50):.0f} p90={np.percentile(x, 90):.0f} "
            f"max={x.max():.0f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--views", type=int, default=64)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--dist", type=float, default=0.5)
    ap.add_argument("--mesh", default="cow")
    a = ap.parse_args()
    L = _lib.load()
    L.mr_debug_set_prof.restype = ctypes.c_int32
    L.mr_debug_set_prof.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    m = load_asset(a.mesh, device=dev)
    v, f = m.shared_verts(), m.shared_faces()
    H = W = a.size
    N = a.views
    R_cv, t_cv, K = bench.canonical_views(v.cpu(), N, H, W, dist_m=a.dist)
    R, T = opencv_to_pytorch3d(R_cv, t_cv)
    s = min(H, W) / 2.0
    intr = torch.tensor([[K[0, 0] / s, 0.0, K[1, 1] / s, 0.0]]).expand(N, 4).contiguous().to(dev)
    R, T = R.to(dev), T.to(dev)
    TX, TY = (W + 7) // 8, (H + 7) // 8
    GX = (TX + 7) // 8
    nwg = N * TY * GX
    buf = torch.zeros(nwg * 8 * 16, dtype=torch.int64, device=dev)
    tex, _ = texture_args(m, True)
    cfg = Kn.ShadeConfig(H=H, W=W)

    def run():
        if a.mode == 1:
            Kn.render_views(v, R, T, f, intr, torch.zeros(1, 3, device=dev), cfg, tex)
        else:
            fv = Kn.ProjectFaces.apply(v, R, T, f, intr)
            Fn = f.shape[0]
            Kn.rasterize_meshes_fwd(fv, torch.arange(N, device=dev) * Fn, torch.full((N,), Fn, device=dev), H, W)

    run()
    torch.cuda.synchronize()
    _lib.check(L.mr_debug_set_prof(buf.data_ptr()))
    run()
    torch.cuda.synchronize()
    _lib.check(L.mr_debug_set_prof(None))
    p = buf.cpu().numpy().view(np.uint64).reshape(nwg, 8, 16).astype(np.float64)
    p = p[p[:, 0, 0] > 0]  # strips k_raster visited (background strips are written by k_bg)
    t0 = p[:, :, 0]
    ne = p[:, 0, 2] > 0
    E = (p[:, 0, 7].astype(np.uint64) >> np.uint64(32)).astype(np.int64)
    passes = (p[:, :, 7].astype(np.uint64) & np.uint64(0xffffffff)).astype(np.int64)
    dur = p[:, :, 6] - t0
    rt0, rt1 = p[:, 0, 8], p[:, 0, 9]
    span = (rt1.max() - rt0.min()) * 10e-3
    print(f"mode {a.mode} {a.mesh} {N} views {H}x{W}: {nwg} WGs, non-empty {ne.sum()}; kernel span (realtime) "
          f"{span:.1f} us")
    print("empty WG wave duration (cycles):", stats(dur[~ne].ravel()))
    print("non-empty WG wave duration      :", stats(dur[ne].ravel()))
    names = ["setup(0-2)", "pairs(2-3)", "sync(3-4)", "finalize(4-5)", "write(5-6)"]
    idx = [(0, 2), (2, 3), (3, 4), (4, 5), (5, 6)]
    for nm, (i, j) in zip(names, idx):
        print(f"  {nm:14s}", stats((p[ne][:, :, j] - p[ne][:, :, i]).ravel()))
    print("entries per non-empty WG:", stats(E[ne]), " passes per wave:", stats(passes[ne].ravel()))
    # time-ordered view of the non-empty workgroups (realtime, us from kernel start)
    st = (rt0 - rt0.min()) * 10e-3
    en = (rt1 - rt0.min()) * 10e-3
    print("non-empty WG start (us):", stats(st[ne]), " end:", stats(en[ne]))
    print("empty WG start (us):", stats(st[~ne]), " end:", stats(en[~ne]))
    order = np.argsort(-(en - st) * ne)[:5]
    for k in order:
        print(f"  longest: wg {k} view {k // (TY * GX)} E={E[k]} start {st[k]:.1f} end {en[k]:.1f} "
              f"passes/wave {passes[k].tolist()}")
    for q in (0.25, 0.5, 0.75, 0.9, 1.0):
        print(f"  {int(q * 100)}% of WGs finished by {np.percentile(en, q * 100):.1f} us")


if __name__ == "__main__":
    main()
