"""Work counters of the K-deep soft raster on bench.py --mode soft's workload (list entries, tiles,
entries per tile): python tools/soft_stats.py [size] [views]."""
import ctypes
import math
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from torch_renderer_amd import _lib, kernels as Kn  # noqa: E402
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.cameras import PerspectiveCameras, view_batch  # noqa: E402
from torch_renderer_amd.transforms import look_at_view_transform  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    H = W = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    m = load_asset("cow", device=dev, textures=False)
    v0 = m.shared_verts().detach()
    c = v0.mean(0)
    v = ((v0 - c) / (v0 - c).abs().max()).contiguous()
    f = m.shared_faces()
    R, T = look_at_view_transform(dist=2.7, elev=torch.linspace(0, 360, N), azim=torch.linspace(-180, 180, N))
    cams = PerspectiveCameras(device=dev, R=R.to(dev), T=T.to(dev))
    Rb, Tb, intr = view_batch(cams, (H, W), R.to(dev), T.to(dev), n_views=N)
    L = _lib.load()
    fi, _, _ = Kn.mesh_topology(f, v.shape[0])
    Fn = fi.shape[0]
    for K, blur in ((1, 0.0), (50, math.log(1.0 / 1e-4 - 1.0) * 1e-4)):
        s = Kn.raster_settings_struct(H, W, K, blur, False, blur > 0, False, None, None)
        ps, keep = Kn._poses_struct(Rb.contiguous(), Tb.contiguous(), intr.contiguous())
        views = torch.empty((N, 16), device=dev)
        fv = torch.empty((N * Fn, 3, 3), device=dev)
        p2f = torch.empty((N, H, W, K), dtype=torch.int64, device=dev)
        zb = torch.empty((N, H, W, K), device=dev)
        ba = torch.empty((N, H, W, K, 3), device=dev)
        di = torch.empty((N, H, W, K), device=dev)
        wsb = L.mr_rasterize_meshes_world_workspace(N, Fn, H, W, 0)
        ws = torch.empty(int(wsb), dtype=torch.uint8, device=dev)
        _lib.check(L.mr_rasterize_meshes_world(_lib.ptr(v), v.shape[0], _lib.ptr(fi), Fn, ctypes.byref(ps), N,
                                               ctypes.byref(s), _lib.ptr(views), _lib.ptr(fv), _lib.ptr(p2f),
                                               _lib.ptr(zb), _lib.ptr(ba), _lib.ptr(di), _lib.ptr(ws), wsb,
                                               _lib.stream_handle(dev)))
        out = (ctypes.c_int64 * 4)()
        _lib.check(L.mr_workspace_stats(_lib.ptr(ws), N, N * Fn, H, W, 0, ctypes.cast(out, ctypes.c_void_p),
                                        _lib.stream_handle(dev)))
        # per-tile list lengths: ws = face records (2 Ftot x 64 B, 256-aligned), then ctr (16 ints), cnt (N T)
        off = ((2 * N * Fn * 64) + 255) // 256 * 256
        T = ((W + 7) // 8) * ((H + 7) // 8)
        cnt = ws[off:off + 4 * (16 + N * T)].view(torch.int32)[16:].float()
        nz = cnt[cnt > 0]
        q = torch.quantile(nz, torch.tensor([0.5, 0.9, 0.99], device=dev)).tolist() if nz.numel() else []
        if nz.numel():
            print(f"  list length per non-empty tile: mean {nz.mean().item():.0f} p50/p90/p99 {q} max {nz.max().item():.0f}")
        frac = float((p2f[..., 0] >= 0).float().mean())
        print(f"K={K} blur={blur:.2e}: entries {out[0]}, tiles {out[2]}, entries/tile {out[0] / max(out[2], 1):.1f}, "
              f"covered fraction {frac:.3f}, filled slots/pixel {(p2f >= 0).sum().item() / (N * H * W):.2f}")


if __name__ == "__main__":
    main()
