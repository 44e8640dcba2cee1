"""Phase timing of the fused backward (k_bwd_fused) on the headline workload, from an experiment build with
per-wave stamps: python tools/build_variant.py stamp -DMR_XP_BWD_STAMP, then (GPU)
MI355R_LIB=exp/stamp.so python tools/bwd_stamps.py
Per wave: global-clock start / end (100 MHz), slots, shader cycles per phase of the slot loop
(0 loop top; 1 half 1: shade fwd+bwd; 2 world corners + the next slots' prefetches + the previous slot's
flush; 3 raster + projection backward; 4 segmented scan + R/T sums). The stamps cost cycles
themselves (s_memtime waits); read the shares, not the absolute time."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from torch_renderer_amd import _lib  # noqa: E402
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.structures import Meshes  # noqa: E402
from torch_renderer_amd.torch_renderer import DepthColorRender  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    H = W = 512
    nv = 64
    meshes = load_asset("cow", device=dev)
    v0 = meshes.shared_verts().detach().cpu()
    R, t, K = bench.canonical_views(v0, nv, H, W, dist_m=bench.view_distance("cow", v0))
    R = R.to(dev).contiguous().requires_grad_(True)
    t = t.to(dev).contiguous().requires_grad_(True)
    verts = meshes.shared_verts().clone().requires_grad_(True)
    bm = Meshes([verts], [meshes.shared_faces()], meshes.textures).extend(nv)
    ren = DepthColorRender(K.to(dev), (H, W), device=dev)
    gen = torch.Generator().manual_seed(1)
    g = [(torch.rand(nv, H, W, generator=gen) * 2 - 1).to(dev), (torch.rand(nv, H, W, generator=gen) * 2 - 1).to(dev),
         (torch.rand(nv, H, W, 3, generator=gen) * 2 - 1).to(dev)]
    for _ in range(6):
        torch.autograd.backward(list(ren.render(bm, R, t)), g)
    torch.cuda.synchronize()
    L = _lib.load()
    fn = L.mr_xp_bwd_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    nw = 16384
    buf = np.zeros((nw, 8), dtype=np.uint64)
    assert fn(buf.ctypes.data, nw) == 0
    live = buf[:, 0] > 0
    b = buf[live].astype(np.float64)
    t0 = b[:, 0].min()
    st, en = (b[:, 0] - t0) * 10.0, (b[:, 1] - t0) * 10.0  # ns (100 MHz)
    span = en.max()
    n = b[:, 2]
    ph = b[:, 3:8]
    print(f"waves {len(b)}, slots {int(n.sum())}, kernel span {span / 1e3:.1f} us (stamped build)")
    print(f"slots per wave: mean {n.mean():.2f}, min {n.min():.0f}, max {n.max():.0f}, hist "
          f"{np.bincount(n.astype(int)).tolist()}")
    life = en - st
    print(f"wave start: max {st.max() / 1e3:.1f} us; end: min {en.min() / 1e3:.1f}, median {np.median(en) / 1e3:.1f}, "
          f"max {span / 1e3:.1f} us; mean lifetime / span {life.mean() / span:.3f}")
    names = ("loop top", "half 1: shade fwd+bwd", "corners + prefetch + flush", "raster + proj bwd",
             "seg scan + R/T sums")
    tot = ph.sum()
    per_slot = ph.sum(0) / n.sum()
    for i, nm in enumerate(names):
        print(f"  {nm:24s} {100 * ph[:, i].sum() / tot:5.1f} %   {per_slot[i]:8.0f} cycles/slot")
    print(f"  total {per_slot.sum():.0f} cycles per slot (shader clock, includes the other waves' issue)")
    # the longest waves: their slots and phases
    idx = np.argsort(-en)[:5]
    for i in idx:
        print(f"  late wave: start {st[i] / 1e3:.1f} end {en[i] / 1e3:.1f} us, slots {n[i]:.0f}, phases "
              f"{(ph[i] / max(n[i], 1)).astype(int).tolist()}")
    # end-time histogram (10 bins)
    h, e = np.histogram(en / 1e3, bins=10)
    print("end-time histogram (us):", [(round(float(e[k]), 1), int(h[k])) for k in range(10)])


if __name__ == "__main__":
    main()
