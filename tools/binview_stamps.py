"""Per-workgroup timeline of k_bin_view on the C5 render (mesh_deformer.py:197: one view of the F=81,920 sphere at
1024x1024, AmbientLights, TexturesVertex), from an experiment build with workgroup stamps:
python tools/build_variant.py bvstamp -DMR_XP_BV_STAMP, then (GPU)
MI355R_LIB=exp/bvstamp.so python tools/binview_stamps.py [--fragments]   (--fragments: the fragment pass's launch)
Roles: binning (one workgroup per band of tile rows), ShadeRec packing, background fill. The launch's span is
the last end minus the first start; each role's start / end spread says which one is the critical path."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from torch_renderer_amd import _lib  # noqa: E402
from torch_renderer_amd.cameras import PerspectiveCameras  # noqa: E402
from torch_renderer_amd.mesh_renderer import (AmbientLights, MeshRasterizer, MeshRenderer,  # noqa: E402
                                              RasterizationSettings, SoftPhongShader)
from torch_renderer_amd.structures import Meshes, TexturesVertex  # noqa: E402
from torch_renderer_amd.transforms import look_at_view_transform  # noqa: E402
from torch_renderer_amd.utils import subdivided_sphere  # noqa: E402


def run_fragments(dev):
    """The fragment pass of bench.py --mode fragments (cow, 512x512, 64 views: k_bin_view<0, 3>)."""
    import argparse

    import bench
    a = argparse.Namespace(gpus=1, steps=3, warmup=1, views=64, size=512, mesh="cow", no_cpu_baseline=True,
                           no_fragment_pass=False, cpu_views=2, no_secondary=True, eager=True, texture="uv",
                           mode="fragments")
    bench.measure_fragments(a, dev, 1, 0)
    torch.cuda.synchronize()


def main():
    dev = torch.device("cuda:0")
    if "--fragments" in sys.argv:
        run_fragments(dev)
        return report()
    sph = subdivided_sphere(2)
    v0, faces = sph.verts_list()[0].to(dev), sph.faces_list()[0].to(dev)
    R, T = look_at_view_transform(dist=2.0, elev=torch.tensor([40.0]), azim=torch.tensor([-140.0]))
    cams = PerspectiveCameras(device=dev, R=R.to(dev), T=T.to(dev))
    rs = RasterizationSettings(image_size=1024, blur_radius=0.0, faces_per_pixel=1, perspective_correct=False)
    lights = AmbientLights(device=dev)
    ren = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs), SoftPhongShader(device=dev, cameras=cams,
                                                                                        lights=lights))
    col = torch.full((1, v0.shape[0], 3), 0.5, device=dev, requires_grad=True)
    mesh = Meshes([v0], [faces], TexturesVertex(verts_features=col))
    for _ in range(5):
        img = ren(mesh, cameras=cams, lights=lights)
        img[..., :3].sum().backward()
    torch.cuda.synchronize()
    report()


def report():
    fn = _lib.load().mr_xp_bv_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    nw = 4096
    buf = np.zeros((nw, 8), dtype=np.uint64)
    assert fn(buf.ctypes.data, nw) == 0
    live = buf[:, 0] > 0
    b = buf[live].astype(np.float64)
    t0 = b[:, 0].min()
    st, en, role = (b[:, 0] - t0) * 10.0 / 1e3, (b[:, 1] - t0) * 10.0 / 1e3, b[:, 2].astype(int)  # us (100 MHz)
    print(f"workgroups {len(b)}, launch span {en.max():.2f} us")
    for r, nm in enumerate(("binning", "ShadeRec", "background")):
        m = role == r
        if not m.any():
            continue
        life = en[m] - st[m]
        print(f"  {nm:10s} wgs {m.sum():4d}  start {st[m].min():6.2f}..{st[m].max():6.2f}  end "
              f"{en[m].min():6.2f}..{en[m].max():6.2f} (median {np.median(en[m]):6.2f})  life median "
              f"{np.median(life):6.2f} max {life.max():6.2f} us")
    # binning workgroups: phase durations (init, count, scan + allocation, units, fill, list store)
    m = role == 0
    ph = np.concatenate([b[m][:, 0:1], b[m][:, 3:8], b[m][:, 1:2]], axis=1)
    d = np.diff(ph, axis=1) * 10.0 / 1e3
    names = ("init", "count", "scan+alloc", "units", "fill", "store")
    order = np.argsort(-(en[m] - st[m]))
    for i in order[:8]:
        print("  band wg life %6.2f us: " % (en[m][i] - st[m][i]) + ", ".join(f"{nm} {d[i, k]:.2f}" for k, nm in
                                                                           enumerate(names)))
    print("  median over bands: " + ", ".join(f"{nm} {np.median(d[:, k]):.2f}" for k, nm in enumerate(names)))
    idx = np.argsort(-en)[:6]
    for i in idx:
        print(f"  late wg {int(np.nonzero(live)[0][i])}: role {role[i]} start {st[i]:.2f} end {en[i]:.2f} us")


if __name__ == "__main__":
    main()
