"""Does the vertex numbering bound C5's vertex-gradient gathers? The C5 render + backward (one view of the F=81,920
sphere, 1024x1024, ambient light, vertex colours) timed per kernel (HIP events) on the sphere as subdivided and on
the same mesh with its vertices renumbered in order of first use by the faces (neighbouring vertices then gather
neighbouring face rows). Experiments only (GPU): python tools/vertex_order_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from torch_renderer_amd import _lib  # noqa: E402
from torch_renderer_amd.cameras import PerspectiveCameras  # noqa: E402
from torch_renderer_amd.mesh_renderer import (AmbientLights, MeshRasterizer, MeshRenderer,  # noqa: E402
                                              RasterizationSettings, SoftPhongShader)
from torch_renderer_amd.structures import Meshes, TexturesVertex  # noqa: E402
from torch_renderer_amd.transforms import look_at_view_transform  # noqa: E402
from torch_renderer_amd.utils import subdivided_sphere  # noqa: E402


def renumber(v, f):
    """Vertices in order of first use by the faces (face-major, corner order)."""
    order = []
    seen = torch.zeros(v.shape[0], dtype=torch.bool)
    for x in f.reshape(-1).tolist():
        if not seen[x]:
            seen[x] = True
            order.append(x)
    order = torch.tensor(order, dtype=torch.long)
    inv = torch.empty_like(order)
    inv[order] = torch.arange(order.numel())
    return v[order], inv[f]


def run(v0, faces, tag, dev):
    R, T = look_at_view_transform(dist=2.0, elev=torch.tensor([40.0]), azim=torch.tensor([-140.0]))
    cams = PerspectiveCameras(device=dev, R=R.to(dev), T=T.to(dev))
    rs = RasterizationSettings(image_size=1024, blur_radius=0.0, faces_per_pixel=1, perspective_correct=False)
    lights = AmbientLights(device=dev)
    ren = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs),
                       SoftPhongShader(device=dev, cameras=cams, lights=lights))
    col = torch.full((1, v0.shape[0], 3), 0.5, device=dev, requires_grad=True)
    vv = v0.clone().requires_grad_(True)

    def step():
        img = ren(Meshes([vv], [faces], TexturesVertex(verts_features=col)), cameras=cams, lights=lights)
        img[..., :3].sum().backward()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    _lib.timing_enable(True)
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    kt = _lib.timing_read()
    _lib.timing_enable(False)
    print(tag, {k: round(v[1] / v[0] * 1e3, 2) for k, v in kt.items()}, flush=True)


def main():
    dev = torch.device("cuda:0")
    sph = subdivided_sphere(2)
    v, f = sph.verts_list()[0], sph.faces_list()[0]
    run(v.to(dev), f.to(dev), "as subdivided", dev)
    v2, f2 = renumber(v, f)
    run(v2.to(dev), f2.to(dev), "renumbered", dev)
    run(v.to(dev), f.to(dev), "as subdivided", dev)
    run(v2.to(dev), f2.to(dev), "renumbered", dev)


if __name__ == "__main__":
    main()
