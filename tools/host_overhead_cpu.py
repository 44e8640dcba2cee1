"""Python-side host cost of one C5 render call (mesh_deformer.py:197: renderer(mesh, cameras=cams[j], lights=lights))
measured on the CPU: the native call and the HIP-only helpers are stubbed, so what is timed is the Python work
around them (MeshRenderer.forward -> render_mesh_batch -> kernels.render_views). Experiments only.
python tools/host_overhead_cpu.py [--profile]"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from torch_renderer_amd import _lib, kernels  # noqa: E402
from torch_renderer_amd.cameras import PerspectiveCameras  # noqa: E402
from torch_renderer_amd.mesh_renderer import (AmbientLights, MeshRasterizer, MeshRenderer,  # noqa: E402
                                              RasterizationSettings, SoftPhongShader)
from torch_renderer_amd.structures import Meshes, TexturesVertex  # noqa: E402
from torch_renderer_amd.transforms import look_at_view_transform  # noqa: E402
from torch_renderer_amd.utils import subdivided_sphere  # noqa: E402


class _Ext:
    @staticmethod
    def render_views(verts, R, T, vcolors, f, vptr, vadj, intr, cc, tex_kind, *a):
        N = R.shape[0]
        out = torch.empty(N, 4, 4, 4)
        return [out, torch.empty(1), torch.empty(N, 16)]


def main():
    kernels._require_cuda = lambda *a: None
    _lib.torch_ext = lambda: _Ext
    _lib.stream_handle = lambda dev=None: type("H", (), {"value": 0})()
    sph = subdivided_sphere(2)
    v0, faces = sph.verts_list()[0], sph.faces_list()[0]
    R, T = look_at_view_transform(dist=2.0, elev=torch.linspace(0, 360, 10), azim=torch.linspace(-180, 180, 10))
    lights = AmbientLights()
    rs = RasterizationSettings(image_size=1024, blur_radius=0.0, faces_per_pixel=1, perspective_correct=False)
    cams = PerspectiveCameras(R=R, T=T)
    renderer = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs),
                            SoftPhongShader(cameras=cams, lights=lights))
    tc = [PerspectiveCameras(R=R[None, i], T=T[None, i]) for i in range(10)]
    rgb = torch.full((1, v0.shape[0], 3), 0.5)
    mesh = Meshes([v0], [faces], TexturesVertex(verts_features=rgb))
    for i in range(50):
        renderer(mesh, cameras=tc[i % 10], lights=lights)
    ts = []
    for i in range(400):
        t0 = time.perf_counter()
        renderer(mesh, cameras=tc[i % 10], lights=lights)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"python host us per render call (native call stubbed): median {ts[len(ts) // 2] * 1e6:.1f}")
    if "--profile" in sys.argv:
        pr = cProfile.Profile()
        pr.enable()
        for i in range(400):
            renderer(mesh, cameras=tc[i % 10], lights=lights)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
