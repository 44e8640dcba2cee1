"""torch.profiler view of one bench step (which torch ops launch the non-mi355r kernels, and
how long the host takes to enqueue a step). python tools/step_profile.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.structures import Meshes  # noqa: E402
from torch_renderer_amd.torch_renderer import DepthColorRender  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    H = W = 512
    nv = 64
    meshes = load_asset("cow", device=dev)
    verts0 = meshes.shared_verts().detach().cpu()
    faces = meshes.shared_faces()
    R_all, t_all, K = bench.canonical_views(verts0, nv, H, W)
    R_cv = R_all.to(dev).requires_grad_(True)
    t_cv = t_all.to(dev).requires_grad_(True)
    verts = meshes.shared_verts().clone().requires_grad_(True)
    bmesh = Meshes([verts], [faces], meshes.textures).extend(nv)
    renderer = DepthColorRender(K.to(dev), (H, W), device=dev)
    gD = torch.rand(nv, H, W, device=dev)
    gS = torch.rand(nv, H, W, device=dev)
    gC = torch.rand(nv, H, W, 3, device=dev)

    def step():
        verts.grad = None
        R_cv.grad = None
        t_cv.grad = None
        depth, sil, rgb = renderer.render(bmesh, R_cv, t_cv)
        torch.autograd.backward([depth, sil, rgb], [gD, gS, gC])

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0) / 20:.3f} ms/step, wall {1e3 * (t2 - t0) / 20:.3f} ms/step")
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(3):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=30,
                                                               max_name_column_width=40, max_shapes_column_width=60))


if __name__ == "__main__":
    main()
