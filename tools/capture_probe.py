"""Experiments only: which HIP-graph capture shapes of the fused render step work (bench.py's step).
python tools/capture_probe.py MODE   (MODE: single | split | fwd)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.structures import Meshes  # noqa: E402
from torch_renderer_amd.torch_renderer import DepthColorRender  # noqa: E402

mode = sys.argv[1]
dev = torch.device("cuda:0")
H = W = int(os.environ.get("PROBE_SIZE", "256"))
nv = int(os.environ.get("PROBE_VIEWS", "8"))
meshes = load_asset("cow", device=dev)
verts0 = meshes.shared_verts().detach().cpu()
R, t, K = bench.canonical_views(verts0, nv, H, W, dist_m=bench.view_distance("cow", verts0))
R = R.to(dev).contiguous().requires_grad_(True)
t = t.to(dev).contiguous().requires_grad_(True)
verts = meshes.shared_verts().clone().requires_grad_(True)
bm = Meshes([verts], [meshes.shared_faces()], meshes.textures).extend(nv)
ren = DepthColorRender(K.to(dev), (H, W), device=dev)
g = [torch.rand(nv, H, W, device=dev), torch.rand(nv, H, W, device=dev), torch.rand(nv, H, W, 3, device=dev)]
for _ in range(int(os.environ.get("PROBE_WARM", "0"))):  # bench.py's warmup: eager steps on the default stream
    verts.grad = R.grad = t.grad = None
    torch.autograd.backward(list(ren.render(bm, R, t)), g)
if os.environ.get("PROBE_STATS"):
    from torch_renderer_amd.kernels import render_stats
    _keep = ren.render(bm, R, t)
    print(render_stats(), flush=True)
    del _keep
torch.cuda.synchronize()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        verts.grad = R.grad = t.grad = None
        torch.autograd.backward(list(ren.render(bm, R, t)), g)
torch.cuda.current_stream().wait_stream(side)
verts.grad = R.grad = t.grad = None
pool = torch.cuda.graph_pool_handle()
print("capturing", mode, flush=True)
if mode == "single":
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, pool=pool):
        outs = ren.render(bm, R, t)
        torch.autograd.backward(list(outs), g)
    gr.replay()
elif mode == "split":
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, pool=pool):
        outs = ren.render(bm, R, t)
    with torch.cuda.graph(g2, pool=pool):
        torch.autograd.backward(list(outs), g, retain_graph=True)
    g1.replay()
    g2.replay()
else:
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, pool=pool):
        outs = ren.render(bm, R, t)
    g1.replay()
torch.cuda.synchronize()
print("ok", mode, float(verts.grad.abs().sum()) if verts.grad is not None else None, flush=True)
