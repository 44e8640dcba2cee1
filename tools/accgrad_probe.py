"""Which object keeps a leaf's AccumulateGrad node alive after a fused render's fwd+bwd (VERDICT r5
"next" #3: the precondition of the HIP-graph-capture crash at bench.py's capture). Tags the node of
verts / R / t through the render output's graph, drops the outputs, then checks — before and after
clearing each module-level cache — whether a fresh view of the leaf still reaches the tagged node.
python tools/accgrad_probe.py   (GPU)"""
import gc
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from torch_renderer_amd import kernels as Kn  # noqa: E402
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.structures import Meshes  # noqa: E402
from torch_renderer_amd.torch_renderer import DepthColorRender  # noqa: E402


def acc_of(t):
    v = t.view_as(t)
    return v.grad_fn.next_functions[0][0]


def alive(leaves, tag):
    return {k: acc_of(t).metadata.get("tag") == tag for k, t in leaves.items()}


def main():
    dev = torch.device("cuda:0")
    H = W = 128
    nv = 4
    meshes = load_asset("cow", device=dev)
    v0 = meshes.shared_verts().detach().cpu()
    R, t, K = bench.canonical_views(v0, nv, H, W, dist_m=bench.view_distance("cow", v0))
    R = R.to(dev).contiguous().requires_grad_(True)
    t = t.to(dev).contiguous().requires_grad_(True)
    verts = meshes.shared_verts().clone().requires_grad_(True)
    bm = Meshes([verts], [meshes.shared_faces()], meshes.textures).extend(nv)
    ren = DepthColorRender(K.to(dev), (H, W), device=dev)
    g = [torch.rand(nv, H, W, device=dev), torch.rand(nv, H, W, device=dev), torch.rand(nv, H, W, 3, device=dev)]
    leaves = {"verts": verts, "R": R, "t": t}
    for it in range(2):
        outs = ren.render(bm, R, t)
        gf = outs[0].grad_fn
        print("iter", it, "grad_fn", type(gf).__name__, "next", [type(n[0]).__name__ if n[0] is not None else None
                                                               for n in gf.next_functions], flush=True)
        tag = f"it{it}"
        for k, x in leaves.items():
            acc_of(x).metadata["tag"] = tag
        del gf
        torch.autograd.backward(list(outs), g)
        del outs
        print(" after del outputs:", alive(leaves, tag), flush=True)
        gc.collect()
        print(" after gc.collect:", alive(leaves, tag), flush=True)
    ent = Kn._RESHADE["entry"]
    print(" reshade entry keys:", None if ent is None else list(ent.keys()), flush=True)
    Kn._RESHADE["entry"] = None
    gc.collect()
    print(" after clearing _RESHADE:", alive(leaves, tag), flush=True)
    Kn._LAST_RENDER = None
    gc.collect()
    print(" after clearing _LAST_RENDER:", alive(leaves, tag), flush=True)
    for c in (ren._cameras,):
        for k in [k for k in vars(c) if k.startswith("_") and k.endswith("cache")]:
            delattr(c, k)
    gc.collect()
    print(" after clearing camera caches:", alive(leaves, tag), flush=True)
    del bm
    gc.collect()
    print(" after del Meshes:", alive(leaves, tag), flush=True)
    # referrers of the leaves (Python side) that are not this frame's dicts
    for k, x in leaves.items():
        refs = [type(r).__name__ for r in gc.get_referrers(x) if r is not leaves]
        print(" referrers of", k, refs, flush=True)


if __name__ == "__main__":
    main()
