"""GPU parity of the fused render path (mr_render_forward/backward: one raster pass ->
depth, silhouette, Phong RGB; backward to vertices and per-view R, T) against the
oracle (C rasterizer + torch-CPU restatement of PyTorch3D's shading/blending, autograd).
Bar: pix_to_face bit-exact; images within 1e-4 abs; gradients within 1e-4 abs
per entry (tests.helpers.report: 1e-4 * max(1, |ref|), conditioning-aware)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import canonical_views, mesh_arrays, oracle_runs, report
from torch_renderer_amd import kernels as Kn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _run(name, H, W, N, texture, light_kind=0, persp=True, seed=1, bg=(1.0, 1.0, 1.0)):
    verts, faces, d = mesh_arrays(name)
    R, T, intr, _ = canonical_views(verts, N, H, W)
    tex_ref, tex_gpu, vcol = None, Kn.TextureArgs(), None
    if texture == "uv":
        img = torch.from_numpy(d["texture_u8"].astype(np.float32) / 255.0)
        vuv = torch.from_numpy(d["verts_uvs"]).float()
        fuv = torch.from_numpy(d["faces_uvs"]).long()
        tex_ref = ("uv", vuv, fuv, img)
        rgba = torch.zeros(img.shape[0], img.shape[1], 4)
        rgba[..., :3] = img
        tex_gpu = Kn.TextureArgs(2, vuv.to(DEV), fuv.to(torch.int32).to(DEV), rgba.to(DEV))
    elif texture == "vertex":
        g = torch.Generator().manual_seed(7)
        vcol = torch.rand(verts.shape, generator=g)
        tex_ref = ("vertex", vcol)
        tex_gpu = Kn.TextureArgs(1)
    light = dict(O.DEFAULT_LIGHT)
    if light_kind == 1:
        light = {"kind": "ambient", "ambient": (1.0, 1.0, 1.0)}
    gen = torch.Generator().manual_seed(seed)
    gD = torch.rand(N, H, W, generator=gen) * 2 - 1
    gS = torch.rand(N, H, W, generator=gen) * 2 - 1
    gC = torch.rand(N, H, W, 3, generator=gen) * 2 - 1

    def oracle(precision):  # reference (CPU autograd); "f64": its float64 shadow
        vr = verts.clone().requires_grad_(True)
        Rr = R.clone().requires_grad_(True)
        Tr = T.clone().requires_grad_(True)
        vcr = vcol.clone().requires_grad_(True) if vcol is not None else None
        tex_r = ("vertex", vcr) if texture == "vertex" else tex_ref
        ref = O.render_ref(vr, faces, Rr, Tr, intr, H, W, texture=tex_r, light=light, persp=persp, bg=bg,
                           precision=precision)
        dt = ref["rgba"].dtype
        loss = (ref["depth"] * gD.to(dt)).sum() + (ref["sil"] * gS.to(dt)).sum() + (ref["rgba"][..., :3] * gC.to(dt)).sum()
        loss.backward()
        return ref, (vr, Rr, Tr, vcr)

    def flat(precision):
        ref, lv = oracle(precision)
        z = torch.zeros(1)
        return (ref["depth"], ref["sil"], ref["rgba"][..., :3]) + tuple(x.grad if x is not None else z for x in lv)

    ref, (vr, Rr, Tr, vcr) = oracle("f32")
    r32, r64, sp = oracle_runs(flat)  # f32 oracle, float64 shadow, per-entry spread (tests.helpers.report)
    ref["shadow"] = (r64, sp)
    # GPU
    cfg = Kn.ShadeConfig(H=H, W=W, persp=persp, light_kind=light_kind, background=bg, want_p2f=True)
    if light_kind == 1:
        cfg.light_ambient = (1.0, 1.0, 1.0)
    vg = verts.to(DEV).requires_grad_(True)
    Rg = R.to(DEV).requires_grad_(True)
    Tg = T.to(DEV).requires_grad_(True)
    vcg = vcol.to(DEV).requires_grad_(True) if vcol is not None else None
    out = Kn.render_views(vg, Rg, Tg, faces.to(DEV), intr.to(DEV), torch.zeros(1, 3, device=DEV), cfg, tex_gpu,
                          vcolors=vcg)
    gl = (out["depth"] * gD.to(DEV)).sum() + (out["sil"] * gS.to(DEV)).sum() + (out["rgb"] * gC.to(DEV)).sum()
    gl.backward()
    return ref, out, (vr, Rr, Tr, vcr), (vg, Rg, Tg, vcg)


def _close(name, a, b, tol=1e-4, rel_scale=True, sens=None, ref64=None):
    """Per-entry bar (tests.helpers.report): |a_i - b_i| <= tol * max(1, |b_i|), or tol absolute
    (rel_scale=False, images), printed under `name`."""
    report(name, a, b, tol=tol, rel_above_one=rel_scale, sens=sens, ref64=ref64)


@pytest.mark.parametrize("name,H,W,N,texture", [
    ("cow", 64, 64, 2, "uv"),
    ("sphere", 48, 64, 2, None),
    ("teapot", 64, 64, 2, "vertex"),
])
def test_render_forward_backward(name, H, W, N, texture):
    ref, out, leaves_r, leaves_g = _run(name, H, W, N, texture)
    p2f_ref = ref["p2f"][..., 0]
    assert torch.equal(out["pix_to_face32"].cpu().long(), p2f_ref)
    r64, sp = ref["shadow"]
    tag = f"render {name} {H}x{W} {texture}"
    _close(f"{tag} depth", out["depth"], ref["depth"], rel_scale=False, ref64=r64[0], sens=sp[0])
    _close(f"{tag} sil", out["sil"], ref["sil"], rel_scale=False, ref64=r64[1], sens=sp[1])
    _close(f"{tag} rgb", out["rgb"], ref["rgba"][..., :3], rel_scale=False, ref64=r64[2], sens=sp[2])
    for i, (gr, gg, nm) in enumerate(zip(leaves_r, leaves_g, ("verts", "R", "T", "vcolors"))):
        if gr is None:
            continue
        assert gg.grad is not None, nm
        _close(f"{tag} grad {nm}", gg.grad, gr.grad, ref64=r64[3 + i], sens=sp[3 + i])


def test_render_ambient_no_perspective():
    ref, out, leaves_r, leaves_g = _run("sphere", 48, 48, 1, "vertex", light_kind=1, persp=False)
    assert torch.equal(out["pix_to_face32"].cpu().long(), ref["p2f"][..., 0])
    r64, sp = ref["shadow"]
    _close("ambient no-persp rgb", out["rgb"], ref["rgba"][..., :3], rel_scale=False, ref64=r64[2], sens=sp[2])
    for i, (gr, gg, nm) in enumerate(zip(leaves_r, leaves_g, ("verts", "R", "T", "vcolors"))):
        if gr is not None:
            _close(f"ambient no-persp grad {nm}", gg.grad, gr.grad, ref64=r64[3 + i], sens=sp[3 + i])
