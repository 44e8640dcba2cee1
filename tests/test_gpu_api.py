"""GPU parity at the user-facing API: the drop-in classes of torch_renderer.py
(DepthRender, ColorRender, DepthColorRender), the PyTorch3D-style MeshRasterizer / MeshRenderer
and renderer.py's Renderer, each against the oracle fed the same camera conversion
(restated here, torch_renderer.py:73-80). Bars as in test_gpu_render.py: pix_to_face bit-exact,
images within 1e-4 abs, gradients within 1e-4 x scale."""
import math

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import canonical_views, fragment_grad_sensitivity, mesh_arrays, oracle_runs, report
from torch_renderer_amd import Meshes, TexturesUV, TexturesVertex
from torch_renderer_amd.cameras import PerspectiveCameras
from torch_renderer_amd.mesh_renderer import (BlendParams, Materials, MeshRasterizer, MeshRenderer, PointLights,
                                              RasterizationSettings, SoftPhongShader, SoftSilhouetteShader)
from torch_renderer_amd.torch_renderer import ColorRender, DepthColorRender, DepthRender

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _cv_to_p3d(R, t):
    Rp = R.transpose(1, 2).clone()
    Rp[:, :, :2] = -Rp[:, :, :2]
    Tp = t.clone()
    Tp[:, :2] = -Tp[:, :2]
    return Rp, Tp


def _intr(K, H, W, N):
    s = min(H, W) / 2.0
    return torch.tensor([[K[0, 0] / s, (W / 2.0 - K[0, 2]) / s, K[1, 1] / s, (H / 2.0 - K[1, 2]) / s]]).expand(N, 4)


def _cow_mesh(N):
    verts, faces, d = mesh_arrays("cow")
    img = torch.from_numpy(d["texture_u8"].astype(np.float32) / 255.0)
    vuv = torch.from_numpy(d["verts_uvs"]).float()
    fuv = torch.from_numpy(d["faces_uvs"]).long()
    tex = TexturesUV(maps=[img.to(DEV)], faces_uvs=[fuv.to(DEV)], verts_uvs=[vuv.to(DEV)])
    v = verts.to(DEV).requires_grad_(True)
    return verts, faces, (vuv, fuv, img), v, Meshes([v], [faces.to(DEV)], tex).extend(N)


def _close(name, a, b, tol=1e-4, sens=None, ref64=None):
    """Per-entry bar |a_i - b_i| <= tol * max(1, |b_i|) (tests.helpers.report), printed under `name`."""
    report(name, a, b, tol=tol, sens=sens, ref64=ref64)


def _oracle_cv(verts, faces, R_cv, t_cv, K, H, W, texture, grads, precision="f32", faces_per_pixel=1):
    """Oracle fwd+bwd of OpenCV-pose views (torch_renderer.py:73-80 conversion restated); returns the
    outputs and the leaves (verts, R_cv, t_cv) holding the gradients. precision="f64": the float64
    shadow (conditioning, tests.helpers.report)."""
    N = R_cv.shape[0]
    vr = verts.clone().requires_grad_(True)
    Rr = R_cv.clone().requires_grad_(True)
    tr = t_cv.clone().requires_grad_(True)
    Rp, Tp = _cv_to_p3d(Rr, tr)
    ref = O.render_ref(vr, faces, Rp, Tp, _intr(K, H, W, N).contiguous(), H, W, texture=texture, precision=precision,
                       K=faces_per_pixel)
    gD, gS, gC = grads
    ((ref["depth"] * gD).sum() + (ref["sil"] * gS).sum() + (ref["rgba"][..., :3] * gC).sum()).backward()
    return ref, (vr, Rr, tr)


_FLAT_NAMES = ("depth", "sil", "rgb", "grad verts", "grad R_cv", "grad t_cv")


def _oracle_cv_flat(*a, **kw):
    """_oracle_cv as a flat tuple (depth, sil, rgb, grad verts, grad R_cv, grad t_cv) for oracle_runs."""
    ref, (vr, Rr, tr) = _oracle_cv(*a, **kw)
    return ref["depth"], ref["sil"], ref["rgba"][..., :3], vr.grad, Rr.grad, tr.grad


def test_depth_color_render_match_oracle():
    H, W, N = 72, 96, 3
    verts, faces, (vuv, fuv, img), v, meshes = _cow_mesh(N)
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, N, H, W)
    # reference path on the CPU
    g = torch.Generator().manual_seed(3)
    gD, gS, gC = (torch.rand(N, H, W, generator=g) - 0.5, torch.rand(N, H, W, generator=g) - 0.5,
                  torch.rand(N, H, W, 3, generator=g) - 0.5)
    ref, r64, sp = oracle_runs(lambda p: _oracle_cv_flat(verts, faces, R_cv, t_cv, K, H, W, ("uv", vuv, fuv, img),
                                                         (gD, gS, gC), precision=p))
    # drop-in classes
    Rg = R_cv.to(DEV).requires_grad_(True)
    tg = t_cv.to(DEV).requires_grad_(True)
    depth, sil = DepthRender(K.to(DEV), (H, W), device=DEV).render(meshes, Rg, tg, return_silhouette=True)
    rgb = ColorRender(K.to(DEV), (H, W), device=DEV).render(meshes, Rg, tg)
    for i, x in enumerate((depth, sil, rgb)):
        _close(f"DepthRender+ColorRender {('depth', 'sil', 'rgb')[i]}", x, ref[i], ref64=r64[i], sens=sp[i])
    assert torch.equal(DepthRender(K.to(DEV), (H, W), device=DEV).render(meshes, Rg, tg).cpu(), depth.cpu())
    d3, s3, c3 = DepthColorRender(K.to(DEV), (H, W), device=DEV).render(meshes, Rg, tg)
    ((d3 * gD.to(DEV)).sum() + (s3 * gS.to(DEV)).sum() + (c3 * gC.to(DEV)).sum()).backward()
    for i, x in ((0, d3), (2, c3), (3, v.grad), (4, Rg.grad), (5, tg.grad)):
        _close(f"DepthColorRender {_FLAT_NAMES[i]}", x, ref[i], ref64=r64[i], sens=sp[i])


@pytest.mark.parametrize("distinct", [False, True])
def test_mesh_rasterizer_fragments_bitexact(distinct):
    H, W = 64, 80
    cv, cf, _ = mesh_arrays("cow")
    tv, tf, _ = mesh_arrays("teapot")
    if distinct:
        vs, fs = [cv, tv], [cf, tf]
    else:
        vs, fs = [cv, cv], [cf, cf]
    R, T, intr, (R_cv, t_cv, K) = canonical_views(cv, 2, H, W)
    # the teapot is ~10x the cow: push its view back along the optical axis
    if distinct:
        T = T.clone()
        T[1, 2] += 3.0
    cams = PerspectiveCameras(focal_length=((K[0, 0].item(), K[1, 1].item()),),
                              principal_point=((K[0, 2].item(), K[1, 2].item()),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]), device=DEV)
    vg = [x.to(DEV).requires_grad_(True) for x in vs]
    meshes = Meshes(vg, [f.to(DEV) for f in fs])
    Rg, Tg = R.to(DEV).requires_grad_(True), T.to(DEV).requires_grad_(True)
    frag = MeshRasterizer(cams, RasterizationSettings(image_size=(H, W)))(meshes, R=Rg, T=Tg)
    # oracle: per-view projection, packed ids, C rasterizer
    vr = [x.clone().requires_grad_(True) for x in vs]
    Rr, Tr = R.clone().requires_grad_(True), T.clone().requires_grad_(True)
    fv = torch.cat([O.project_faces_torch(vr[i], fs[i], Rr[i:i + 1], Tr[i:i + 1], intr[i:i + 1]) for i in range(2)])
    first = torch.tensor([0, fs[0].shape[0]])
    count = torch.tensor([fs[0].shape[0], fs[1].shape[0]])
    p2f, zbuf, bary, dists = O.RasterizeRef.apply(fv, first, count, H, W, 1, 0.0, True, False, False)
    assert torch.equal(frag.pix_to_face.cpu(), p2f)
    assert (p2f >= 0).sum() > 0.02 * 2 * H * W
    for a, b in ((frag.zbuf, zbuf), (frag.bary_coords, bary), (frag.dists, dists)):
        assert torch.equal(a.detach().cpu().view(torch.int32), b.detach().view(torch.int32))
    g = torch.Generator().manual_seed(5)
    gz = torch.rand(zbuf.shape, generator=g)
    gb = torch.rand(bary.shape, generator=g)
    ((frag.zbuf * gz.to(DEV)).sum() + (frag.bary_coords * gb.to(DEV)).sum()).backward()
    ((zbuf * gz).sum() + (bary * gb).sum()).backward()
    for nm, a, b in zip(("grad verts[0]", "grad verts[1]", "grad R", "grad T"), vg + [Rg, Tg], vr + [Rr, Tr]):
        _close(f"MeshRasterizer fragments (distinct={distinct}) {nm}", a.grad, b.grad)


@pytest.mark.parametrize("shader,W", [("phong", 64), ("silhouette", 64), ("silhouette", 66)])
def test_mesh_renderer_matches_oracle(shader, W):
    """Cameras built with R, T (renderer.py:65-69): specular uses the real camera centre. The
    silhouette's RGBA (1, 1, 1, alpha) comes straight from the kernels (W = 66: the per-pixel
    background stores instead of the 4-pixel vector ones)."""
    H, N = 64, 2
    verts, faces, d = mesh_arrays("teapot")
    R, T, intr, (R_cv, t_cv, K) = canonical_views(verts, N, H, W)
    g = torch.Generator().manual_seed(11)
    vcol = torch.rand(verts.shape, generator=g)
    cams = PerspectiveCameras(focal_length=((K[0, 0].item(), K[1, 1].item()),),
                              principal_point=((K[0, 2].item(), K[1, 2].item()),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]), R=R.to(DEV), T=T.to(DEV), device=DEV)
    lights = PointLights(location=[[0.5, 1.0, -2.0]], device=DEV)
    mats = Materials(shininess=32, device=DEV)
    blend = BlendParams(sigma=1e-4, gamma=1e-4, background_color=(0.0, 0.0, 0.0))
    sh = (SoftPhongShader(device=DEV, cameras=cams, lights=lights, materials=mats, blend_params=blend)
          if shader == "phong" else SoftSilhouetteShader(blend_params=blend))
    renderer = MeshRenderer(MeshRasterizer(cams, RasterizationSettings(image_size=(H, W))), sh)
    vg = verts.to(DEV).requires_grad_(True)
    img = renderer(Meshes([vg], [faces.to(DEV)], TexturesVertex([vcol.to(DEV)])).extend(N))
    cc = -torch.bmm(T[:, None, :], R.transpose(1, 2))[:, 0, :]
    light = dict(O.DEFAULT_LIGHT)
    light["location"] = (0.5, 1.0, -2.0)
    mat = dict(O.DEFAULT_MAT)
    mat["shininess"] = 32.0
    vr = verts.clone().requires_grad_(True)
    ref = O.render_ref(vr, faces, R, T, intr, H, W, texture=("vertex", vcol), light=light, mat=mat, cam_center=cc,
                       bg=(0.0, 0.0, 0.0))
    assert img.shape == (N, H, W, 4)
    if shader == "phong":
        _close(f"MeshRenderer {shader} W={W} rgba", img, ref["rgba"])
        go = torch.rand(N, H, W, 4, generator=g) - 0.5
        (ref["rgba"] * go).sum().backward()
    else:
        _close(f"MeshRenderer {shader} W={W} alpha", img[..., 3], ref["sil"])
        assert torch.equal(img[..., :3].cpu(), torch.ones(N, H, W, 3))
        go = torch.rand(N, H, W, 4, generator=g) - 0.5
        (ref["sil"] * go[..., 3]).sum().backward()
    (img * go.to(DEV)).sum().backward()
    _close(f"MeshRenderer {shader} W={W} grad verts", vg.grad, vr.grad)


def test_renderer_class_matches_oracle():
    """renderer.py:34-101 with the cow in place of the reference's (absent) mug."""
    from torch_renderer_amd.renderer import Renderer, _EXTRINSIC, _K

    H, W = 180, 320
    ren = Renderer(image_size=(H, W))
    verts, faces, d = mesh_arrays("cow")
    img = torch.from_numpy(d["texture_u8"].astype(np.float32) / 255.0)
    vuv = torch.from_numpy(d["verts_uvs"]).float()
    fuv = torch.from_numpy(d["faces_uvs"]).long()
    ren.meshes = Meshes([verts.to(DEV)], [faces.to(DEV)],
                        TexturesUV(maps=[img.to(DEV)], faces_uvs=[fuv.to(DEV)], verts_uvs=[vuv.to(DEV)]))
    ren.build_color_renderer()
    out = ren.render()
    R = torch.tensor(_EXTRINSIC[:3, :3], dtype=torch.float32)[None]
    T = torch.tensor(_EXTRINSIC[:3, 3], dtype=torch.float32)[None]
    K = torch.tensor(_K)
    s = min(H, W) / 2.0
    intr = torch.tensor([[K[0, 0] / s, (W / 2.0 - K[0, 2]) / s, K[1, 1] / s, (H / 2.0 - K[1, 2]) / s]])
    cc = -torch.bmm(T[:, None, :], R.transpose(1, 2))[:, 0, :]
    ref = O.render_ref(verts, faces, R, T, intr, H, W, texture=("uv", vuv, fuv, img), cam_center=cc)
    assert (ref["p2f"] >= 0).sum() > 50, "degenerate: the mesh is not in view"
    assert out.shape == (1, H, W, 4)
    _close("Renderer (renderer.py) rgba", out, ref["rgba"])


@pytest.mark.parametrize("broadcast", [False, True])
def test_native_pose_conversion_is_bitwise_the_torch_one(broadcast):
    """mr_views_from_opencv / mr_view_grads_to_opencv (the drop-in classes' camera conversion,
    torch_renderer.py:73-80) give bitwise the images and pose gradients of the torch conversion."""
    from torch_renderer_amd.kernels import ShadeConfig
    from torch_renderer_amd.torch_renderer import render_mesh_batch
    from torch_renderer_amd.transforms import opencv_to_pytorch3d
    H = W = 64
    N = 3
    verts, faces, _, _, mesh = _cow_mesh(N)
    _, _, _, (R, T, K) = canonical_views(verts, N, H, W)
    r = DepthColorRender(K.to(DEV), (H, W), device=DEV)
    if broadcast:
        R, T = R[:1], T[:1]
    outs, grads = [], []
    for native in (True, False):
        Rg = R.clone().to(DEV).requires_grad_(True)
        tg = T.clone().to(DEV).requires_grad_(True)
        Rin, tin = (Rg, tg) if native else opencv_to_pytorch3d(Rg, tg)
        if broadcast:
            Rin, tin = Rin.expand(N, 3, 3), tin.expand(N, 3)
        cfg = ShadeConfig(H=H, W=W, light_location=(0.0, 0.0, -3.0))
        o = render_mesh_batch(mesh, r._cameras, (H, W), Rin, tin, cfg, pose_cv=native)
        g = torch.Generator().manual_seed(3)
        loss = sum((o[k] * (torch.rand(o[k].shape, generator=g) * 2 - 1).to(DEV)).sum() for k in ("depth", "sil", "rgb"))
        loss.backward()
        outs.append([o[k].detach().cpu() for k in ("depth", "sil", "rgb")])
        grads.append((Rg.grad.cpu(), tg.grad.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    for a, b in zip(*grads):
        assert a.shape == b.shape
        assert torch.allclose(a, b, rtol=0, atol=1e-6 * max(1.0, b.abs().max().item()))


def test_drop_in_classes_faces_per_pixel_3_match_oracle():
    """faces_per_pixel > 1: DepthRender / ColorRender build the K-deep
    rasterizer + Soft* shaders as torch_renderer.py:90-108,132-153; gradients reach verts, R, t."""
    H, W, N, Kf = 48, 64, 2, 3
    verts, faces, (vuv, fuv, img), v, meshes = _cow_mesh(N)
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, N, H, W)
    g = torch.Generator().manual_seed(5)
    gD, gS, gC = (torch.rand(N, H, W, generator=g) - 0.5, torch.rand(N, H, W, generator=g) - 0.5,
                  torch.rand(N, H, W, 3, generator=g) - 0.5)
    ref, r64, sp = oracle_runs(lambda p: _oracle_cv_flat(verts, faces, R_cv, t_cv, K, H, W, ("uv", vuv, fuv, img),
                                                         (gD, gS, gC), precision=p, faces_per_pixel=Kf))
    Rg = R_cv.to(DEV).requires_grad_(True)
    tg = t_cv.to(DEV).requires_grad_(True)
    depth, sil = DepthRender(K.to(DEV), (H, W), faces_per_pixel=Kf, device=DEV).render(meshes, Rg, tg,
                                                                                      return_silhouette=True)
    rgb = ColorRender(K.to(DEV), (H, W), faces_per_pixel=Kf, device=DEV).render(meshes, Rg, tg)
    for i, x in enumerate((depth, sil, rgb)):
        _close(f"soft K={Kf} drop-in {_FLAT_NAMES[i]}", x, ref[i], ref64=r64[i], sens=sp[i])
    ((depth * gD.to(DEV)).sum() + (sil * gS.to(DEV)).sum() + (rgb * gC.to(DEV)).sum()).backward()
    for i, x in ((3, v.grad), (4, Rg.grad), (5, tg.grad)):
        _close(f"soft K={Kf} drop-in {_FLAT_NAMES[i]}", x, ref[i], ref64=r64[i], sens=sp[i])


@pytest.mark.parametrize("shader", ["phong", "silhouette"])
@pytest.mark.parametrize("Kf", [3, 8, 50])
def test_mesh_renderer_soft_raster_matches_oracle(shader, Kf):
    """MeshRenderer with faces_per_pixel = K and deform_mesh_with_color.py's blur_radius =
    ln(1/1e-4 - 1) * 1e-4 (clip_barycentric_coords defaults to True): K-deep HIP raster + the HIP
    soft shader (mr_shade_fragments_*) vs the oracle, fwd and grads."""
    H, W, N, blur = 40, 40, 2, math.log(1.0 / 1e-4 - 1.0) * 1e-4
    verts, faces, d = mesh_arrays("teapot")
    R, T, intr, (R_cv, t_cv, K) = canonical_views(verts, N, H, W)
    g = torch.Generator().manual_seed(13)
    vcol = torch.rand(verts.shape, generator=g)
    cams = PerspectiveCameras(focal_length=((K[0, 0].item(), K[1, 1].item()),),
                              principal_point=((K[0, 2].item(), K[1, 2].item()),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]), R=R.to(DEV), T=T.to(DEV), device=DEV)
    lights = PointLights(location=[[0.5, 1.0, -2.0]], device=DEV)
    blend = BlendParams(sigma=1e-4, gamma=1e-4, background_color=(0.2, 0.3, 0.4))
    sh = (SoftPhongShader(device=DEV, cameras=cams, lights=lights, blend_params=blend)
          if shader == "phong" else SoftSilhouetteShader(blend_params=blend))
    rs = RasterizationSettings(image_size=(H, W), blur_radius=blur, faces_per_pixel=Kf)
    renderer = MeshRenderer(MeshRasterizer(cams, rs), sh)
    vg = verts.to(DEV).requires_grad_(True)
    vc = vcol.to(DEV).requires_grad_(True)
    img = renderer(Meshes([vg], [faces.to(DEV)], TexturesVertex([vc])).extend(N))
    cc = -torch.bmm(T[:, None, :], R.transpose(1, 2))[:, 0, :]
    light = dict(O.DEFAULT_LIGHT)
    light["location"] = (0.5, 1.0, -2.0)
    # the camera's own NDC affine (focal length rounded to f32 first), so both sides rasterize the
    # same projected vertices and the fragments are bitwise equal
    intr = cams.ndc_affine((H, W)).cpu().expand(N, 4).contiguous()
    out = {}

    def run_oracle(precision="f32"):
        vr = verts.clone().requires_grad_(True)
        vcr = vcol.clone().requires_grad_(True)
        ref = O.render_ref(vr, faces, R, T, intr, H, W, texture=("vertex", vcr), light=light, cam_center=cc,
                           bg=(0.2, 0.3, 0.4), K=Kf, blur=blur, clip=True, precision=precision)
        out.setdefault("ref" if precision == "f32" else "ref64", ref)
        gg = go.to(ref["rgba"].dtype)
        loss = (ref["rgba"] * gg).sum() if shader == "phong" else (ref["sil"] * gg[..., 3]).sum()
        loss.backward()
        return (vr.grad, vcr.grad) if shader == "phong" else (vr.grad,)

    go = torch.rand(N, H, W, 4, generator=g) - 0.5
    # the teapot at 40x40 has sliver faces (projected area down to ~1e-5 px^2): the gradient of
    # their vertices is ill-conditioned in f32 on both sides, measured by the oracle's own spread
    refs, sens = fragment_grad_sensitivity(run_oracle)
    r64 = run_oracle("f64")
    ref = out["ref"]
    assert img.shape == (N, H, W, 4)
    if shader == "phong":
        _close(f"soft K={Kf} {shader} rgba", img, ref["rgba"], ref64=out["ref64"]["rgba"])
    else:
        _close(f"soft K={Kf} {shader} alpha", img[..., 3], ref["sil"], ref64=out["ref64"]["sil"])
    (img * go.to(DEV)).sum().backward()
    report(f"soft K={Kf} {shader} grad verts", vg.grad, refs[0], sens=sens[0], ref64=r64[0])
    if shader == "phong":
        report(f"soft K={Kf} {shader} grad vcolors", vc.grad, refs[1], sens=sens[1], ref64=r64[1])


def test_soft_raster_distinct_meshes_batch_equals_single_renders():
    """A batch of two different meshes (packed face ids, per-mesh textures) through the K-deep
    soft path equals rendering each mesh alone, images and vertex gradients."""
    H, W, Kf = 40, 48, 3
    g = torch.Generator().manual_seed(21)
    mv = []
    for name in ("teapot", "sphere"):
        v, f, _ = mesh_arrays(name)
        mv.append((v, f, torch.rand(v.shape, generator=g)))
    R, T, intr, (R_cv, t_cv, K) = canonical_views(mv[0][0], 2, H, W)
    cams = PerspectiveCameras(focal_length=((K[0, 0].item(), K[1, 1].item()),),
                              principal_point=((K[0, 2].item(), K[1, 2].item()),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]), device=DEV)
    rs = RasterizationSettings(image_size=(H, W), blur_radius=1e-4, faces_per_pixel=Kf)
    renderer = MeshRenderer(MeshRasterizer(cams, rs),
                            SoftPhongShader(device=DEV, cameras=cams, lights=PointLights(location=[[0.0, 1.0, -2.0]])))
    vb = [m[0].to(DEV).requires_grad_(True) for m in mv]
    batch = Meshes(vb, [m[1].to(DEV) for m in mv], TexturesVertex([m[2].to(DEV) for m in mv]))
    img = renderer(batch, R=R.to(DEV), T=T.to(DEV))
    go = torch.rand(img.shape, generator=g).to(DEV) - 0.5
    (img * go).sum().backward()
    for i, (v, f, c) in enumerate(mv):
        vs = v.to(DEV).requires_grad_(True)
        one = renderer(Meshes([vs], [f.to(DEV)], TexturesVertex([c.to(DEV)])), R=R[i:i + 1].to(DEV),
                       T=T[i:i + 1].to(DEV))
        (one * go[i:i + 1]).sum().backward()
        _close(f"distinct-mesh batch view {i} image vs single render", img[i:i + 1], one, tol=1e-6)
        _close(f"distinct-mesh batch mesh {i} grad verts vs single render", vb[i].grad, vs.grad, tol=1e-5)


def test_second_backward_over_one_forward_accumulates_exactly():
    """The fused backward accumulates its per-face gradient rows in the forward's workspace, which
    the forward clears (MR_GRAD_ROWS_CLEARED on the first backward). A second backward over the same
    forward (retain_graph) must clear them again: it yields the same gradients as the first."""
    verts, faces, _ = mesh_arrays("cow")
    H = W = 96
    N = 3
    R_cv, t_cv, K = canonical_views(verts, N, H, W)[3]
    vg = verts.to(DEV).requires_grad_(True)
    m = Meshes([vg], [faces.to(DEV)], TexturesVertex([torch.ones_like(vg).detach()])).extend(N)
    Rg = R_cv.float().to(DEV).requires_grad_(True)
    tg = t_cv.float().to(DEV).requires_grad_(True)
    d, s, c = DepthColorRender(K.to(DEV), (H, W), device=DEV).render(m, Rg, tg)
    g = torch.Generator(device=DEV).manual_seed(3)
    gd, gs, gc = (torch.rand(x.shape, generator=g, device=DEV) - 0.5 for x in (d, s, c))
    torch.autograd.backward([d, s, c], [gd, gs, gc], retain_graph=True)
    first = [x.grad.clone() for x in (vg, Rg, tg)]
    for x in (vg, Rg, tg):
        x.grad = None
    torch.autograd.backward([d, s, c], [gd, gs, gc])
    for a, b, nm in zip((vg.grad, Rg.grad, tg.grad), first, ("verts", "R", "t")):
        report(f"second backward {nm}", a.cpu(), b.cpu())


@pytest.mark.parametrize("texture", ["vertex", "uv_shared_map"])
def test_distinct_meshes_one_launch_equals_per_mesh_renders(texture):
    """renderer.py:78-80,100-101: a Meshes of N different meshes rendered in one call. The fused
    path renders their union in ONE launch (view n rasterizes only mesh n's faces); images must
    equal rendering each mesh alone bitwise, gradients within float-summation-order noise."""
    from torch_renderer_amd import kernels as Kn
    from torch_renderer_amd.torch_renderer import render_mesh_batch

    H, W = 56, 64
    g = torch.Generator().manual_seed(8)
    cv, cf, d = mesh_arrays("cow")
    if texture == "vertex":
        names = ("cow", "teapot", "sphere")
        mv = []
        for name in names:
            v, f, _ = mesh_arrays(name)
            v = (v - v.mean(0)) / (v - v.mean(0)).abs().max() * 0.4 + cv.mean(0)  # every mesh cow-sized
            mv.append((v, f))
        tex_of = lambda vs: TexturesVertex([torch.rand(v.shape, generator=g).to(DEV) for v in vs])  # noqa: E731
    else:  # two cows (one deformed) sharing ONE texture map: the union keeps one map
        img = torch.from_numpy(d["texture_u8"].astype(np.float32) / 255.0).to(DEV)
        vuv = torch.from_numpy(d["verts_uvs"]).float().to(DEV)
        fuv = torch.from_numpy(d["faces_uvs"]).long().to(DEV)
        mv = [(cv, cf), (cv + 0.01 * torch.randn(cv.shape, generator=g), cf)]
        tex_of = lambda vs: TexturesUV(maps=[img] * len(vs), faces_uvs=[fuv] * len(vs), verts_uvs=[vuv] * len(vs))  # noqa: E731
    N = len(mv)
    R, T, intr, (R_cv, t_cv, K) = canonical_views(cv, N, H, W)
    cams = PerspectiveCameras(focal_length=((K[0, 0].item(), K[1, 1].item()),),
                              principal_point=((K[0, 2].item(), K[1, 2].item()),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]), device=DEV)
    cfg = Kn.ShadeConfig(H=H, W=W, want_p2f=True, light_location=(0.0, 1.0, -2.0))
    vb = [m[0].to(DEV).requires_grad_(True) for m in mv]
    tex = tex_of(vb)
    Rg, Tg = R.to(DEV).requires_grad_(True), T.to(DEV).requires_grad_(True)
    out = render_mesh_batch(Meshes(vb, [m[1].to(DEV) for m in mv], tex), cams, (H, W), Rg, Tg, cfg)
    gD, gS, gC = (torch.rand(out[k].shape, generator=g).to(DEV) - 0.5 for k in ("depth", "sil", "rgb"))
    ((out["depth"] * gD).sum() + (out["sil"] * gS).sum() + (out["rgb"] * gC).sum()).backward()
    Fsum = 0
    for i, (v, f) in enumerate(mv):
        vs = v.to(DEV).requires_grad_(True)
        Ri, Ti = R[i:i + 1].to(DEV).requires_grad_(True), T[i:i + 1].to(DEV).requires_grad_(True)
        one = render_mesh_batch(Meshes([vs], [f.to(DEV)], tex[i]), cams, (H, W), Ri, Ti, cfg)
        ((one["depth"] * gD[i:i + 1]).sum() + (one["sil"] * gS[i:i + 1]).sum() +
         (one["rgb"] * gC[i:i + 1]).sum()).backward()
        for k in ("depth", "sil", "rgb"):
            assert torch.equal(out[k][i:i + 1], one[k]), (i, k)
        p1 = one["pix_to_face32"]
        assert torch.equal(out["pix_to_face32"][i:i + 1], torch.where(p1 >= 0, p1 + Fsum, p1)), i
        assert (p1 >= 0).sum() > 0.02 * H * W
        Fsum += f.shape[0]
        _close(f"fused distinct-mesh batch mesh {i} grad verts", vb[i].grad, vs.grad, tol=1e-5)
        _close(f"fused distinct-mesh batch view {i} grad R", Rg.grad[i:i + 1], Ri.grad, tol=1e-5)
        _close(f"fused distinct-mesh batch view {i} grad T", Tg.grad[i:i + 1], Ti.grad, tol=1e-5)
