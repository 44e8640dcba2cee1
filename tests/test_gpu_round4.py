"""Round-4 GPU checks:

* MeshRasterizer's lazy K = 1 Fragments: ``zbuf`` read alone comes from the fused render in zbuf mode
  (MR_OUT_ZBUF) — bitwise the modular rasterizer's zbuf, and the gradient of relu(zbuf[..., 0]) (what
  camera_pose_optimizer.py:244-246 backpropagates) equal to the modular path's within the per-entry bar.
* pose_loss on the RGBA slices the reference passes (camera_pose_optimizer.py:248,250: ``[..., 3]`` and
  ``[..., :3]``): read in place, gradients returned for the whole images — against torch autograd through
  the same slices.
* quaternion_to_matrix on HIP tensors (one launch each way) against the torch formula, values and gradients.
* The fused soft silhouette at the soft bench config (deform_mesh_with_color.py:153-165: 128x128, K = 50,
  blur = ln(1/1e-4 - 1) 1e-4, perspective_correct=False, 64 views) against the oracle on two of the views:
  images and vertex gradients of an L2 silhouette loss within the per-entry bars, and the depth-ordered
  list walk (count > 64 listed faces in a tile) exercised — read from the workspace's work counter.
"""
import ctypes
import math

import pytest
import torch

from oracle import oracle as O
from tests.helpers import mesh_arrays, oracle_runs, report
from torch_renderer_amd import _lib
from torch_renderer_amd.assets import load_asset
from torch_renderer_amd.cameras import FoVPerspectiveCameras, PerspectiveCameras
from torch_renderer_amd.losses import pose_loss
from torch_renderer_amd.mesh_renderer import (BlendParams, MeshRasterizer, MeshRenderer, RasterizationSettings,
                                              SoftSilhouetteShader, _LazyFragments)
from torch_renderer_amd.structures import Meshes
from torch_renderer_amd.transforms import look_at_view_transform, quaternion_to_matrix, quaternion_to_matrix_torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("camera", ["fov_clip", "perspective"])
def test_lazy_zbuf_fused_equals_modular(camera):
    """camera_pose_optimizer.py:244-246: rasterizer(meshes_world=..., R=, T=).zbuf[..., 0] (FoV camera:
    near-plane clipping at znear / 2) and the PerspectiveCameras rasterizer of batch_rendering_test.py:274.
    zbuf bitwise the modular rasterizer's; the gradients of relu(zbuf) (the fused depth backward) against the
    oracle's within the per-entry bar (the modular path's too)."""
    H = W = 192
    N = 3
    meshes = load_asset("cow", device=DEV, textures=False)
    v0 = meshes.shared_verts().detach()
    dist = 0.35 if camera == "fov_clip" else 0.7
    R, T = look_at_view_transform(dist, torch.linspace(5, 60, N), torch.linspace(0, 330, N), device=DEV,
                                  at=(v0.mean(0).tolist(),))
    if camera == "fov_clip":
        znear = 0.3
        cams = FoVPerspectiveCameras(device=DEV, znear=znear)
        t = 1.0 / math.tan(math.radians(30.0))
        intr, z_clip = torch.tensor([[t, 0.0, t, 0.0]]), znear / 2
    else:
        cams = PerspectiveCameras(device=DEV, focal_length=((2.0, 2.0),))
        intr, z_clip = torch.tensor([[2.0, 0.0, 2.0, 0.0]]), None
    rs = RasterizationSettings(image_size=H, blur_radius=0.0, faces_per_pixel=1)
    rast = MeshRasterizer(cameras=cams, raster_settings=rs)
    g = torch.Generator().manual_seed(5)
    go = (torch.rand(N, H, W, generator=g) * 2 - 1).to(DEV)

    def run(lazy):
        v = v0.clone().requires_grad_(True)
        Rg, Tg = R.clone().requires_grad_(True), T.clone().requires_grad_(True)
        m = Meshes([v], [meshes.shared_faces()]).extend(N)
        frags = rast(meshes_world=m, R=Rg, T=Tg)
        assert isinstance(frags, _LazyFragments)
        if not lazy:
            frags.materialize()  # the modular rasterizer for every field
        z = frags.zbuf
        (torch.relu(z[..., 0]) * go).sum().backward()
        torch.cuda.synchronize()
        return z.detach(), v.grad, Rg.grad, Tg.grad

    zl, *gl = run(True)
    zm, *gm = run(False)
    assert zl.shape == (N, H, W, 1)
    assert torch.equal(zl, zm), "fused zbuf differs from the modular rasterizer's"
    cov = int((zl >= 0).sum())
    print(f"[lazy zbuf] {camera}: covered {cov} of {zl.numel()} pixels, bitwise equal")
    assert cov > 0.02 * zl.numel()
    # the oracle: the same relu(zbuf) loss on the CPU restatement (and its float64 shadow)
    verts_c, faces_c = v0.cpu(), meshes.shared_faces().cpu()
    Rc, Tc, goc = R.cpu(), T.cpu(), go.cpu()

    def oracle(precision):
        vo = verts_c.clone().requires_grad_(True)
        Ro, To = Rc.clone().requires_grad_(True), Tc.clone().requires_grad_(True)
        ref = O.render_ref(vo, faces_c, Ro, To, intr.expand(N, 4).contiguous(), H, W, z_clip=z_clip,
                           precision=precision)
        (torch.relu(ref["zbuf"][..., 0]) * goc.to(ref["zbuf"].dtype)).sum().backward()
        return ref["zbuf"].detach(), vo.grad, Ro.grad, To.grad

    ref, r64, spread = oracle_runs(oracle, seeds=1)
    assert torch.equal(zl.cpu(), ref[0]), "zbuf differs from the oracle's"
    for nm, a, b, i in zip(("verts", "R", "T"), gl, gm, (1, 2, 3)):
        report(f"lazy zbuf {camera} grad {nm} (fused depth backward)", a, ref[i], ref64=r64[i], sens=spread[i])
        report(f"lazy zbuf {camera} grad {nm} (modular raster backward)", b, ref[i], ref64=r64[i], sens=spread[i])


def test_pose_loss_rgba_slices_match_torch():
    g = torch.Generator().manual_seed(11)
    shape = (3, 41, 37)
    depth = torch.rand(shape, generator=g)
    depth_ref = depth + (torch.rand(shape, generator=g) - 0.5) * 0.3
    mask = torch.rand(shape, generator=g) > 0.3
    sil_img = torch.rand(shape + (4,), generator=g)
    col_img = torch.rand(shape + (4,), generator=g)
    rgb_ref = torch.rand(shape + (3,), generator=g)
    dr_, sr_, cr_ = (t.clone().requires_grad_(True) for t in (depth, sil_img, col_img))
    ref = (torch.nn.L1Loss()(sr_[..., 3], mask.float()) +
           torch.nn.HuberLoss(delta=0.05)(torch.masked_select(dr_, mask), torch.masked_select(depth_ref, mask)) +
           0.01 * torch.nn.MSELoss()(cr_[..., :3], rgb_ref))
    ref.backward()
    dg, sg, cg = (t.to(DEV).requires_grad_(True) for t in (depth, sil_img, col_img))
    tot = pose_loss(dg, sg[..., 3], cg[..., :3], mask.to(DEV), depth_ref.to(DEV), rgb_ref.to(DEV))
    tot.backward()
    print(f"[parity] pose_loss on RGBA slices: {float(tot):.9g} vs torch {float(ref):.9g}")
    assert abs(float(tot) - float(ref)) <= 1e-5 * abs(float(ref))
    report("pose_loss RGBA-slice grad depth", dg.grad, dr_.grad, tol=1e-6)
    report("pose_loss RGBA-slice grad sil image", sg.grad, sr_.grad, tol=1e-6)
    report("pose_loss RGBA-slice grad colour image", cg.grad, cr_.grad, tol=1e-6)
    assert not sg.grad[..., :3].any() and not cg.grad[..., 3].any()


def test_quaternion_to_matrix_kernel():
    g = torch.Generator().manual_seed(2)
    q7 = torch.randn(37, 7, generator=g)
    qt = q7.clone().requires_grad_(True)
    Rt = quaternion_to_matrix_torch(qt[:, 3:])
    gR = torch.randn(Rt.shape, generator=g)
    (Rt * gR).sum().backward()
    qg = q7.to(DEV).requires_grad_(True)
    Rg = quaternion_to_matrix(qg[:, 3:])  # the pose's quaternion slice, rows 7 floats apart
    (Rg * gR.to(DEV)).sum().backward()
    report("quaternion_to_matrix R", Rg, Rt, tol=1e-6)
    report("quaternion_to_matrix grad q", qg.grad, qt.grad, tol=1e-5)
    # the torch formula on the same device agrees to float32 rounding
    report("quaternion_to_matrix R vs torch on GPU", Rg, quaternion_to_matrix_torch(q7.to(DEV)[:, 3:]), tol=1e-6)


def test_soft_silhouette_bench_config_vs_oracle():
    """bench.py --mode soft's workload; the oracle on views 0 and 40 of the 64 (loss restricted to them)."""
    H = W = 128
    K = 50
    sigma = 1e-4
    blur = math.log(1.0 / 1e-4 - 1.0) * sigma
    verts0, faces, _ = mesh_arrays("cow")
    c = verts0.mean(0)
    verts = (verts0 - c) / (verts0 - c).abs().max()
    nv = 64
    elev = torch.linspace(0, 360, nv)
    azim = torch.linspace(-180, 180, nv)
    R, T = look_at_view_transform(dist=2.7, elev=elev, azim=azim)
    idx = [0, 40]
    g = torch.Generator().manual_seed(3)
    target = (torch.rand(len(idx), H, W, generator=g) > 0.5).float()
    # GPU: every view rendered, the loss over the two
    v = verts.to(DEV).requires_grad_(True)
    Rd, Td = R.to(DEV).contiguous(), T.to(DEV).contiguous()
    cams = PerspectiveCameras(device=DEV, R=Rd, T=Td)
    rs = RasterizationSettings(image_size=H, blur_radius=blur, faces_per_pixel=K, perspective_correct=False)
    ren = MeshRenderer(rasterizer=MeshRasterizer(cameras=cams, raster_settings=rs),
                       shader=SoftSilhouetteShader(blend_params=BlendParams(sigma=sigma)))
    img = ren(Meshes([v], [faces.to(DEV)]).extend(nv), cameras=cams, R=Rd, T=Td)
    ws = img.grad_fn.saved_tensors[6]  # (read before the backward frees the saved tensors)
    sel = img[idx, ..., 3]
    ((sel - target.to(DEV)) ** 2).mean().backward()
    torch.cuda.synchronize()
    # the workspace's counters: the K-deep raster walked some tiles near-to-far (> 64 listed faces)
    out8 = (ctypes.c_int32 * 8)()
    _lib.check(_lib.load().mr_workspace_counters(_lib.ptr(ws), nv, nv * faces.shape[0], H, W, 0,
                                                 ctypes.cast(out8, ctypes.c_void_p), _lib.stream_handle(DEV)))
    print(f"[soft bench config] non-empty tiles {out8[1]}, kept fragments {out8[3]}, tiles walked near-to-far {out8[6]}")
    assert out8[6] > 0, "the depth-ordered walk never ran"
    # oracle on the two views
    intr = torch.tensor([[1.0, 0.0, 1.0, 0.0]]).expand(len(idx), 4).contiguous()
    Rc, Tc = R[idx], T[idx]

    def run(precision):
        vo = verts.clone().requires_grad_(True)  # the f64 shadow promotes inside render_ref
        ref = O.render_ref(vo, faces, Rc, Tc, intr, H, W, persp=False, K=K, blur=blur, clip=True, sigma_sil=sigma,
                           light={"kind": "ambient", "ambient": (1.0, 1.0, 1.0)}, precision=precision)
        ((ref["sil"] - target.to(ref["sil"].dtype)) ** 2).mean().backward()
        return ref["sil"].detach(), vo.grad

    ref, r64, spread = oracle_runs(run, seeds=1)
    report("soft bench config silhouette (views 0, 40)", sel.detach(), ref[0], ref64=r64[0], sens=spread[0])
    report("soft bench config vertex grad", v.grad, ref[1], ref64=r64[1], sens=spread[1])


def test_c3_three_calls_share_one_raster():
    """camera_pose_optimizer.py:244,248,250: the rasterizer's zbuf, the silhouette render and the Phong render of
    the same meshes / R / T / cameras / settings. The second and third calls re-shade the first call's raster
    (mr_render_reshade). Outputs bitwise, and pose / vertex gradients bitwise, against three independent passes."""
    from torch_renderer_amd import kernels as Kn
    from torch_renderer_amd.mesh_renderer import PointLights, SoftPhongShader
    from torch_renderer_amd.transforms import matrix_to_quaternion

    H = W = 256
    N = 6
    base = load_asset("cow", device=DEV)
    v0, f0 = base.shared_verts().detach(), base.shared_faces()
    cams = FoVPerspectiveCameras(device=DEV)
    blend = BlendParams(sigma=1e-4, gamma=1e-4, background_color=(0, 0, 0))
    rs = RasterizationSettings(image_size=H, blur_radius=0.0, faces_per_pixel=1)
    sil_r = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs), SoftSilhouetteShader(blend_params=blend))
    rast = MeshRasterizer(cameras=cams, raster_settings=rs)
    lights = PointLights(device=DEV, location=[[0.0, 0.0, -3.0]])
    phong = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs),
                         SoftPhongShader(device=DEV, cameras=cams, lights=lights, blend_params=blend))
    R0, T0 = look_at_view_transform(0.7, torch.linspace(10, 50, N), torch.linspace(0, 300, N), device=DEV)
    q0 = torch.cat((T0, matrix_to_quaternion(R0)), -1)
    g = torch.Generator().manual_seed(9)
    gd, gs, gc = ((torch.rand(N, H, W, generator=g) - 0.5).to(DEV), (torch.rand(N, H, W, generator=g) - 0.5).to(DEV),
                  (torch.rand(N, H, W, 3, generator=g) - 0.5).to(DEV))

    def step(enabled):
        Kn._RESHADE["enabled"] = enabled
        Kn._RESHADE["entry"] = None
        try:
            # the shared vertices require grad too: three backwards accumulate into the one workspace's
            # face totals (the first over the forward's clear, the later ones clear them again)
            v = v0.clone().requires_grad_(True)
            meshes = Meshes([v], [f0], base.textures).extend(N)
            q = q0.clone().requires_grad_(True)
            R = quaternion_to_matrix(q[:, 3:])
            T = q[:, :3]
            depth = torch.relu(rast(meshes_world=meshes, R=R, T=T).zbuf[..., 0])
            reused_after_sil = None
            sil = sil_r(meshes, R=R, T=T)[..., 3]
            ent = Kn._RESHADE["entry"]
            reused_after_sil = None if ent is None else len(ent["served"])
            color = phong(meshes, R=R, T=T)[..., :3]
            ((depth * gd).sum() + (sil * gs).sum() + (color * gc).sum()).backward()
            torch.cuda.synchronize()
            return (depth.detach(), sil.detach(), color.detach(), q.grad.detach().clone(), v.grad.clone()), reused_after_sil
        finally:
            Kn._RESHADE["enabled"] = True
            Kn._RESHADE["entry"] = None

    shared, served = step(True)
    indep, served_off = step(False)
    print(f"[reshade] shadings served by the first raster: {served} (disabled: {served_off})")
    assert served == 2 and served_off == 1
    assert shared[4].abs().max() > 0
    for nm, a, b in zip(("depth", "silhouette", "colour", "pose grad", "vertex grad"), shared, indep):
        assert torch.equal(a, b), f"{nm} differs between the shared raster and three passes"


def _icosahedron():
    """12 vertices, 20 faces (outward winding), slightly perturbed so no two faces tie exactly."""
    p = (1.0 + 5 ** 0.5) / 2.0
    v = torch.tensor([[-1, p, 0], [1, p, 0], [-1, -p, 0], [1, -p, 0], [0, -1, p], [0, 1, p], [0, -1, -p],
                      [0, 1, -p], [p, 0, -1], [p, 0, 1], [-p, 0, -1], [-p, 0, 1]], dtype=torch.float32)
    f = torch.tensor([[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2],
                      [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5],
                      [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]], dtype=torch.int64)
    g = torch.Generator().manual_seed(5)
    return v + (torch.rand(v.shape, generator=g) - 0.5) * 0.05, f


def test_large_faces_deterministic_vs_oracle():
    """Faces far larger than a tile (an icosahedron filling a 128x128 image: ~20 tiles per face, so each
    face total is the sum of ~60 (record, tile) runs whose fixed-point atomics arrive in a different order
    every run): vertex and pose gradients against the oracle within the per-entry bars, and bitwise equal
    over two runs. (Round 4 gave such faces rows in an overflow pool; round 5 sums in fixed point.)"""
    from tests.helpers import canonical_views
    from torch_renderer_amd import kernels as Kn

    verts, faces = _icosahedron()
    N, H, W = 3, 128, 128
    R, T, intr, _ = canonical_views(verts, N, H, W, dist=4.0)
    gen = torch.Generator().manual_seed(2)
    gD = torch.rand(N, H, W, generator=gen) * 2 - 1
    gS = torch.rand(N, H, W, generator=gen) * 2 - 1
    gC = torch.rand(N, H, W, 3, generator=gen) * 2 - 1
    light = dict(O.DEFAULT_LIGHT)

    def flat(precision):
        vr, Rr, Tr = (x.clone().requires_grad_(True) for x in (verts, R, T))
        ref = O.render_ref(vr, faces, Rr, Tr, intr, H, W, light=light, precision=precision)
        dt = ref["rgba"].dtype
        ((ref["depth"] * gD.to(dt)).sum() + (ref["sil"] * gS.to(dt)).sum() +
         (ref["rgba"][..., :3] * gC.to(dt)).sum()).backward()
        return ref["depth"].detach(), ref["rgba"][..., :3].detach(), vr.grad, Rr.grad, Tr.grad

    ref, r64, sp = oracle_runs(flat)

    def gpu():
        cfg = Kn.ShadeConfig(H=H, W=W)
        vg, Rg, Tg = (x.to(DEV).requires_grad_(True) for x in (verts, R, T))
        out = Kn.render_views(vg, Rg, Tg, faces.to(DEV), intr.to(DEV), torch.zeros(1, 3, device=DEV), cfg)
        ((out["depth"] * gD.to(DEV)).sum() + (out["sil"] * gS.to(DEV)).sum() + (out["rgb"] * gC.to(DEV)).sum()).backward()
        torch.cuda.synchronize()
        return out, (vg.grad, Rg.grad, Tg.grad)

    out, g1 = gpu()
    report("large faces depth", out["depth"], ref[0], rel_above_one=False, ref64=r64[0], sens=sp[0])
    report("large faces rgb", out["rgb"], ref[1], rel_above_one=False, ref64=r64[1], sens=sp[1])
    for i, nm in enumerate(("verts", "R", "T")):
        report(f"large faces grad {nm}", g1[i], ref[2 + i], ref64=r64[2 + i], sens=sp[2 + i])
    _, g2 = gpu()
    for a, b, nm in zip(g1, g2, ("verts", "R", "T")):
        assert torch.equal(a, b), f"{nm} gradient differs between two runs"
