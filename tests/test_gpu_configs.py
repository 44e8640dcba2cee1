"""GPU parity at every BASELINE.json configuration (C1-C5) and at the benchmarked workload.

Each test runs the HIP path at the configuration's full size. The oracle (C naive rasterizer +
torch-CPU restatement of PyTorch3D's shading, blending and autograd) is run where it finishes in
seconds — a few views, or a pixel window of a large image — and the rest of the batch is checked
through size-independent properties:
  * the fused render's pix_to_face equals the modular rasterizer's (mr_rasterize_meshes, K=1)
    bit for bit, for every view;
  * no NaN/inf anywhere; uncovered pixels hold exactly the background (depth 0, silhouette 0,
    rgb = background colour);
  * per-view results do not depend on the batch they are rendered in (bitwise);
  * a view-sharded batch equals the unsharded one (bitwise images, global packed ids, pose grads).
Bars: pix_to_face bit-exact; images and gradients within 1e-4 absolute, scaled by the value's
magnitude when it exceeds 1 (tests/helpers.report prints both numbers).
"""
import math

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import canonical_views, cv_to_p3d, intr_from_K, mesh_arrays, oracle_runs, report
from torch_renderer_amd import Meshes, TexturesUV, TexturesVertex
from torch_renderer_amd.cameras import FoVPerspectiveCameras, PerspectiveCameras
from torch_renderer_amd.kernels import ShadeConfig, rasterize_meshes_fwd
from torch_renderer_amd.mesh_renderer import (AmbientLights, BlendParams, MeshRasterizer, MeshRenderer, PointLights,
                                              RasterizationSettings, SoftPhongShader, SoftSilhouetteShader)
from torch_renderer_amd.torch_renderer import DepthColorRender, render_mesh_batch
from torch_renderer_amd.transforms import (look_at_view_transform, matrix_to_quaternion, opencv_to_pytorch3d,
                                           quaternion_to_matrix)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
LIGHT = (0.0, 0.0, -3.0)


def _uv_texture(d):
    img = torch.from_numpy(d["texture_u8"].astype(np.float32) / 255.0)
    vuv = torch.from_numpy(d["verts_uvs"]).float()
    fuv = torch.from_numpy(d["faces_uvs"]).long()
    return img, vuv, fuv


def _modular_p2f(verts, faces, R_cv, t_cv, K, H, W):
    """mr_rasterize_meshes (K=1) pix_to_face of the same views (the PyTorch3D _C boundary)."""
    cams = PerspectiveCameras(focal_length=((K[0, 0].item(), K[1, 1].item()),),
                              principal_point=((K[0, 2].item(), K[1, 2].item()),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]), device=DEV)
    Rp, Tp = opencv_to_pytorch3d(R_cv.to(DEV), t_cv.to(DEV))
    N = R_cv.shape[0]
    m = Meshes([verts.to(DEV)], [faces.to(DEV)]).extend(N)
    with torch.no_grad():
        return MeshRasterizer(cams, RasterizationSettings(image_size=(H, W)))(m, R=Rp, T=Tp).pix_to_face[..., 0]


def _check_background(out, p2f, bg):
    """Uncovered pixels: depth 0, silhouette 0, rgb = background; nothing non-finite."""
    empty = p2f < 0
    for k in ("depth", "sil", "rgb"):
        assert torch.isfinite(out[k]).all(), f"{k} has non-finite values"
    assert torch.equal(out["depth"][empty], torch.zeros_like(out["depth"][empty]))
    assert torch.equal(out["sil"][empty], torch.zeros_like(out["sil"][empty]))
    bgt = torch.tensor(bg, device=out["rgb"].device).expand(int(empty.sum()), 3)
    assert torch.equal(out["rgb"][empty], bgt)
    assert (~empty).any(), "degenerate view: nothing covered"


def _oracle_views(verts, faces, R_cv, t_cv, K, H, W, texture, grads, bg=(1.0, 1.0, 1.0), window=None,
                  precision="f32"):
    """Reference fwd+bwd (CPU) of views given as OpenCV poses: outputs, leaf grads (verts, R, t).
    precision="f64": the oracle's float64 shadow (tests.helpers.report's conditioning measure)."""
    N = R_cv.shape[0]
    vr = verts.clone().requires_grad_(True)
    Rr = R_cv.clone().requires_grad_(True)
    tr = t_cv.clone().requires_grad_(True)
    Rp, Tp = cv_to_p3d(Rr, tr)
    ref = O.render_ref(vr, faces, Rp, Tp, intr_from_K(K, H, W, N), H, W, texture=texture, bg=bg, window=window,
                       precision=precision)
    gD, gS, gC = grads
    ((ref["depth"] * gD).sum() + (ref["sil"] * gS).sum() + (ref["rgba"][..., :3] * gC).sum()).backward()
    return ref, (vr.grad, Rr.grad, tr.grad)


def _oracle_flat(*a, **kw):
    """_oracle_views as a flat tuple for tests.helpers.oracle_runs: (depth, sil, rgb, grad verts,
    grad R_cv, grad t_cv, pix_to_face[..., 0])."""
    ref, g = _oracle_views(*a, **kw)
    return (ref["depth"], ref["sil"], ref["rgba"][..., :3]) + tuple(g) + (ref["p2f"][..., 0],)


_NAMES = ("depth", "sil", "rgb", "grad verts", "grad R_cv", "grad t_cv")


def _report_all(tag, gots, ref, r64, sp):
    """report() every output and gradient against the f32 oracle, its f64 shadow and the spread."""
    for i, (nm, a) in enumerate(zip(_NAMES, gots)):
        report(f"{tag} {nm}", a, ref[i], ref64=r64[i], sens=sp[i])


def _gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, grads, want_p2f=True, bg=(1.0, 1.0, 1.0)):
    """Fused drop-in render (DepthColorRender's path, OpenCV poses) fwd+bwd on the GPU."""
    r = DepthColorRender(K.to(DEV), (H, W), device=DEV)
    v = verts.to(DEV).requires_grad_(True)
    Rg = R_cv.to(DEV).requires_grad_(True)
    tg = t_cv.to(DEV).requires_grad_(True)
    m = Meshes([v], [faces.to(DEV)], tex).extend(R_cv.shape[0])
    cfg = ShadeConfig(H=H, W=W, light_location=LIGHT, want_p2f=want_p2f, background=bg)
    out = render_mesh_batch(m, r._cameras, (H, W), Rg, tg, cfg, pose_cv=True)
    if grads is not None:
        gD, gS, gC = (g.to(DEV) for g in grads)
        ((out["depth"] * gD).sum() + (out["sil"] * gS).sum() + (out["rgb"] * gC).sum()).backward()
    return out, (v.grad, Rg.grad, tg.grad)


def _upstream(N, H, W, seed=1, window=None):
    g = torch.Generator().manual_seed(seed)
    gD = torch.rand(N, H, W, generator=g) * 2 - 1
    gS = torch.rand(N, H, W, generator=g) * 2 - 1
    gC = torch.rand(N, H, W, 3, generator=g) * 2 - 1
    if window is not None:
        y0, y1, x0, x1 = window
        m = torch.zeros(H, W)
        m[y0:y1, x0:x1] = 1.0
        gD, gS, gC = gD * m, gS * m, gC * m[..., None]
    return gD, gS, gC


def test_c1_sphere_256_one_view():
    """C1: data/sphere.obj, 1 view, 256x256 (white vertex texture: its map_Kd is missing)."""
    H = W = 256
    verts, faces, _ = mesh_arrays("sphere")
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, 1, H, W)
    white = torch.ones_like(verts)
    grads = _upstream(1, H, W)
    ref, r64, sp = oracle_runs(lambda p: _oracle_flat(verts, faces, R_cv, t_cv, K, H, W, ("vertex", white), grads,
                                                      precision=p))
    out, gg = _gpu_views(verts, faces, TexturesVertex([white.to(DEV)]), R_cv, t_cv, K, H, W, grads)
    assert torch.equal(out["pix_to_face32"].cpu().long(), ref[6])
    _report_all("C1", (out["depth"], out["sil"], out["rgb"]) + tuple(gg), ref, r64, sp)
    _check_background(out, out["pix_to_face32"], (1.0, 1.0, 1.0))


def test_c2_teapot_512_batch8_forward():
    """C2: data/teapot.obj, 512x512, batch 8, forward. Oracle on 2 of the views; fused == modular
    pix_to_face and background checks on all 8."""
    H = W = 512
    N = 8
    verts, faces, _ = mesh_arrays("teapot")
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, N, H, W)
    g = torch.Generator().manual_seed(7)
    vcol = torch.rand(verts.shape, generator=g)
    out, _ = _gpu_views(verts, faces, TexturesVertex([vcol.to(DEV)]), R_cv, t_cv, K, H, W, None)
    p2f = out["pix_to_face32"].long()
    assert torch.equal(p2f, _modular_p2f(verts, faces, R_cv, t_cv, K, H, W))
    _check_background(out, p2f, (1.0, 1.0, 1.0))
    sel = [0, 5]
    grads = _upstream(2, H, W)
    ref, _ = _oracle_views(verts, faces, R_cv[sel], t_cv[sel], K, H, W, ("vertex", vcol), grads)
    r64, _ = _oracle_views(verts, faces, R_cv[sel], t_cv[sel], K, H, W, ("vertex", vcol), grads, precision="f64")
    Fn = faces.shape[0]
    for j, n in enumerate(sel):
        exp = ref["p2f"][j, ..., 0]
        exp = torch.where(exp >= 0, exp - j * Fn + n * Fn, exp)  # packed id of view n in the batch of 8
        assert torch.equal(p2f[n].cpu(), exp), f"view {n}: pix_to_face differs from the oracle"
        report(f"C2 view{n} depth", out["depth"][n], ref["depth"][j], ref64=r64["depth"][j])
        report(f"C2 view{n} sil", out["sil"][n], ref["sil"][j], ref64=r64["sil"][j])
        report(f"C2 view{n} rgb", out["rgb"][n], ref["rgba"][j, ..., :3], ref64=r64["rgba"][j, ..., :3])


def test_metric_config_cow_512_64views_fwd_bwd():
    """The benchmarked workload (bench.py): cow + its UV texture, 512x512, 64 views, fwd+bwd through
    DepthColorRender's fused path. All 64 views: fused p2f == modular p2f, exact background, no NaN.
    Views 0 and 37: rendered alone they equal their slice of the 64-view batch bitwise (images and
    per-view pose gradients), and match the oracle (p2f exact, images and grads within the bars)."""
    H = W = 512
    N = 64
    verts, faces, d = mesh_arrays("cow")
    img, vuv, fuv = _uv_texture(d)
    tex = TexturesUV(maps=[img.to(DEV)], faces_uvs=[fuv.to(DEV)], verts_uvs=[vuv.to(DEV)])
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, N, H, W, dist=0.5)
    grads = _upstream(N, H, W)
    out, gg = _gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, grads)
    p2f = out["pix_to_face32"].long()
    assert torch.equal(p2f, _modular_p2f(verts, faces, R_cv, t_cv, K, H, W))
    _check_background(out, p2f, (1.0, 1.0, 1.0))
    for gr in gg:
        assert torch.isfinite(gr).all()
    assert (p2f >= 0).sum() > 0.02 * N * H * W
    sel = [0, 37]
    sub_grads = tuple(x[sel] for x in grads)
    out2, gg2 = _gpu_views(verts, faces, tex, R_cv[sel], t_cv[sel], K, H, W, sub_grads)
    Fn = faces.shape[0]
    for j, n in enumerate(sel):
        for k in ("depth", "sil", "rgb"):
            assert torch.equal(out2[k][j], out[k][n]), f"view {n} {k} depends on the batch"
        q = out2["pix_to_face32"][j].long()
        assert torch.equal(torch.where(q >= 0, q - j * Fn + n * Fn, q), p2f[n])
        assert torch.equal(gg2[1][j], gg[1][n]) and torch.equal(gg2[2][j], gg[2][n]), \
            f"view {n}: pose gradients depend on the batch"
    ref, r64, sp = oracle_runs(lambda p: _oracle_flat(verts, faces, R_cv[sel], t_cv[sel], K, H, W,
                                                      ("uv", vuv, fuv, img), sub_grads, precision=p))
    assert torch.equal(out2["pix_to_face32"].cpu().long(), ref[6])
    _report_all("metric", (out2["depth"], out2["sil"], out2["rgb"]) + tuple(gg2), ref, r64, sp)


def _pose_model_step(meshes, verts_leaf, cams, q_init, refs, lr=1e-3):
    """camera_pose_optimizer.py:237-305 one step, with the caller's exact keyword calls."""
    rasterizer, silhouette_renderer, phong_renderer = refs["renderers"]
    q = torch.nn.Parameter(q_init.clone())
    opt = torch.optim.Adam([q], lr=lr)
    opt.zero_grad()
    R = quaternion_to_matrix(q[:, 3:])
    T = q[:, :3]
    fragments = rasterizer(meshes_world=meshes, R=R, T=T)
    depth = torch.relu(fragments.zbuf[..., 0])
    silhouette = silhouette_renderer(meshes, R=R, T=T)[..., 3]
    color = phong_renderer(meshes, R=R, T=T)[..., :3]
    loss = _calc_loss(depth, silhouette, color, refs)
    loss.backward()
    g = q.grad.detach().clone()
    opt.step()
    return loss.detach(), g, q.detach().clone(), (depth.detach(), silhouette.detach(), color.detach())


def _calc_loss(depth, depth_mask, color, refs):
    """camera_pose_optimizer.py:257-276 (the wandb logging dropped)."""
    mask = refs["sil"]
    sil_loss = torch.nn.functional.l1_loss(depth_mask, mask.float())
    color_loss = torch.nn.functional.mse_loss(color, refs["rgb"])
    depth_gt = torch.masked_select(refs["depth"], mask)
    d = torch.masked_select(depth, mask)
    hloss = torch.nn.functional.huber_loss(d, depth_gt, delta=0.05)
    return sil_loss + hloss + color_loss * 0.01


def test_c3_camera_pose_optimizer_step_cow_512():
    """C3: camera_pose_optimizer.py's step at 512x512 on the cow: FoVPerspectiveCameras,
    look_at_view_transform(0.7, 30, 60), 7-vector pose (T, quaternion) + noise, the three renders
    called exactly as the reference calls them (rasterizer(meshes_world=..., R=, T=) etc.), the
    L1 + Huber + 0.01 MSE loss, backward and one Adam step. Compared with the same step on the
    oracle (loss, pose gradient, updated pose, rendered depth / silhouette / colour)."""
    H = W = 512
    from torch_renderer_amd.assets import load_asset

    meshes = load_asset("cow", device=DEV)
    cams = FoVPerspectiveCameras(device=DEV)
    blend = BlendParams(sigma=1e-4, gamma=1e-4, background_color=(0, 0, 0))
    rs = RasterizationSettings(image_size=512, blur_radius=0.0, faces_per_pixel=1)
    silhouette_renderer = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs),
                                       SoftSilhouetteShader(blend_params=blend))
    rasterizer = MeshRasterizer(cameras=cams, raster_settings=rs)
    lights = PointLights(device=DEV, location=[[0.0, 0.0, -3.0]])
    phong = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs),
                         SoftPhongShader(device=DEV, cameras=cams, lights=lights, blend_params=blend))
    R, T = look_at_view_transform(0.7, 30.0, 60.0, device=DEV)
    q_ref = torch.cat((T, matrix_to_quaternion(R)), -1)
    with torch.no_grad():
        sil_ref = silhouette_renderer(meshes_world=meshes, R=R, T=T)
        depth_ref = rasterizer(meshes_world=meshes, R=R, T=T).zbuf[..., 0]
        rgb_full = phong(meshes_world=meshes, R=R, T=T)[..., :3]
    depth_ref = torch.where(depth_ref == -1.0, torch.zeros_like(depth_ref), depth_ref)
    sil_mask = depth_ref != 0.0
    rgb_ref = torch.where(sil_mask[..., None], rgb_full, torch.zeros_like(rgb_full))
    assert sil_mask.sum() > 1000 and (sil_ref[..., 3] != 0).sum() >= sil_mask.sum()
    gen = torch.Generator().manual_seed(0)
    q0 = q_ref.cpu() + torch.randn(1, 7, generator=gen) * 0.03
    refs = {"renderers": (rasterizer, silhouette_renderer, phong), "sil": sil_mask, "depth": depth_ref,
            "rgb": rgb_ref}
    loss, g, q1, imgs = _pose_model_step(meshes, None, cams, q0.to(DEV), refs)

    # oracle: the same step on the CPU restatement (FoV camera: ax = ay = 1/tan(30 deg), znear 1,
    # zfar 100; specular camera centre = the camera object's own (R = I, T = 0) -> world origin)
    verts, faces, d = mesh_arrays("cow")
    img, vuv, fuv = _uv_texture(d)
    t = 1.0 / math.tan(math.radians(30.0))
    intr = torch.tensor([[t, 0.0, t, 0.0]])
    qo = torch.nn.Parameter(q0.clone())
    opt = torch.optim.Adam([qo], lr=1e-3)
    opt.zero_grad()
    Ro = quaternion_to_matrix(qo[:, 3:])
    To = qo[:, :3]
    light = dict(O.DEFAULT_LIGHT)
    refo = O.render_ref(verts, faces, Ro, To, intr, H, W, texture=("uv", vuv, fuv, img), light=light,
                        bg=(0.0, 0.0, 0.0), z_clip=0.5)
    refs_c = {"sil": sil_mask.cpu(), "depth": depth_ref.cpu(), "rgb": rgb_ref.cpu()}
    depth_o = torch.relu(refo["zbuf"][..., 0])
    loss_o = _calc_loss(depth_o, refo["sil"], refo["rgba"][..., :3], refs_c)
    loss_o.backward()
    go = qo.grad.detach().clone()
    opt.step()
    report("C3 depth", imgs[0], depth_o)
    report("C3 silhouette", imgs[1], refo["sil"])
    report("C3 colour", imgs[2], refo["rgba"][..., :3])
    report("C3 loss", loss, loss_o)
    report("C3 pose grad", g, go)
    # one Adam step from the same state moves each coordinate by ~lr * sign(grad)
    report("C3 pose after Adam", q1, qo.detach(), tol=1e-6)


def test_c4_dolphin_1024_64views_sharded_equals_unsharded():
    """C4 (batch_rendering_test.py:320-328): dolphin, 1024x1024, 64 views sharded across 8 ranks. The
    batch rendered as C4's 8 shards of 8 views (distributed.shard_views(..., world_size=8); global packed
    ids via global_view_offset), one shard after another on this GPU, equals the unsharded render
    bitwise: images, pix_to_face, per-view pose gradients; the shared vertex gradient (the sum of the
    8 shards' gradients, what allreduce_grads forms) matches within the bar. Fused p2f == modular p2f on
    all views."""
    from torch_renderer_amd import distributed as D

    H = W = 1024
    N = 64
    verts, faces, _ = mesh_arrays("dolphin")
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, N, H, W)
    white = TexturesVertex([torch.ones_like(verts).to(DEV)])
    grads = _upstream(N, H, W)
    full, gfull = _gpu_views(verts, faces, white, R_cv, t_cv, K, H, W, grads)
    Fn = faces.shape[0]
    p2f = full["pix_to_face32"].long()
    assert torch.equal(p2f, _modular_p2f(verts, faces, R_cv, t_cv, K, H, W))
    _check_background(full, p2f, (1.0, 1.0, 1.0))
    vsum = torch.zeros_like(gfull[0])
    world = 8
    for rank in range(world):
        Rs, ts = D.shard_views(R_cv, t_cv, rank=rank, world_size=world)
        gs = D.shard_views(*grads, rank=rank, world_size=world)
        s0 = D.global_view_offset(N, rank=rank, world_size=world)
        assert Rs.shape[0] == N // world
        sh, gsh = _gpu_views(verts, faces, white, Rs, ts, K, H, W, gs)
        n = Rs.shape[0]
        for k in ("depth", "sil", "rgb"):
            assert torch.equal(sh[k], full[k][s0:s0 + n]), f"shard {rank}: {k} differs"
        q = sh["pix_to_face32"].long()
        assert torch.equal(torch.where(q >= 0, q + s0 * Fn, q), p2f[s0:s0 + n])
        assert torch.equal(gsh[1], gfull[1][s0:s0 + n]) and torch.equal(gsh[2], gfull[2][s0:s0 + n])
        vsum += gsh[0]
    # inside one call each face's total is an exact fixed-point sum (order-independent); the sharded
    # gradient is instead the f32 sum of 8 per-shard vertex gradients, each rounded from its own
    # total, so it differs from the unsharded one by float rounding: its conditioning is the sum of
    # the views' absolute contributions, measured from 64 single-view renders; an 8-ulp (1e-6
    # relative) change of every view's contribution bounds the spread (tests.helpers.report)
    cond = torch.zeros_like(gfull[0])
    for n in range(N):
        _, g1 = _gpu_views(verts, faces, white, R_cv[n:n + 1], t_cv[n:n + 1], K, H, W,
                           tuple(x[n:n + 1] for x in grads), want_p2f=False)
        cond += g1[0].abs()
    report("C4 vertex grad (sum of shards)", vsum, gfull[0], sens=1e-6 * cond)


def test_c5_subdivided_sphere_1024_vertex_grads():
    """C5 (mesh_deformer.py color_train at the C5 scale): ico-sphere of F=81,920 (data/sphere.obj
    subdivided twice), 1024x1024, PerspectiveCameras(R, T) (NDC, focal 1), perspective_correct=False,
    AmbientLights, TexturesVertex colours with grad, renderer(mesh, cameras=cams[j], lights=lights)
    as mesh_deformer.py:197 calls it. Oracle on a 128x128 window crossing the silhouette edge
    (upstream gradients zero outside it, on both sides); full-size property checks."""
    from torch_renderer_amd.utils import subdivided_sphere

    H = W = 1024
    sph = subdivided_sphere(2)
    verts, faces = sph.verts_list()[0], sph.faces_list()[0]
    assert faces.shape[0] == 81920 and verts.shape[0] == 40962
    elev = torch.linspace(0, 360, 10)
    azim = torch.linspace(-180, 180, 10)
    R, T = look_at_view_transform(dist=2.0, elev=elev, azim=azim)
    cams = PerspectiveCameras(device=DEV, R=R.to(DEV), T=T.to(DEV))
    j = 3
    lights = AmbientLights(device=DEV)
    rs = RasterizationSettings(image_size=1024, blur_radius=0.0, faces_per_pixel=1, perspective_correct=False)
    renderer = MeshRenderer(MeshRasterizer(cameras=cams, raster_settings=rs),
                            SoftPhongShader(device=DEV, cameras=cams, lights=lights))
    vg = verts.to(DEV).requires_grad_(True)
    rgb = torch.full((1, verts.shape[0], 3), 0.5, device=DEV, requires_grad=True)
    g = torch.Generator().manual_seed(3)
    mesh = Meshes([vg], [faces.to(DEV)])
    mesh.textures = TexturesVertex(verts_features=torch.nn.functional.hardtanh(
        rgb + (torch.rand(rgb.shape, generator=g) * 0.5).to(DEV), min_val=0.0, max_val=1.0))
    img = renderer(mesh, cameras=cams[j], lights=lights)
    assert img.shape == (1, H, W, 4) and torch.isfinite(img).all()
    win = (400, 528, 760, 888)
    y0, y1, x0, x1 = win
    go = (torch.rand(1, H, W, 4, generator=g) * 2 - 1)
    mwin = torch.zeros(1, H, W, 1)
    mwin[:, y0:y1, x0:x1] = 1.0
    go = go * mwin
    (img * go.to(DEV)).sum().backward()
    # full-size properties: fused p2f == modular p2f; background exact
    with torch.no_grad():
        frag = MeshRasterizer(cameras=cams[j], raster_settings=rs)(Meshes([verts.to(DEV)], [faces.to(DEV)]))
        cov = frag.pix_to_face[..., 0] >= 0
        assert cov.sum() > 0.2 * H * W
        assert torch.equal(img[~cov], torch.tensor([1.0, 1.0, 1.0, 0.0], device=DEV).expand(int((~cov).sum()), 4))
    # oracle on the window
    vr = verts.clone().requires_grad_(True)
    rr = rgb.detach().cpu().clone().requires_grad_(True)
    g = torch.Generator().manual_seed(3)
    vcol = torch.nn.functional.hardtanh(rr + torch.rand(rr.shape, generator=g) * 0.5, 0.0, 1.0)[0]
    intr = torch.tensor([[1.0, 0.0, 1.0, 0.0]])
    ref = O.render_ref(vr, faces, R[j:j + 1], T[j:j + 1], intr, H, W, texture=("vertex", vcol),
                       light={"kind": "ambient", "ambient": (1.0, 1.0, 1.0)}, persp=False, window=win)
    (ref["rgba"] * go).sum().backward()
    # float64 shadow of the same (conditioning of each entry, tests.helpers.report)
    v64 = verts.clone().requires_grad_(True)
    r64 = rgb.detach().cpu().clone().requires_grad_(True)
    g = torch.Generator().manual_seed(3)
    vcol64 = torch.nn.functional.hardtanh(r64 + torch.rand(r64.shape, generator=g) * 0.5, 0.0, 1.0)[0]
    s64 = O.render_ref(v64, faces, R[j:j + 1], T[j:j + 1], intr, H, W, texture=("vertex", vcol64),
                       light={"kind": "ambient", "ambient": (1.0, 1.0, 1.0)}, persp=False, window=win,
                       precision="f64")
    (s64["rgba"] * go.double()).sum().backward()
    p2f_ref = ref["p2f"][0, y0:y1, x0:x1, 0]
    assert (p2f_ref >= 0).any() and (p2f_ref < 0).any(), "window must cross the silhouette"
    assert torch.equal(frag.pix_to_face[0, y0:y1, x0:x1, 0].cpu(), p2f_ref)
    report("C5 rgba (window)", img[0, y0:y1, x0:x1], ref["rgba"][0, y0:y1, x0:x1],
           ref64=s64["rgba"][0, y0:y1, x0:x1])
    report("C5 grad verts", vg.grad, vr.grad, ref64=v64.grad)
    report("C5 grad colours", rgb.grad, rr.grad, ref64=r64.grad)


def test_determinism_metric_config():
    """Rendering the benchmarked batch twice gives bitwise-identical images, pix_to_face, per-view
    pose gradients AND shared vertex gradients: the backward adds one gradient row per (record, tile)
    into each face's total as 64-bit fixed-point integers (order-independent integer atomics,
    mr_common.h fix_of), and the vertex gathers sum a vertex's faces in CSR order (no float atomics)."""
    H = W = 512
    N = 16
    verts, faces, d = mesh_arrays("cow")
    img, vuv, fuv = _uv_texture(d)
    tex = TexturesUV(maps=[img.to(DEV)], faces_uvs=[fuv.to(DEV)], verts_uvs=[vuv.to(DEV)])
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, N, H, W, dist=0.5)
    grads = _upstream(N, H, W)
    a, ga = _gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, grads)
    b, gb = _gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, grads)
    for k in ("depth", "sil", "rgb", "pix_to_face32"):
        assert torch.equal(a[k], b[k]), k
    assert torch.equal(ga[1], gb[1]) and torch.equal(ga[2], gb[2])
    dv = (ga[0] - gb[0]).abs().max().item()
    print(f"[determinism] vertex grad run-to-run max |diff| = {dv:.3e} (scale {ga[0].abs().max().item():.3e})")
    assert torch.equal(ga[0], gb[0]), "vertex gradients differ between two identical runs"


def test_large_image_count_scan_fill_path():
    """Tile grids above the per-view binning's LDS limit (1040x1040 = 130x130 tiles > 16384) take the
    count -> scan -> fill binning. Fused render fwd+bwd of one cow view against the oracle on a window
    crossing the silhouette (upstream gradients zero outside it on both sides), fused == modular
    pix_to_face and exact background on the whole image."""
    H = W = 1040
    verts, faces, d = mesh_arrays("cow")
    img, vuv, fuv = _uv_texture(d)
    tex = TexturesUV(maps=[img.to(DEV)], faces_uvs=[fuv.to(DEV)], verts_uvs=[vuv.to(DEV)])
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, 1, H, W, dist=0.5)
    out, _ = _gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, None)
    p2f = out["pix_to_face32"][0]
    cov = (p2f >= 0).nonzero()
    cy, cx = cov[:, 0].float().mean().item(), cov[:, 1].float().min().item()
    y0, x0 = int(cy) - 48, max(int(cx) - 16, 0)
    win = (y0, y0 + 96, x0, x0 + 96)
    grads = _upstream(1, H, W, window=win)
    out, gg = _gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, grads)
    ref, r64, sp = oracle_runs(lambda p: _oracle_flat(verts, faces, R_cv, t_cv, K, H, W, ("uv", vuv, fuv, img),
                                                      grads, window=win, precision=p))
    p2f_ref = ref[6][0, y0:y0 + 96, x0:x0 + 96]
    assert (p2f_ref >= 0).any() and (p2f_ref < 0).any(), "window must cross the silhouette"
    assert torch.equal(out["pix_to_face32"][0, y0:y0 + 96, x0:x0 + 96].cpu().long(), p2f_ref)
    crop = lambda t: t[0, y0:y0 + 96, x0:x0 + 96]  # noqa: E731
    for i, k in enumerate(("depth", "sil", "rgb")):
        report(f"1040 {k} (window)", crop(out[k]), crop(ref[i]), ref64=crop(r64[i]), sens=crop(sp[i]))
    for i, (nm, a) in enumerate(zip(("verts", "R_cv", "t_cv"), gg)):
        report(f"1040 grad {nm}", a, ref[3 + i], ref64=r64[3 + i], sens=sp[3 + i])
    assert torch.equal(out["pix_to_face32"].long(), _modular_p2f(verts, faces, R_cv, t_cv, K, H, W))
    _check_background(out, out["pix_to_face32"], (1.0, 1.0, 1.0))


def test_vertex_grads_additive_over_view_batches():
    """The shared vertex gradient of 80 views in one call equals the sum of three calls over 5, 16 and
    59 of those views within float rounding (each call's per-face totals are exact fixed-point sums,
    converted to f32 once per call), and each view's R / t gradient is bitwise the same in any batch
    (its slots' partial rows are summed as one sequence whatever the band split, i.e. whatever the
    batch size)."""
    H = W = 128
    N = 80
    verts, faces, d = mesh_arrays("cow")
    img, vuv, fuv = _uv_texture(d)
    tex = TexturesUV(maps=[img.to(DEV)], faces_uvs=[fuv.to(DEV)], verts_uvs=[vuv.to(DEV)])
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, N, H, W, dist=0.5)
    grads = _upstream(N, H, W, seed=3)
    out, (gv, gR, gt) = _gpu_views(verts, faces, tex, R_cv, t_cv, K, H, W, grads)
    acc = torch.zeros_like(gv)
    for a, b in ((0, 5), (5, 21), (21, 80)):
        texs = TexturesUV(maps=[img.to(DEV)], faces_uvs=[fuv.to(DEV)], verts_uvs=[vuv.to(DEV)])
        o, (sv, sR, st) = _gpu_views(verts, faces, texs, R_cv[a:b], t_cv[a:b], K, H, W,
                                     tuple(g[a:b] for g in grads))
        p = o["pix_to_face32"]  # packed ids: view n's faces are n * F + f
        assert torch.equal(torch.where(p >= 0, p + a * faces.shape[0], p), out["pix_to_face32"][a:b])
        assert torch.equal(sR, gR[a:b]) and torch.equal(st, gt[a:b]), (a, b)
        acc += sv
    scale = gv.abs().max().item()
    err = (acc - gv).abs().max().item()
    print(f"[view batches] vertex grad |sum of 5+16+59 views - 80 views| max {err:.3e} (scale {scale:.3e})")
    assert err <= 1e-4 * scale
