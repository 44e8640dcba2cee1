"""Host logic added for the reference callers (no GPU): Meshes in-place utilities
(mesh_deformer.py:103-104), camera indexing (:197), SubdivideMeshes / ico_sphere (the C5 mesh),
the drop-in call signatures (camera_pose_optimizer.py:175-177,244: meshes_world=...), per-call
lights/materials/blend_params, refusal of differentiable lights, and the oracle's restatement of
near-plane clipping (upstream mesh/clip.py) and the clipped-face neighbour rule."""
import inspect

import pytest
import torch

from oracle import oracle as O
from tests.helpers import mesh_arrays
from torch_renderer_amd import Meshes, TexturesUV, TexturesVertex
from torch_renderer_amd.cameras import FoVPerspectiveCameras, PerspectiveCameras
from torch_renderer_amd.mesh_renderer import (AmbientLights, BlendParams, Materials, MeshRasterizer, MeshRenderer,
                                              PointLights, RasterizationSettings, SoftPhongShader,
                                              SoftSilhouetteShader)
from torch_renderer_amd.transforms import look_at_view_transform
from torch_renderer_amd.utils import SubdivideMeshes, ico_sphere, subdivide, subdivided_sphere


def test_offset_and_scale_verts_inplace():
    v, f, _ = mesh_arrays("cow")
    m = Meshes([v.clone()], [f])
    c = m.verts_packed().mean(0)
    s = (m.verts_packed() - c).abs().max(0)[0].max()
    assert m.offset_verts_(-c) is m
    m.scale_verts_(1.0 / float(s))
    w = m.verts_packed()
    assert torch.allclose(w.mean(0), torch.zeros(3), atol=1e-6)
    assert abs((w.abs().max() - 1.0).item()) < 1e-6
    # a per-vertex offset keeps an extended batch shared
    e = Meshes([v.clone()], [f]).extend(3)
    e.offset_verts_(torch.ones_like(v))
    assert e.is_shared() and torch.equal(e.verts_list()[2], v + 1)
    two = Meshes([v.clone(), v.clone()], [f, f])
    two.scale_verts_(torch.tensor([1.0, 2.0]))
    assert torch.equal(two.verts_list()[1], v * 2)
    with pytest.raises(ValueError):
        two.offset_verts_(torch.ones(5, 3))


def test_subdivision_counts_orientation_and_midpoints():
    s = ico_sphere(2)
    v, f = s.verts_list()[0], s.faces_list()[0]
    assert (v.shape[0], f.shape[0]) == (162, 320)
    assert torch.allclose(v.norm(dim=1), torch.ones(v.shape[0]))
    c = subdivided_sphere(2)
    assert (c.verts_list()[0].shape[0], c.faces_list()[0].shape[0]) == (40962, 81920)
    # one plain SubdivideMeshes step: new vertices are edge midpoints, faces keep orientation
    tv = torch.tensor([[0.0, 0, 0], [1, 0, 0], [0, 1, 0]])
    tf = torch.tensor([[0, 1, 2]])
    nv, nf = subdivide(tv, tf)
    assert nf.shape == (4, 3) and nv.shape == (6, 3)
    tri = nv[nf]
    n = torch.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0], dim=1)
    assert (n[:, 2] > 0).all() and torch.allclose(n[:, 2], torch.full((4,), 0.25))
    m2 = SubdivideMeshes()(Meshes([tv], [tf]))
    assert torch.equal(m2.verts_list()[0], nv)


def test_camera_indexing():
    R, T = look_at_view_transform(dist=2.0, elev=torch.linspace(0, 360, 10), azim=torch.linspace(-180, 180, 10))
    cams = PerspectiveCameras(R=R, T=T)
    c3 = cams[3]
    assert len(c3) == 1 and torch.equal(c3.R, R[3:4]) and torch.equal(c3.T, T[3:4])
    assert torch.equal(c3.ndc_affine((64, 64)), cams.ndc_affine((64, 64))[:1])
    with pytest.raises(IndexError):
        cams[10]


def test_reference_call_signatures():
    """The reference calls rasterizer(meshes_world=...) and renderer(meshes_world=...)."""
    assert list(inspect.signature(MeshRasterizer.forward).parameters)[1] == "meshes_world"
    assert list(inspect.signature(MeshRenderer.forward).parameters)[1] == "meshes_world"
    v, f, _ = mesh_arrays("sphere")
    cams = FoVPerspectiveCameras()
    R, T = look_at_view_transform(3.0, 10.0, 20.0)
    with pytest.raises(RuntimeError):  # reaches the HIP path, which refuses CPU tensors
        MeshRasterizer(cams, RasterizationSettings(image_size=16))(meshes_world=Meshes([v], [f]), R=R, T=T)


def test_per_call_lights_materials_blend_override_the_shader():
    cams = PerspectiveCameras()
    sh = SoftPhongShader(cameras=cams, lights=PointLights(location=[[0.0, 0.0, -3.0]]))
    r = MeshRenderer(MeshRasterizer(cams, RasterizationSettings(image_size=8)), sh)
    rs = r.rasterizer.raster_settings
    base = r._config(cams, rs, 8, 8, {})
    assert base.light_kind == 0 and base.light_location == (0.0, 0.0, -3.0)
    cfg = r._config(cams, rs, 8, 8, {"lights": AmbientLights(ambient_color=((0.2, 0.3, 0.4),)),
                                     "materials": Materials(shininess=10),
                                     "blend_params": BlendParams(background_color=(0.0, 0.5, 0.0))})
    assert cfg.light_kind == 1 and cfg.light_ambient == pytest.approx((0.2, 0.3, 0.4))
    assert cfg.shininess == 10.0 and cfg.background == (0.0, 0.5, 0.0)
    cfg = r._config(cams, rs, 8, 8, {"lights": PointLights(location=[[1.0, 2.0, 3.0]])})
    assert cfg.light_location == (1.0, 2.0, 3.0)
    s = MeshRenderer(MeshRasterizer(cams, rs), SoftSilhouetteShader(BlendParams(sigma=2e-4)))
    assert s._config(cams, rs, 8, 8, {"blend_params": BlendParams(sigma=3e-4)}).sigma_sil == pytest.approx(3e-4)
    assert r._config(FoVPerspectiveCameras(), rs, 8, 8, {}).z_clip == 0.5


def test_differentiable_lights_are_refused():
    with pytest.raises(NotImplementedError):
        PointLights(location=torch.zeros(1, 3, requires_grad=True))
    with pytest.raises(NotImplementedError):
        Materials(diffuse_color=torch.ones(1, 3, requires_grad=True))


def test_uv_texture_requiring_grad_takes_the_modular_path():
    from torch_renderer_amd.torch_renderer import textures_need_modular

    v, f, d = mesh_arrays("cow")
    img = torch.rand(8, 8, 3)
    tex = TexturesUV(maps=[img], faces_uvs=[torch.from_numpy(d["faces_uvs"]).long()],
                     verts_uvs=[torch.from_numpy(d["verts_uvs"]).float()])
    assert not textures_need_modular(Meshes([v], [f], tex))
    tex2 = TexturesUV(maps=[img.clone().requires_grad_(True)], faces_uvs=tex.faces_uvs_list(),
                      verts_uvs=tex.verts_uvs_list())
    assert textures_need_modular(Meshes([v], [f], tex2))
    assert not textures_need_modular(Meshes([v], [f], TexturesVertex([torch.ones_like(v).requires_grad_(True)])))


# ----------------------------------------------------------------- oracle: near-plane clipping
def _view_pos(fv):
    """View-space position of NDC (intr ax = ay = 1, bx = by = 0) vertices: (x z, y z, z)."""
    return torch.stack([fv[..., 0] * fv[..., 2], fv[..., 1] * fv[..., 2], fv[..., 2]], -1)


@pytest.mark.parametrize("zs,n_out", [((1.0, 1.0, 1.0), 1), ((0.2, 1.0, 1.5), 2), ((0.2, 0.3, 1.5), 1),
                                      ((0.1, 0.2, 0.3), 0)])
def test_clip_faces_cases(zs, n_out):
    xy = torch.tensor([[0.1, -0.2], [0.6, 0.1], [-0.3, 0.5]])
    fv = torch.cat([xy, torch.tensor(zs)[:, None]], 1)[None].double()
    for rot in range(3):  # every corner can be the odd one out
        f = torch.roll(fv, rot, dims=1)
        cf = O.clip_faces_ref(f, torch.tensor([0]), torch.tensor([1]), 0.5, persp=True)
        assert cf["face_verts"].shape[0] == n_out and int(cf["count"][0]) == n_out
        if n_out == 0:
            continue
        sub = cf["face_verts"]
        assert (sub[..., 2] >= 0.5 - 1e-12).all()
        # conversion rows reproduce the sub-triangle's view-space vertices from the original's
        P = _view_pos(f[0])
        rec = torch.einsum("tsc,cd->tsd", cf["conversion"], P)
        assert torch.allclose(rec, _view_pos(sub), atol=1e-12)
        # orientation kept
        def area(t):
            return (t[:, 1, 0] - t[:, 0, 0]) * (t[:, 2, 1] - t[:, 0, 1]) - (t[:, 1, 1] - t[:, 0, 1]) * (t[:, 2, 0] - t[:, 0, 0])
        assert (torch.sign(area(_view_pos(sub))) == torch.sign(area(_view_pos(f)))).all()
        if n_out == 2:
            assert cf["neighbor"].tolist() == [1, 0]
        assert (cf["orig"] == 0).all()


def test_clip_faces_is_differentiable():
    g = torch.Generator().manual_seed(0)
    fv = torch.rand(6, 3, 3, generator=g, dtype=torch.float64)
    fv[..., 2] = fv[..., 2] * 1.5 + 0.05
    fv.requires_grad_(True)

    def f(x):
        cf = O.clip_faces_ref(x, torch.tensor([0]), torch.tensor([6]), 0.5, persp=True)
        return cf["face_verts"], cf["conversion"]
    assert torch.autograd.gradcheck(f, (fv,))


def test_neighbor_rule_in_c_oracle():
    """Two halves of a clipped quad: a pixel within blur of both keeps only the nearer-edged one."""
    fv = torch.tensor([[[-0.5, -0.5, 1.0], [0.5, -0.5, 1.0], [0.5, 0.5, 1.0]],
                       [[-0.5, -0.5, 1.0], [0.5, 0.5, 1.0], [-0.5, 0.5, 1.0]]])
    first, count = torch.tensor([0]), torch.tensor([2])
    H = W = 16
    a = O.raster_fwd(fv, first, count, H, W, K=2, blur=1e-3, persp=True)
    b = O.raster_fwd(fv, first, count, H, W, K=2, blur=1e-3, persp=True, neighbor=torch.tensor([1, 0]))
    both = (a[0] >= 0).all(-1)
    assert both.any()                       # without the rule some pixels keep both halves
    assert ((b[0] >= 0).sum(-1) <= 1).all()  # with it, never
    win = O.raster_fwd(fv, first, count, H, W, K=2, blur=1e-3, persp=True, window=(4, 9, 2, 7))
    assert torch.equal(win[0][:, 4:9, 2:7], a[0][:, 4:9, 2:7]) and (win[0][:, :4] == -1).all()


def test_hard_rgb_blend_oracle_known_answer():
    """upstream hard_rgb_blend (HardPhongShader): nearest fragment's colour or background, alpha =
    coverage; the oracle restatement on a 1x1x2 image with K = 2."""
    colors = torch.tensor([[[[[0.1, 0.2, 0.3], [0.9, 0.9, 0.9]], [[0.4, 0.5, 0.6], [0.7, 0.7, 0.7]]]]])
    p2f = torch.tensor([[[[3, 5], [-1, -1]]]])
    out = O.hard_rgb_blend(colors, p2f, (1.0, 0.5, 0.25))
    assert torch.equal(out, torch.tensor([[[[0.1, 0.2, 0.3, 1.0], [1.0, 0.5, 0.25, 0.0]]]]))


def test_pose_loss_needs_device_tensors():
    from torch_renderer_amd.losses import pose_loss

    t = torch.zeros(1, 4, 4)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        pose_loss(t, t, torch.zeros(1, 4, 4, 3), t > 0, t, torch.zeros(1, 4, 4, 3))


def test_hard_phong_shader_is_exported_and_routed_to_fragments():
    import torch_renderer_amd as T
    from torch_renderer_amd.mesh_renderer import HardPhongShader, _shade_config

    assert T.HardPhongShader is HardPhongShader
    cfg = _shade_config(HardPhongShader(), None, 8, 8, {})
    assert cfg.hard and cfg.want_rgb and not cfg.want_sil


def test_u8_texture_copy_only_when_exact():
    """TexturesUV.u8_map: an 8-bit copy is offered only when every texel is exactly float32(k)/255
    (then the kernels' table lookup returns the identical floats); otherwise None (f32 texels)."""
    g = torch.Generator().manual_seed(0)
    u8 = torch.randint(0, 256, (16, 12, 3), generator=g, dtype=torch.uint8)
    exact = u8.float() / 255.0
    t = TexturesUV(maps=[exact], faces_uvs=[torch.zeros(1, 3, dtype=torch.long)], verts_uvs=[torch.zeros(1, 2)])
    q, lut = t.u8_map(0)
    assert q.dtype == torch.uint8 and q.shape == (16, 12, 4)
    assert torch.equal(lut[q.long()][..., :3], exact) and not q[..., 3].any()
    off = exact.clone()
    off[3, 4, 1] = 0.5  # not k/255 for any k
    t2 = TexturesUV(maps=[off], faces_uvs=[torch.zeros(1, 3, dtype=torch.long)], verts_uvs=[torch.zeros(1, 2)])
    assert t2.u8_map(0) is None
