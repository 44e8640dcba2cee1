"""CPU checks of the round-3 drop-in fidelity fixes (no GPU): camera indexing, light / material /
background updates taking effect, the per-call raster settings reaching MeshRasterizer.transform,
and the oracle's float64 shadow and conditioning probe."""
import torch

from oracle import oracle as O
from tests.helpers import canonical_views, mesh_arrays, oracle_runs
from torch_renderer_amd.cameras import PerspectiveCameras
from torch_renderer_amd.mesh_renderer import (AmbientLights, BlendParams, Materials, MeshRasterizer, MeshRenderer,
                                              PointLights, RasterizationSettings, SoftPhongShader, _bg_triple,
                                              _shade_config)


def test_negative_camera_index_is_the_last_camera():
    R = torch.eye(3).repeat(4, 1, 1)
    T = torch.arange(12, dtype=torch.float32).reshape(4, 3)
    cams = PerspectiveCameras(focal_length=torch.tensor([[1.0, 1.0]]).repeat(4, 1), R=R, T=T)
    last = cams[-1]
    assert last.T.shape == (1, 3) and torch.equal(last.T, T[3:4])
    assert torch.equal(cams[-4].T, T[0:1])
    assert last.fx.shape == (1,)


def test_update_light_position_takes_effect():
    """renderer.py:82-83 assigns lights.location; the next render must use it."""
    from torch_renderer_amd.renderer import Renderer

    r = Renderer(image_size=(32, 48))
    r.build_color_renderer()
    cfg0 = _shade_config(r.color_renderer.shader, r.cameras, 32, 48, {})
    assert cfg0.light_location == (0.0, 0.0, -3.0)
    r.update_light_position([1.0, 2.0, -4.0])
    cfg1 = _shade_config(r.color_renderer.shader, r.cameras, 32, 48, {})
    assert cfg1.light_location == (1.0, 2.0, -4.0)
    assert torch.equal(torch.as_tensor(r.lights.location), torch.tensor([[1.0, 2.0, -4.0]]))


def test_light_and_material_colour_assignment_takes_effect():
    sh = SoftPhongShader(lights=PointLights(), materials=Materials())
    sh.lights.ambient_color = ((0.1, 0.2, 0.3),)
    sh.lights.specular_color = torch.tensor([[0.0, 0.5, 1.0]])
    sh.materials.diffuse_color = ((0.7, 0.7, 0.7),)
    sh.materials.shininess = 12
    cams = PerspectiveCameras()
    cfg = _shade_config(sh, cams, 8, 8, {})
    f32 = lambda *x: tuple(float(torch.tensor(v, dtype=torch.float32)) for v in x)  # noqa: E731
    assert cfg.light_ambient == f32(0.1, 0.2, 0.3) and cfg.light_specular == (0.0, 0.5, 1.0)
    assert cfg.mat_diffuse == f32(0.7, 0.7, 0.7) and cfg.shininess == 12.0
    amb = AmbientLights()
    amb.ambient_color = ((0.25, 0.5, 0.75),)
    assert _shade_config(sh, cams, 8, 8, {"lights": amb}).light_ambient == (0.25, 0.5, 0.75)
    try:
        sh.lights.location = torch.zeros(1, 3, requires_grad=True)
    except NotImplementedError:
        pass
    else:
        raise AssertionError("a light location that requires grad must be refused, not dropped")


def test_background_colour_mutation_is_read_each_call():
    bp = BlendParams(background_color=[1.0, 1.0, 1.0])
    assert _bg_triple(bp) == (1.0, 1.0, 1.0)
    bp.background_color[1] = 0.0  # mutated in place: same object id
    assert _bg_triple(bp) == (1.0, 0.0, 1.0)
    t = torch.tensor([0.5, 0.5, 0.5])
    bp.background_color = t
    assert _bg_triple(bp) == (0.5, 0.5, 0.5)
    t[0] = 0.25  # in-place on the tensor bumps its version
    assert _bg_triple(bp) == (0.25, 0.5, 0.5)


def test_transform_uses_the_per_call_image_size(monkeypatch):
    """MeshRasterizer.transform with a per-call raster_settings builds the intrinsics for THAT size
    (as the shared-mesh world path does)."""
    from torch_renderer_amd import mesh_renderer as M
    from torch_renderer_amd.structures import Meshes

    seen = {}

    def fake_apply(v, R, T, f, intr, *ranges):
        seen["intr"] = intr.clone()
        return torch.zeros(f.shape[0], 3, 3)

    monkeypatch.setattr(M.ProjectFacesMeshes, "apply", fake_apply)  # two distinct meshes: one union launch
    cams = PerspectiveCameras(focal_length=((100.0, 100.0),), principal_point=((40.0, 30.0),), in_ndc=False,
                              image_size=torch.tensor([[60, 80]]))
    v = torch.rand(4, 3)
    f = torch.tensor([[0, 1, 2], [1, 2, 3]])
    rast = MeshRasterizer(cams, RasterizationSettings(image_size=(60, 80)))
    rast.transform(Meshes([v, v], [f, f]), raster_settings=RasterizationSettings(image_size=(120, 160)))
    big = seen["intr"]
    rast.transform(Meshes([v, v], [f, f]))
    small = seen["intr"]
    # in_ndc=False cameras carry their own image_size: the affine follows the camera, and both calls
    # must at least agree with the camera's ndc_affine for the size they pass
    assert torch.equal(big, cams.ndc_affine((120, 160)).expand_as(big))
    assert torch.equal(small, cams.ndc_affine((60, 80)).expand_as(small))


def test_f64_shadow_matches_f32_oracle_and_probe_is_local():
    """The float64 shadow takes the f32 run's decisions (identical pix_to_face) and agrees with it to
    f32 accuracy; the conditioning probe only runs inside its context."""
    verts, faces, _ = mesh_arrays("teapot")
    H = W = 24
    R, T, intr, _ = canonical_views(verts, 2, H, W)
    g = torch.Generator().manual_seed(0)
    gC = torch.rand(2, H, W, 3, generator=g) - 0.5

    def run(p):
        vr = verts.clone().requires_grad_(True)
        ref = O.render_ref(vr, faces, R, T, intr, H, W, precision=p)
        (ref["rgba"][..., :3] * gC.to(ref["rgba"].dtype)).sum().backward()
        return ref["rgba"], vr.grad, ref["p2f"]

    ref, r64, sp = oracle_runs(run, seeds=2)
    assert torch.equal(ref[2], r64[2])
    assert (ref[0].double() - r64[0]).abs().max() < 1e-5
    assert sp[0].max() < 1e-5
    assert O._PERTURB is None
    a = run("f32")
    assert torch.equal(a[0], ref[0]) and torch.equal(a[1], ref[1])


def test_meshrenderer_soft_modular_path_rasterizes_once(monkeypatch):
    """DepthColorRender's modular path (UV map with grad) runs ONE rasterizer call for depth,
    silhouette and colour (it used to rasterize three times)."""
    from torch_renderer_amd import torch_renderer as TR
    from torch_renderer_amd.mesh_renderer import Fragments

    calls = {"n": 0}

    def fake_forward(self, meshes_world, **kw):
        calls["n"] += 1
        z = torch.zeros(1, 4, 4, 1)
        return Fragments(z.long() - 1, z - 1, torch.zeros(1, 4, 4, 1, 3) - 1, z - 1)

    def fake_shade(self, fragments, meshes, **kw):
        return torch.zeros(1, 4, 4, 4)

    monkeypatch.setattr(MeshRasterizer, "forward", fake_forward)
    monkeypatch.setattr(SoftPhongShader, "forward", fake_shade)
    monkeypatch.setattr(TR, "textures_need_modular", lambda m: True)
    from torch_renderer_amd.mesh_renderer import SoftSilhouetteShader
    monkeypatch.setattr(SoftSilhouetteShader, "forward", fake_shade)
    from torch_renderer_amd.structures import Meshes

    K = torch.tensor([[10.0, 0.0, 2.0], [0.0, 10.0, 2.0], [0.0, 0.0, 1.0]])
    r = TR.DepthColorRender(K, (4, 4), device="cpu")
    m = Meshes([torch.rand(3, 3)], [torch.tensor([[0, 1, 2]])])
    d, s, c = r.render(m, torch.eye(3)[None], torch.zeros(1, 3))
    assert calls["n"] == 1 and d.shape == (1, 4, 4) and s.shape == (1, 4, 4) and c.shape == (1, 4, 4, 3)
    assert isinstance(r._soft[0][1], MeshRenderer)
