"""Host-side behaviour of the PyTorch3D-style API and the drop-in classes that needs no GPU:
settings, error behaviour of unsupported settings, and the loud failure
on CPU tensors (the MI355X path has no CPU fallback)."""
import pytest
import torch

from tests.helpers import mesh_arrays
from torch_renderer_amd import Meshes, TexturesVertex
from torch_renderer_amd.cameras import FoVPerspectiveCameras, PerspectiveCameras
from torch_renderer_amd.mesh_renderer import (MeshRasterizer, MeshRenderer, RasterizationSettings, SoftPhongShader,
                                              _check_cull_to_frustum, _z_clip_value)
from torch_renderer_amd.torch_renderer import ColorRender, DepthRender


def test_settings_and_zclip_value():
    assert RasterizationSettings(image_size=128).hw() == (128, 128)
    assert RasterizationSettings(image_size=(72, 96)).hw() == (72, 96)
    rs = RasterizationSettings()
    assert _z_clip_value(FoVPerspectiveCameras(znear=1.0), rs) == 0.5        # MeshRasterizer: znear / 2
    assert _z_clip_value(PerspectiveCameras(), rs) is None                    # no znear -> no clipping
    assert _z_clip_value(PerspectiveCameras(), RasterizationSettings(z_clip_value=0.2)) == 0.2


def test_cull_to_frustum_raises():
    _check_cull_to_frustum(False)
    with pytest.raises(NotImplementedError):
        _check_cull_to_frustum(True)


def test_unsupported_settings_raise():
    verts, faces, _ = mesh_arrays("sphere")
    m = Meshes([verts], [faces], TexturesVertex([torch.ones_like(verts)]))
    cams = PerspectiveCameras()
    r = MeshRenderer(MeshRasterizer(cams, RasterizationSettings(image_size=32, faces_per_pixel=4)),
                     SoftPhongShader(cameras=cams))
    with pytest.raises(RuntimeError):    # K-deep soft path: the HIP rasterizer refuses CPU tensors
        r(m)
    d3 = DepthRender(torch.eye(3), (32, 32), faces_per_pixel=3, device="cpu")
    with pytest.raises(RuntimeError):    # no CPU fallback behind the drop-in classes either
        d3.render(m, torch.eye(3)[None], torch.tensor([[0.0, 0.0, 3.0]]))
    with pytest.raises(NotImplementedError):
        ColorRender(torch.eye(3), (32, 32), blur_radius=1e-4, device="cpu")
    with pytest.raises(AssertionError):
        DepthRender([[1.0]], (32, 32), device="cpu")
    with pytest.raises(RuntimeError):
        DepthRender(torch.eye(3), [32, 32], device="cpu")


def test_cpu_tensors_fail_loudly():
    verts, faces, _ = mesh_arrays("sphere")
    m = Meshes([verts], [faces], TexturesVertex([torch.ones_like(verts)])).extend(2)
    K = torch.tensor([[40.0, 0, 16], [0, 40.0, 16], [0, 0, 1]])
    R = torch.eye(3).expand(2, 3, 3).contiguous()
    t = torch.tensor([[0.0, 0.0, 4.0]]).expand(2, 3).contiguous()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ColorRender(K, (32, 32), device="cpu").render(m, R, t)
    cams = PerspectiveCameras()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        MeshRasterizer(cams, RasterizationSettings(image_size=32))(m, R=R, T=t)
    from torch_renderer_amd.renderer import Renderer
    ren = Renderer(image_size=(36, 64))           # CPU-only container: device falls back to cpu
    ren.meshes = m[0]
    ren.build_color_renderer()
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ren.render()


def test_soft_shading_matches_oracle_on_cpu_fragments():
    """soft_shading.py (the modular K > 1 shader) restates the same upstream formulas as the
    oracle: fed the oracle's own K=3 fragments on the CPU, both give identical images."""
    import torch

    from oracle import oracle as O
    from tests.helpers import canonical_views, mesh_arrays
    from torch_renderer_amd import Meshes, TexturesVertex
    from torch_renderer_amd import soft_shading as S
    from torch_renderer_amd.mesh_renderer import BlendParams, Fragments, Materials, PointLights

    H, W, N, Kf = 24, 24, 2, 3
    verts, faces, _ = mesh_arrays("teapot")
    R, T, intr, _ = canonical_views(verts, N, H, W)
    vcol = torch.rand(verts.shape, generator=torch.Generator().manual_seed(2))
    cc = torch.tensor([[0.1, 0.2, -0.3]])
    ref = O.render_ref(verts, faces, R, T, intr, H, W, texture=("vertex", vcol), cam_center=cc, K=Kf, blur=1e-4,
                       bg=(0.0, 0.5, 1.0))
    frags = Fragments(ref["p2f"], ref["zbuf"], ref["bary"], ref["dists"])
    meshes = Meshes([verts], [faces], TexturesVertex([vcol])).extend(N)
    texels = S.sample_textures(meshes, frags)
    colors = S.phong_shading(meshes, frags, texels, PointLights(location=((0.0, 0.0, -3.0),)), Materials(), cc)
    bp = BlendParams(background_color=(0.0, 0.5, 1.0))
    rgba = S.softmax_rgb_blend(colors, frags, bp)
    sil = S.sigmoid_alpha_blend(frags, bp)
    assert (ref["p2f"][..., 1] >= 0).any()
    assert torch.allclose(rgba, ref["rgba"], atol=1e-6, rtol=0)
    assert torch.allclose(sil[..., 3], ref["sil"], atol=1e-6, rtol=0)


def test_soft_shading_uv_texture_matches_oracle_on_cpu_fragments():
    """TexturesUV branch of soft_shading.sample_textures (per-view map expand, y flip, border
    bilinear) against the oracle's texture sampling on the oracle's K=2 fragments."""
    import numpy as np
    import torch

    from oracle import oracle as O
    from tests.helpers import canonical_views, mesh_arrays
    from torch_renderer_amd import Meshes, TexturesUV
    from torch_renderer_amd import soft_shading as S
    from torch_renderer_amd.mesh_renderer import Fragments

    H, W, N, Kf = 20, 28, 2, 2
    verts, faces, d = mesh_arrays("cow")
    R, T, intr, _ = canonical_views(verts, N, H, W)
    img = torch.from_numpy(d["texture_u8"].astype(np.float32) / 255.0)
    vuv = torch.from_numpy(d["verts_uvs"]).float()
    fuv = torch.from_numpy(d["faces_uvs"]).long()
    ref = O.render_ref(verts, faces, R, T, intr, H, W, texture=("uv", vuv, fuv, img), K=Kf)
    frags = Fragments(ref["p2f"], ref["zbuf"], ref["bary"], ref["dists"])
    local = ref["p2f"].clone()
    local[local >= 0] %= faces.shape[0]
    want = O.sample_textures_uv(local, ref["bary"], vuv, fuv, img)
    meshes = Meshes([verts], [faces], TexturesUV(maps=[img], faces_uvs=[fuv], verts_uvs=[vuv])).extend(N)
    got = S.sample_textures(meshes, frags)
    assert got.shape == (N, H, W, Kf, 3)
    assert (ref["p2f"] >= 0).any()
    assert torch.allclose(got, want, atol=1e-6, rtol=0)
