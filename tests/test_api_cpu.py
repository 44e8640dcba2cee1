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
