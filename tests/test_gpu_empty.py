"""Empty scenes (no face lands in any view: the mesh sits behind every camera) through the fused render
path and the modular rasterizer, fwd + bwd, with the caching allocator's recycled memory holding
garbage. The raster then emits no slot, and the kernels whose prefetches read the winners of slot 0
must not touch them (they were never written). Expected: background everywhere, zero gradients —
PyTorch3D's result for a mesh that projects nowhere."""
import pytest
import torch

from tests.helpers import canonical_views, mesh_arrays
from torch_renderer_amd import Meshes, TexturesVertex
from torch_renderer_amd.cameras import PerspectiveCameras
from torch_renderer_amd.mesh_renderer import MeshRasterizer, RasterizationSettings
from torch_renderer_amd.torch_renderer import DepthColorRender

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _dirty_allocator():
    """Recycled device memory full of large positive ints (a face id far past any record)."""
    junk = torch.full((32 << 20,), 0x3FFFFFF0, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    del junk


def test_fused_render_of_an_empty_scene():
    verts, faces, _ = mesh_arrays("cow")
    H = W = 64
    N = 3
    R_cv, t_cv, K = canonical_views(verts, N, H, W)[3]
    t_cv = t_cv.clone()
    t_cv[:, 2] -= 50.0  # the mesh behind every camera
    vg = verts.to(DEV).requires_grad_(True)
    m = Meshes([vg], [faces.to(DEV)], TexturesVertex([torch.ones_like(vg).detach()])).extend(N)
    Rg = R_cv.float().to(DEV).requires_grad_(True)
    tg = t_cv.float().to(DEV).requires_grad_(True)
    _dirty_allocator()
    d, s, c = DepthColorRender(K.to(DEV), (H, W), device=DEV).render(m, Rg, tg)
    torch.autograd.backward([d, s, c], [torch.ones_like(d), torch.ones_like(s), torch.ones_like(c)])
    torch.cuda.synchronize()
    assert torch.equal(d.detach().cpu(), torch.zeros(N, H, W))
    assert torch.equal(s.detach().cpu(), torch.zeros(N, H, W))
    assert torch.equal(c.detach().cpu(), torch.ones(N, H, W, 3))
    for g in (vg.grad, Rg.grad, tg.grad):
        assert g is not None and torch.equal(g.cpu(), torch.zeros_like(g.cpu()))


@pytest.mark.parametrize("K", [1, 8])
def test_mesh_rasterizer_of_an_empty_scene(K):
    verts, faces, _ = mesh_arrays("cow")
    H, W = 48, 56
    R, T, _, (R_cv, t_cv, Kc) = canonical_views(verts, 2, H, W)
    T = T.clone()
    T[:, 2] -= 50.0
    cams = PerspectiveCameras(focal_length=((Kc[0, 0].item(), Kc[1, 1].item()),),
                              principal_point=((Kc[0, 2].item(), Kc[1, 2].item()),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]), device=DEV)
    vg = verts.to(DEV).requires_grad_(True)
    meshes = Meshes([vg], [faces.to(DEV)]).extend(2)
    rs = RasterizationSettings(image_size=(H, W), faces_per_pixel=K, blur_radius=1e-4 if K > 1 else 0.0)
    _dirty_allocator()
    frag = MeshRasterizer(cams, rs)(meshes, R=R.to(DEV), T=T.to(DEV))
    (frag.zbuf.sum() + frag.dists.sum() + frag.bary_coords.sum()).backward()
    torch.cuda.synchronize()
    assert torch.equal(frag.pix_to_face.cpu(), torch.full((2, H, W, K), -1, dtype=torch.int64))
    for x in (frag.zbuf, frag.dists, frag.bary_coords):
        assert bool((x.detach() == -1).all())
    assert torch.equal(vg.grad.cpu(), torch.zeros_like(verts))


def test_fused_soft_silhouette_of_an_empty_scene():
    """MeshRenderer(MeshRasterizer(K = 8), SoftSilhouetteShader): no occupied tile, so the fused raster emits
    no slot and k_sil_bwd's grid exits on the slot counter; every pixel keeps the prefilled (1, 1, 1, 0)."""
    from torch_renderer_amd.mesh_renderer import MeshRenderer, SoftSilhouetteShader
    verts, faces, _ = mesh_arrays("cow")
    H, W = 48, 56
    R, T, _, _ = canonical_views(verts, 2, H, W)
    T = T.clone()
    T[:, 2] -= 50.0
    cams = PerspectiveCameras(device=DEV)
    vg = verts.to(DEV).requires_grad_(True)
    meshes = Meshes([vg], [faces.to(DEV)]).extend(2)
    rs = RasterizationSettings(image_size=(H, W), faces_per_pixel=8, blur_radius=1e-4)
    renderer = MeshRenderer(MeshRasterizer(cams, rs), SoftSilhouetteShader())
    _dirty_allocator()
    img = renderer(meshes, R=R.to(DEV), T=T.to(DEV))
    img.sum().backward()
    torch.cuda.synchronize()
    bg = torch.zeros(2, H, W, 4)
    bg[..., :3] = 1.0
    assert torch.equal(img.detach().cpu(), bg)
    assert torch.equal(vg.grad.cpu(), torch.zeros_like(verts))
