"""mr_rasterize_meshes_world (MeshRasterizer.forward for one mesh shared by every view) against the
two-step boundary it fuses: mr_project_faces -> mr_rasterize_meshes (upstream
MeshRasterizer.transform + _RasterizeFaceVerts). The projection runs inside the binning's first
launch there, so the fragments must be BITWISE the two-step ones (same projection arithmetic, same
raster), on the per-view binning path, on its count -> scan fallback (a 1040x1040 tile grid), with
K > 1 and with near-plane clipping. Gradients to vertices / R / T go through the same backward
kernels (float atomics: summation order differs run to run), compared within 1e-4 x scale."""
import math

import pytest
import torch

from tests.helpers import canonical_views, mesh_arrays, report
from torch_renderer_amd import kernels as Kn
from torch_renderer_amd.transforms import look_at_view_transform

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _two_step(verts, faces, R, T, intr, N, H, W, K, blur, persp, clip, z_clip):
    Fn = faces.shape[0]
    fv = Kn.ProjectFaces.apply(verts, R, T, faces, intr.contiguous())
    first = (torch.arange(N, device=DEV) * Fn).contiguous()
    count = torch.full((N,), Fn, device=DEV, dtype=torch.int64)
    return Kn.RasterizeFaceVerts.apply(fv, first, count, H, W, K, blur, persp, clip, False, None, z_clip)


CASES = [  # name, H, W, N, K, blur, z_clip, dist
    ("cow", 96, 128, 3, 1, 0.0, None, None),
    ("cow", 512, 512, 4, 1, 0.0, None, None),
    ("teapot", 80, 80, 2, 3, 2e-4, None, None),
    ("cow", 96, 96, 3, 1, 0.0, 0.5, 0.52),      # near-plane clipping: the views cut the cow
    ("cow", 96, 96, 3, 3, 2e-4, 0.5, 0.52),
    ("sphere", 1040, 1040, 1, 1, 0.0, None, None),  # > 16384 tiles: count -> scan fallback
]


@pytest.mark.parametrize("name,H,W,N,K,blur,z_clip,dist", CASES)
def test_world_fragments_bitwise_two_step(name, H, W, N, K, blur, z_clip, dist):
    verts, faces, _ = mesh_arrays(name)
    if dist is None:
        R, T, intr, _ = canonical_views(verts, N, H, W)
    else:  # FoV camera placed inside the near plane's reach (test_gpu_clip.py's setup)
        R, T = look_at_view_transform(dist, torch.linspace(-10.0, 35.0, N), torch.linspace(0.0, 300.0, N))
        f = 1.0 / math.tan(math.radians(30.0))
        intr = torch.tensor([[f, 0.0, f, 0.0]]).expand(N, 4)
    v = verts.to(DEV)
    fc = faces.to(DEV)
    Rd, Td, Id = R.float().to(DEV), T.float().to(DEV), intr.float().to(DEV)
    persp = True
    clip = blur > 0.0
    args = (H, W, K, blur, persp, clip, False, None, z_clip)
    vw, Rw, Tw = v.clone().requires_grad_(True), Rd.clone().requires_grad_(True), Td.clone().requires_grad_(True)
    got = Kn.RasterizeMeshesWorld.apply(vw, Rw, Tw, fc, Id, N, *args)
    vr, Rr, Tr = v.clone().requires_grad_(True), Rd.clone().requires_grad_(True), Td.clone().requires_grad_(True)
    ref = _two_step(vr, fc, Rr, Tr, Id, N, H, W, K, blur, persp, clip, z_clip)
    for a, b, nm in zip(got, ref, ("pix_to_face", "zbuf", "bary", "dists")):
        assert a.shape == b.shape, nm
        if a.dtype == torch.int64:
            assert torch.equal(a, b), f"{nm}: {(a != b).sum().item()} differ"
        else:
            assert torch.equal(a.view(torch.int32), b.view(torch.int32)), f"{nm}: max {(a - b).abs().max().item()}"
    assert (got[0] >= 0).any(), "the views must see the mesh"
    g = torch.Generator(device=DEV).manual_seed(1)
    gz = torch.rand(got[1].shape, generator=g, device=DEV) - 0.5
    gb = torch.rand(got[2].shape, generator=g, device=DEV) - 0.5
    gd = torch.rand(got[3].shape, generator=g, device=DEV) - 0.5
    ((got[1] * gz).sum() + (got[2] * gb).sum() + (got[3] * gd).sum()).backward()
    ((ref[1] * gz).sum() + (ref[2] * gb).sum() + (ref[3] * gd).sum()).backward()
    # both paths run the same backward kernels, whose float atomics sum in a different order each
    # run: the two-step path re-run 3 times gives each entry's run-to-run spread (its conditioning)
    spread = [torch.zeros_like(x) for x in (vr.grad, Rr.grad, Tr.grad)]
    for _ in range(3):
        leaves = [x.detach().clone().requires_grad_(True) for x in (v, Rd, Td)]
        r2 = _two_step(leaves[0], fc, leaves[1], leaves[2], Id, N, H, W, K, blur, persp, clip, z_clip)
        ((r2[1] * gz).sum() + (r2[2] * gb).sum() + (r2[3] * gd).sum()).backward()
        for sp, x, y in zip(spread, leaves, (vr.grad, Rr.grad, Tr.grad)):
            torch.maximum(sp, (x.grad - y).abs(), out=sp)
    for (a, b, nm), sp in zip(((vw.grad, vr.grad, "verts"), (Rw.grad, Rr.grad, "R"), (Tw.grad, Tr.grad, "T")), spread):
        report(f"world {name} {H}x{W} K={K} clip={z_clip} grad {nm}", a.cpu(), b.cpu(), sens=sp.cpu())


def test_meshrasterizer_uses_world_path_and_matches_transform():
    """MeshRasterizer.forward on an extended mesh takes the one-call path; its fragments equal
    rasterizing MeshRasterizer.transform's face_verts."""
    from torch_renderer_amd import Meshes
    from torch_renderer_amd.cameras import PerspectiveCameras
    from torch_renderer_amd.mesh_renderer import MeshRasterizer, RasterizationSettings

    verts, faces, _ = mesh_arrays("cow")
    H = W = 128
    N = 5
    R, T, intr, (R_cv, t_cv, Kcv) = canonical_views(verts, N, H, W)
    cams = PerspectiveCameras(focal_length=((float(Kcv[0, 0]), float(Kcv[1, 1])),),
                              principal_point=((float(Kcv[0, 2]), float(Kcv[1, 2])),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]), device=DEV)
    rs = RasterizationSettings(image_size=(H, W))
    m = Meshes([verts.to(DEV)], [faces.to(DEV)]).extend(N)
    ras = MeshRasterizer(cams, rs)
    frag = ras(meshes_world=m, R=R.to(DEV), T=T.to(DEV))
    fv = ras.transform(m, R=R.to(DEV), T=T.to(DEV))
    Fn = faces.shape[0]
    first = (torch.arange(N, device=DEV) * Fn).contiguous()
    count = torch.full((N,), Fn, device=DEV, dtype=torch.int64)
    ref = Kn.RasterizeFaceVerts.apply(fv, first, count, H, W, 1, 0.0, True, False, False, None, None)
    assert torch.equal(frag.pix_to_face, ref[0])
    assert torch.equal(frag.zbuf.view(torch.int32), ref[1].view(torch.int32))
    assert torch.equal(frag.bary_coords.view(torch.int32), ref[2].view(torch.int32))
    assert torch.equal(frag.dists.view(torch.int32), ref[3].view(torch.int32))
