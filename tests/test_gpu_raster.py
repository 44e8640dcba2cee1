"""GPU parity of the rasterizer boundary (mr_project_faces, mr_rasterize_meshes[_backward])
against the C oracle (restated RasterizeMeshesNaiveCpu / BackwardCpu) on identical inputs.
Bar: pix_to_face bit-exact; zbuf/bary/dists bit-exact (same operand order, no FMA);
grad_face_verts within 1e-4 abs (float atomics change the summation order)."""
import pytest
import torch

from oracle import oracle as O
from tests.helpers import canonical_views, mesh_arrays, report
from torch_renderer_amd import kernels as Kn

pytestmark = pytest.mark.gpu

CASES = [
    ("sphere", 64, 64, 2, True),
    ("cow", 96, 128, 3, True),
    ("teapot", 80, 80, 2, False),
    ("dolphin", 64, 96, 1, True),
    # W % 8 == 4: the last tile column is half outside the image, 256-pixel background chunks span rows
    ("cow", 60, 100, 2, True),
]


def _inputs(name, H, W, N):
    verts, faces, _ = mesh_arrays(name)
    R, T, intr, _ = canonical_views(verts, N, H, W)
    views = O.views_tensor(R, T, intr)
    return verts, faces, views


@pytest.mark.parametrize("name,H,W,N,persp", CASES)
def test_projection_bitexact(name, H, W, N, persp):
    verts, faces, views = _inputs(name, H, W, N)
    ref = O.project_faces_c(verts, faces, views)
    dev = torch.device("cuda:0")
    R, T, intr = views[:, :9].reshape(N, 3, 3), views[:, 9:12], views[:, 12:]
    got = Kn.ProjectFaces.apply(verts.to(dev), R.to(dev), T.to(dev), faces.to(dev), intr.to(dev)).cpu()
    assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), (got - ref).abs().max()
    # the torch restatement used by the autograd oracle is bitwise identical too
    tor = O.project_faces_torch(verts, faces, R, T, intr)
    assert torch.equal(tor.view(torch.int32), ref.view(torch.int32))


@pytest.mark.parametrize("name,H,W,N,persp", CASES)
def test_raster_forward_matches_oracle(name, H, W, N, persp):
    verts, faces, views = _inputs(name, H, W, N)
    fv = O.project_faces_c(verts, faces, views)
    F = faces.shape[0]
    first = torch.arange(N) * F
    count = torch.full((N,), F)
    ref = O.raster_fwd(fv, first, count, H, W, 1, 0.0, persp)
    dev = torch.device("cuda:0")
    got = Kn.rasterize_meshes_fwd(fv.to(dev), first.to(dev), count.to(dev), H, W, 1, 0.0, persp)
    got = [t.cpu() for t in got]
    assert torch.equal(got[0], ref[0]), f"pix_to_face mismatch at {(got[0] != ref[0]).sum()} px"
    assert (ref[0] >= 0).sum() > 0.02 * N * H * W, "degenerate test: almost nothing covered"
    for a, b, nm in zip(got[1:], ref[1:], ("zbuf", "bary", "dists")):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), f"{nm}: max diff {(a - b).abs().max()}"


@pytest.mark.parametrize("cap", [1, 7])
def test_bin_overflow_is_exact(cap):
    """max_faces_per_bin smaller than the real per-tile load: the overflow path rescans the view."""
    verts, faces, views = _inputs("cow", 64, 64, 2)
    fv = O.project_faces_c(verts, faces, views)
    F = faces.shape[0]
    first, count = torch.arange(2) * F, torch.full((2,), F)
    ref = O.raster_fwd(fv, first, count, 64, 64)
    dev = torch.device("cuda:0")
    got = Kn.rasterize_meshes_fwd(fv.to(dev), first.to(dev), count.to(dev), 64, 64, max_faces_per_bin=cap)
    assert torch.equal(got[0].cpu(), ref[0])


def test_raster_backward_matches_oracle():
    name, H, W, N = "cow", 64, 80, 2
    verts, faces, views = _inputs(name, H, W, N)
    fv = O.project_faces_c(verts, faces, views)
    F = faces.shape[0]
    first, count = torch.arange(N) * F, torch.full((N,), F)
    p2f, zbuf, bary, dists = O.raster_fwd(fv, first, count, H, W)
    g = torch.Generator().manual_seed(1)
    gz = torch.rand(zbuf.shape, generator=g) * 2 - 1
    gb = torch.rand(bary.shape, generator=g) * 2 - 1
    gd = torch.rand(dists.shape, generator=g) * 2e-5 - 1e-5
    ref = O.raster_bwd(fv, p2f, gz, gb, gd)
    dev = torch.device("cuda:0")
    got = Kn.rasterize_meshes_bwd(fv.to(dev), p2f.to(dev), gz.to(dev), gb.to(dev), gd.to(dev), H, W).cpu()
    report("raster bwd K=1 grad face_verts", got, ref)


def test_empty_views_and_background():
    """No face in view (camera looking away): everything is background (-1)."""
    verts, faces, views = _inputs("teapot", 32, 32, 1)
    views = views.clone()
    views[0, 11] = -50.0  # push the mesh behind the camera
    fv = O.project_faces_c(verts, faces, views)
    F = faces.shape[0]
    dev = torch.device("cuda:0")
    got = Kn.rasterize_meshes_fwd(fv.to(dev), torch.zeros(1, dtype=torch.int64, device=dev),
                                  torch.full((1,), F, device=dev), 32, 32)
    ref = O.raster_fwd(fv, torch.zeros(1, dtype=torch.int64), torch.full((1,), F), 32, 32)
    assert torch.equal(got[0].cpu(), ref[0])
    assert (ref[0] == -1).all() and (got[1].cpu() == -1).all()


@pytest.mark.parametrize("name,H,W,N,K,blur,clip,cap", [
    ("cow", 96, 128, 2, 3, 0.0, False, None),
    ("teapot", 64, 64, 2, 8, 0.0, False, None),
    # soft rasterization as deform_mesh_with_color.py:153-159 configures it (blur > 0 => clip)
    ("sphere", 64, 64, 1, 6, 2e-3, True, None),
    ("cow", 64, 64, 2, 4, 0.0, False, 5),  # overflowing tile lists: whole-view scan
    # every register-list width of k_raster_kr4 (KP = 16 / 32 / 50 / 64, K below KP too) and the
    # LDS-list kernel beyond 64, with a blur wide enough to fill deep lists
    ("cow", 48, 48, 1, 13, 2e-3, True, None),
    ("cow", 48, 48, 1, 20, 2e-3, True, None),
    ("cow", 48, 48, 1, 50, 2e-3, True, None),
    ("cow", 48, 48, 1, 64, 2e-3, True, None),
    ("cow", 48, 48, 1, 100, 2e-3, True, None),
])
def test_raster_k_nearest_matches_oracle(name, H, W, N, K, blur, clip, cap):
    """faces_per_pixel > 1: the K nearest faces per pixel in ascending
    (z, face) order, with their zbuf / bary / dists, bit-exact against the C oracle."""
    verts, faces, views = _inputs(name, H, W, N)
    fv = O.project_faces_c(verts, faces, views)
    F = faces.shape[0]
    first, count = torch.arange(N) * F, torch.full((N,), F)
    ref = O.raster_fwd(fv, first, count, H, W, K, blur, True, clip)
    dev = torch.device("cuda:0")
    got = Kn.rasterize_meshes_fwd(fv.to(dev), first.to(dev), count.to(dev), H, W, K, blur, True, clip,
                                  max_faces_per_bin=cap)
    got = [t.cpu() for t in got]
    assert got[0].shape == (N, H, W, K)
    assert (ref[0][..., 1] >= 0).sum() > 0, "degenerate test: no pixel has a second face"
    assert torch.equal(got[0], ref[0]), f"pix_to_face mismatch at {(got[0] != ref[0]).sum()} entries"
    for a, b, nm in zip(got[1:], ref[1:], ("zbuf", "bary", "dists")):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), f"{nm}: max diff {(a - b).abs().max()}"


def test_raster_k_backward_matches_oracle():
    name, H, W, N, K = "cow", 64, 80, 2, 3
    verts, faces, views = _inputs(name, H, W, N)
    fv = O.project_faces_c(verts, faces, views)
    F = faces.shape[0]
    first, count = torch.arange(N) * F, torch.full((N,), F)
    p2f, zbuf, bary, dists = O.raster_fwd(fv, first, count, H, W, K)
    g = torch.Generator().manual_seed(2)
    gz = torch.rand(zbuf.shape, generator=g) * 2 - 1
    gb = torch.rand(bary.shape, generator=g) * 2 - 1
    gd = torch.rand(dists.shape, generator=g) * 2e-5 - 1e-5
    ref = O.raster_bwd(fv, p2f, gz, gb, gd)
    dev = torch.device("cuda:0")
    got = Kn.rasterize_meshes_bwd(fv.to(dev), p2f.to(dev), gz.to(dev), gb.to(dev), gd.to(dev), H, W, K).cpu()
    report(f"raster bwd K={K} grad face_verts", got, ref)
