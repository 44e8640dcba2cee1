"""CPU tests that pin the oracle (there are no reference-produced vectors: SURVEY.md §4/§8c).

* analytic known answers: fronto-parallel depth, perspective-correct depth on a tilted
  plane, sphere silhouette area, background sentinels, K ordering, signed distances;
* the C oracle (float32, PyTorch3D operand order) against an independent float64 NumPy
  restatement (oracle/spec_np.py);
* the C oracle backward against float64 autograd of the same per-pixel math;
* the committed golden fixtures (tests/golden/*.npz) reproduce.
"""
import math
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle import spec_np
from tests.helpers import canonical_views, mesh_arrays

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _single(fv):
    fv = torch.as_tensor(np.asarray(fv, np.float32)).reshape(-1, 3, 3)
    return fv, torch.zeros(1, dtype=torch.int64), torch.tensor([fv.shape[0]])


def test_fronto_parallel_depth_and_coverage():
    Z = 2.5
    fv, first, count = _single([[[-0.5, -0.4, Z], [0.6, -0.5, Z], [0.05, 0.7, Z]]])
    H = W = 32
    p2f, zbuf, bary, dists = O.raster_fwd(fv, first, count, H, W)
    inside = p2f[0, ..., 0] == 0
    assert inside.sum() > 100
    assert torch.allclose(zbuf[0, ..., 0][inside], torch.full_like(zbuf[0, ..., 0][inside], Z), rtol=2e-7, atol=0)
    assert torch.allclose(bary[0, ..., 0, :][inside].sum(-1), torch.ones(int(inside.sum())), atol=1e-6)
    assert (dists[0, ..., 0][inside] < 0).all()
    # background sentinels
    assert (zbuf[0, ..., 0][~inside] == -1).all() and (dists[0, ..., 0][~inside] == -1).all()
    assert (bary[0, ..., 0, :][~inside] == -1).all()
    # analytic point-in-triangle (float64) on unambiguous pixels
    ys = np.array([spec_np.pix_to_ndc(H - 1 - i, H, W) for i in range(H)])
    xs = np.array([spec_np.pix_to_ndc(W - 1 - i, W, H) for i in range(W)])
    Px, Py = np.meshgrid(xs, ys)
    v = fv[0, :, :2].double().numpy()

    def e(a, b):
        return (Px - a[0]) * (b[1] - a[1]) - (Py - a[1]) * (b[0] - a[0])

    E = np.stack([e(v[1], v[2]), e(v[2], v[0]), e(v[0], v[1])], -1)
    sgn = np.sign(e(v[2], v[0])[0, 0] * 0 + ((v[2][0] - v[0][0]) * (v[1][1] - v[0][1]) - (v[2][1] - v[0][1]) * (v[1][0] - v[0][0])))
    ins = (E * sgn > 0).all(-1)
    clear = (np.abs(E) > 1e-5).all(-1)
    assert np.array_equal(ins[clear], inside.numpy()[clear])


def test_perspective_correct_depth_on_tilted_plane():
    # plane Z = a + b*X in view space, pinhole ndc = (X/Z, Y/Z); exact depth along the
    # pixel ray (x, y, 1) is Z = a / (1 - b x)
    a, b = 3.0, 0.8
    Xs = [(-1.0, -1.0), (1.2, -1.0), (1.2, 1.1), (-1.0, 1.1)]
    vv = [(X, Y, a + b * X) for X, Y in Xs]
    ndc = [(X / Z, Y / Z, Z) for X, Y, Z in vv]
    fv, first, count = _single([[ndc[0], ndc[1], ndc[2]], [ndc[0], ndc[2], ndc[3]]])
    H = W = 48
    p2f, zbuf, _, _ = O.raster_fwd(fv, first, count, H, W, persp=True)
    xs = torch.tensor([spec_np.pix_to_ndc(W - 1 - i, W, H) for i in range(W)]).float()
    cov = p2f[0, ..., 0] >= 0
    assert cov.sum() > 0.1 * H * W
    want = (a / (1 - b * xs))[None, :].expand(H, W)
    err = (zbuf[0, ..., 0] - want).abs()[cov]
    assert err.max() < 1e-5 * a, err.max()
    # without perspective correction the depth is affine in screen space -> visibly wrong
    _, zaff, _, _ = O.raster_fwd(fv, first, count, H, W, persp=False)
    assert (zaff[0, ..., 0] - want).abs()[cov].max() > 1e-3


def test_sphere_silhouette_area():
    verts, faces, _ = mesh_arrays("sphere")
    r = (verts.norm(dim=1)).mean().item()
    H = W = 96
    D = 3.0
    R = torch.eye(3)[None]
    T = torch.tensor([[0.0, 0.0, D]])
    f = 1.0 / math.tan(math.radians(30.0))
    intr = torch.tensor([[f, 0.0, f, 0.0]])
    fv = O.project_faces_c(verts, faces, O.views_tensor(R, T, intr))
    p2f, _, _, _ = O.raster_fwd(fv, torch.zeros(1, dtype=torch.int64), torch.tensor([faces.shape[0]]), H, W)
    area_px = (p2f >= 0).sum().item()
    rad_ndc = f * r / math.sqrt(D * D - r * r)
    want = math.pi * (rad_ndc * W / 2) ** 2
    assert abs(area_px - want) / want < 0.03, (area_px, want)


def test_k_ordering_and_consistency():
    verts, faces, _ = mesh_arrays("sphere")
    R, T, intr, _ = canonical_views(verts, 1, 40, 40)
    fv = O.project_faces_c(verts, faces, O.views_tensor(R, T, intr))
    first, count = torch.zeros(1, dtype=torch.int64), torch.tensor([faces.shape[0]])
    p1, z1, b1, d1 = O.raster_fwd(fv, first, count, 40, 40, K=1)
    p3, z3, b3, d3 = O.raster_fwd(fv, first, count, 40, 40, K=3)
    assert torch.equal(p1[..., 0], p3[..., 0]) and torch.equal(z1[..., 0], z3[..., 0])
    two = p3[..., 1] >= 0
    assert two.any() and (z3[..., 1][two] >= z3[..., 0][two]).all()
    assert (p3[..., 1][two] != p3[..., 0][two]).all()


@pytest.mark.parametrize("name,H,W,persp", [("cow", 40, 48, True), ("teapot", 32, 32, False)])
def test_c_oracle_matches_float64_spec(name, H, W, persp):
    verts, faces, _ = mesh_arrays(name)
    R, T, intr, _ = canonical_views(verts, 2, H, W, seed=3)
    fv = O.project_faces_c(verts, faces, O.views_tensor(R, T, intr))
    Fn = faces.shape[0]
    first, count = torch.arange(2) * Fn, torch.full((2,), Fn)
    p2f, zbuf, bary, dists = O.raster_fwd(fv, first, count, H, W, persp=persp)
    sp, sz, sb, sd, gap = spec_np.rasterize(fv.numpy(), first.numpy(), count.numpy(), H, W, persp=persp)
    # ambiguous pixels: near-tie in depth or a barycentric within float32 noise of 0
    near_edge = (np.abs(sb[..., 0, :]) < 1e-5).any(-1) & (sp[..., 0] >= 0)
    amb = (gap < 1e-5 * np.abs(sz[..., 0]).clip(1)) | near_edge
    got = p2f[..., 0].numpy()
    ok = ~amb
    assert ok.mean() > 0.95
    assert np.array_equal(got[ok], sp[..., 0][ok])
    both = ok & (got >= 0)
    assert np.abs(zbuf[..., 0].numpy()[both] - sz[..., 0][both]).max() < 1e-5
    assert np.abs(bary[..., 0, :].numpy()[both] - sb[..., 0, :][both]).max() < 1e-4
    assert np.abs(dists[..., 0].numpy()[both] - sd[..., 0][both]).max() < 1e-6


def _pixel_math_torch(fv, p2f, H, W, persp):
    """float64 differentiable restatement of (zbuf, bary, dists) at covered pixels."""
    N = p2f.shape[0]
    ys = torch.tensor([spec_np.pix_to_ndc(H - 1 - i, H, W) for i in range(H)], dtype=torch.float64)
    xs = torch.tensor([spec_np.pix_to_ndc(W - 1 - i, W, H) for i in range(W)], dtype=torch.float64)
    idx = (p2f[..., 0] >= 0).nonzero()
    f = p2f[..., 0][p2f[..., 0] >= 0]
    px, py = xs[idx[:, 2]], ys[idx[:, 1]]
    v = fv[f]
    x0, y0, z0 = v[:, 0, 0], v[:, 0, 1], v[:, 0, 2]
    x1, y1, z1 = v[:, 1, 0], v[:, 1, 1], v[:, 1, 2]
    x2, y2, z2 = v[:, 2, 0], v[:, 2, 1], v[:, 2, 2]

    def e(ax, ay, bx, by):
        return (px - ax) * (by - ay) - (py - ay) * (bx - ax)

    area = (x2 - x0) * (y1 - y0) - (y2 - y0) * (x1 - x0) + 1e-8
    w = torch.stack([e(x1, y1, x2, y2), e(x2, y2, x0, y0), e(x0, y0, x1, y1)], -1) / area[:, None]
    if persp:
        top = torch.stack([w[:, 0] * z1 * z2, w[:, 1] * z0 * z2, w[:, 2] * z0 * z1], -1)
        w = top / top.sum(-1, keepdim=True).clamp(min=1e-8)
    z = w[:, 0] * z0 + w[:, 1] * z1 + w[:, 2] * z2

    def seg(ax, ay, bx, by):
        dx, dy = bx - ax, by - ay
        t = (((px - ax) * dx + (py - ay) * dy) / (dx * dx + dy * dy)).clamp(0, 1)
        qx, qy = ax + t * dx, ay + t * dy
        return (px - qx) ** 2 + (py - qy) ** 2

    d = torch.stack([seg(x0, y0, x1, y1), seg(x0, y0, x2, y2), seg(x1, y1, x2, y2)], -1).min(-1).values
    inside = (w > 0).all(-1)
    sd = torch.where(inside, -d, d)
    return idx, z, w, sd


def test_c_backward_matches_float64_autograd():
    verts, faces, _ = mesh_arrays("cow")
    H, W = 40, 40
    R, T, intr, _ = canonical_views(verts, 2, H, W, seed=5)
    fv = O.project_faces_c(verts, faces, O.views_tensor(R, T, intr))
    Fn = faces.shape[0]
    first, count = torch.arange(2) * Fn, torch.full((2,), Fn)
    p2f, zbuf, bary, dists = O.raster_fwd(fv, first, count, H, W)
    g = torch.Generator().manual_seed(2)
    gz = torch.rand(zbuf.shape, generator=g) - 0.5
    gb = torch.rand(bary.shape, generator=g) - 0.5
    gd = (torch.rand(dists.shape, generator=g) - 0.5) * 1e-3
    got = O.raster_bwd(fv, p2f, gz, gb, gd)
    fv64 = fv.double().requires_grad_(True)
    idx, z, w, sd = _pixel_math_torch(fv64, p2f, H, W, True)
    sel = tuple(idx.T)
    loss = (gz[..., 0][sel].double() * z).sum() + (gb[..., 0, :][sel].double() * w).sum() + \
        (gd[..., 0][sel].double() * sd).sum()
    loss.backward()
    ref = fv64.grad.float()
    scale = ref.abs().max().item()
    assert (got - ref).abs().max().item() < 2e-3 * scale


@pytest.mark.parametrize("fname", sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz")) if os.path.isdir(GOLDEN)
                         else [])
def test_golden_fixtures_reproduce(fname):
    with np.load(os.path.join(GOLDEN, fname), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    fv = torch.from_numpy(d["face_verts"])
    first, count = torch.from_numpy(d["first"]), torch.from_numpy(d["count"])
    H, W, K = (int(x) for x in d["hwk"])
    p2f, zbuf, bary, dists = O.raster_fwd(fv, first, count, H, W, K, float(d["blur"]), bool(d["persp"]))
    assert np.array_equal(p2f.numpy(), d["pix_to_face"])
    assert np.array_equal(zbuf.numpy().view(np.int32), d["zbuf"].view(np.int32))
    assert np.array_equal(bary.numpy().view(np.int32), d["bary"].view(np.int32))
    assert np.array_equal(dists.numpy().view(np.int32), d["dists"].view(np.int32))


def test_oracle_under_address_and_ub_sanitizers():
    """the C restatement built with -fsanitize=address,undefined and driven through
    every entry point (forward, neighbour rule, pair mode, window, K > 1, blur, backward,
    projection) runs clean."""
    import os
    import shutil
    import subprocess

    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    if shutil.which(os.environ.get("CC", "gcc")) is None:
        pytest.skip("no C compiler")
    subprocess.run(["make", "-s", "-C", here, "asan"], check=True)
    r = subprocess.run([os.path.join(here, "asan_driver")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ERROR" not in r.stderr and "runtime error" not in r.stderr, r.stderr
