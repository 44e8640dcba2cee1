"""Round-5 GPU checks:

* The lazy K = 1 Fragments of MeshRasterizer (camera_pose_optimizer.py:244-246) use what the call saw:
  a zbuf first read inside a no_grad block still carries the call's autograd graph, and an in-place
  vertex edit between the call and the first read raises instead of rasterizing the edited mesh.
* The reshade entry (one raster shared by the zbuf / silhouette / Phong calls of one step) never pins a
  workspace: after an inference render whose outputs are discarded the workspace is freed.
* Fixed-point face totals: the vertex gradient of a batch is bitwise the same whatever the view order
  inside the batch (the integer sums are order-independent; the per-view R / T gradients permute with
  the views).
"""
import gc

import pytest
import torch

from torch_renderer_amd import kernels as Kn
from torch_renderer_amd.assets import load_asset
from torch_renderer_amd.cameras import FoVPerspectiveCameras
from torch_renderer_amd.mesh_renderer import MeshRasterizer, RasterizationSettings, _LazyFragments
from torch_renderer_amd.structures import Meshes
from torch_renderer_amd.transforms import look_at_view_transform

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _cow_views(N, dist=0.7):
    base = load_asset("cow", device=DEV, textures=False)
    v0, f0 = base.shared_verts().detach(), base.shared_faces()
    R, T = look_at_view_transform(dist, torch.linspace(5, 60, N), torch.linspace(0, 330, N), device=DEV,
                                  at=(v0.mean(0).tolist(),))
    return v0, f0, R, T


def test_lazy_fragments_capture_call_state():
    N, H = 3, 96
    v0, f0, R, T = _cow_views(N)
    rast = MeshRasterizer(cameras=FoVPerspectiveCameras(device=DEV),
                          raster_settings=RasterizationSettings(image_size=H, faces_per_pixel=1))
    v = v0.clone().requires_grad_(True)
    frags = rast(meshes_world=Meshes([v], [f0]).extend(N), R=R, T=T)
    assert isinstance(frags, _LazyFragments)
    with torch.no_grad():
        z = frags.zbuf  # first read under no_grad: the call ran with grad enabled
    assert z.requires_grad and z.grad_fn is not None
    torch.relu(z[..., 0]).sum().backward()
    assert v.grad is not None and v.grad.abs().sum() > 0
    v2 = v0.clone()
    frags2 = rast(meshes_world=Meshes([v2], [f0]).extend(N), R=R, T=T)
    v2.add_(0.01)  # in place, before the first access
    with pytest.raises(RuntimeError, match="modified in place"):
        _ = frags2.zbuf


def test_reshade_entry_does_not_pin_the_workspace():
    N, H = 4, 128
    v0, f0, R, T = _cow_views(N)
    cfg = Kn.ShadeConfig(H=H, W=H)
    cc = torch.zeros(1, 3, device=DEV)
    intr = torch.tensor([[2.0, 0.0, 2.0, 0.0]], device=DEV).expand(N, 4).contiguous()
    Kn._RESHADE["entry"] = None
    with torch.no_grad():
        Kn.render_views(v0, R, T, f0, intr, cc, cfg)
    gc.collect()
    ent = Kn._RESHADE["entry"]
    assert ent is not None and ent["ws"]() is None, "an inference render pinned its workspace"
    # with a graph alive the workspace stays reachable (and reusable) until the backward
    v = v0.clone().requires_grad_(True)
    out = Kn.render_views(v, R, T, f0, intr, cc, cfg)
    ent = Kn._RESHADE["entry"]
    assert ent["ws"]() is not None
    out["depth"].sum().backward()
    del out
    gc.collect()
    assert Kn._RESHADE["entry"]["ws"]() is None, "the workspace outlived its graph"
    Kn._RESHADE["entry"] = None


def test_second_backward_over_one_forward():
    """retain_graph: a second backward over the same forward workspace clears the face totals the first
    one consumed (the C++ node tracks the first use; MR_GRAD_ROWS_CLEARED only on it): both backwards give
    the same, bitwise, vertex and pose gradients."""
    N, H = 4, 128
    v0, f0, R, T = _cow_views(N)
    cfg = Kn.ShadeConfig(H=H, W=H)
    cc = torch.zeros(1, 3, device=DEV)
    intr = torch.tensor([[2.0, 0.0, 2.0, 0.0]], device=DEV).expand(N, 4).contiguous()
    v = v0.clone().requires_grad_(True)
    Rg = R.clone().requires_grad_(True)
    out = Kn.render_views(v, Rg, T, f0, intr, cc, cfg)
    loss = out["depth"].sum() + out["sil"].sum() + out["rgb"].sum()
    loss.backward(retain_graph=True)
    g1, r1 = v.grad.clone(), Rg.grad.clone()
    v.grad = None
    Rg.grad = None
    loss.backward()
    assert torch.equal(v.grad, g1) and torch.equal(Rg.grad, r1)


def test_vertex_grad_independent_of_view_order():
    N, H = 16, 192
    v0, f0, R, T = _cow_views(N, dist=0.6)
    intr = torch.tensor([[2.0, 0.0, 2.0, 0.0]], device=DEV).expand(N, 4).contiguous()
    cfg = Kn.ShadeConfig(H=H, W=H)
    cc = torch.zeros(1, 3, device=DEV)
    g = torch.Generator().manual_seed(3)
    gD, gS, gC = (torch.rand(N, H, H, generator=g).to(DEV) - 0.5, torch.rand(N, H, H, generator=g).to(DEV) - 0.5,
                  torch.rand(N, H, H, 3, generator=g).to(DEV) - 0.5)
    perm = torch.randperm(N, generator=g).to(DEV)

    def run(p):
        v = v0.clone().requires_grad_(True)
        Rp, Tp = R[p].clone().requires_grad_(True), T[p].clone().requires_grad_(True)
        Kn._RESHADE["entry"] = None
        out = Kn.render_views(v, Rp, Tp, f0, intr, cc, cfg)
        ((out["depth"] * gD[p]).sum() + (out["sil"] * gS[p]).sum() + (out["rgb"] * gC[p]).sum()).backward()
        torch.cuda.synchronize()
        return v.grad, Rp.grad, Tp.grad

    ident = torch.arange(N, device=DEV)
    va, Ra, Ta = run(ident)
    vb, Rb, Tb = run(perm)
    print(f"[determinism] vertex grad under a view permutation: max |diff| = {(va - vb).abs().max().item():.3e}")
    assert torch.equal(va, vb)
    assert torch.equal(Ra[perm], Rb) and torch.equal(Ta[perm], Tb)


@pytest.mark.parametrize("clip", [False, True])
def test_geometry_only_backward_equals_full(clip):
    """A backward without an RGB gradient (depth / silhouette renders: camera_pose_optimizer.py:244,248) runs
    the geometry-only k_bwd_fused (no Phong / texture backward, 9 values per face row). Its vertex and pose
    gradients equal, bitwise, those of the full kernel given an all-zero RGB gradient."""
    N, H = 4, 160
    v0, f0, R, T = _cow_views(N, dist=0.4 if clip else 0.7)
    intr = torch.tensor([[2.0, 0.0, 2.0, 0.0]], device=DEV).expand(N, 4).contiguous()
    cfg = Kn.ShadeConfig(H=H, W=H, clip=False, z_clip=0.3 if clip else None)
    cc = torch.zeros(1, 3, device=DEV)
    g = torch.Generator().manual_seed(4)
    gD = (torch.rand(N, H, H, generator=g) - 0.5).to(DEV)
    gS = (torch.rand(N, H, H, generator=g) - 0.5).to(DEV)

    def run(zero_rgb):
        v = v0.clone().requires_grad_(True)
        Rg, Tg = R.clone().requires_grad_(True), T.clone().requires_grad_(True)
        Kn._RESHADE["entry"] = None
        out = Kn.render_views(v, Rg, Tg, f0, intr, cc, cfg)
        loss = (out["depth"] * gD).sum() + (out["sil"] * gS).sum()
        if zero_rgb:
            loss = loss + (out["rgb"] * 0.0).sum()
        loss.backward()
        torch.cuda.synchronize()
        return v.grad, Rg.grad, Tg.grad

    geo, full = run(False), run(True)
    assert geo[0].abs().max() > 0
    for a, b, nm in zip(geo, full, ("verts", "R", "T")):
        assert torch.equal(a, b), f"{nm}: geometry-only backward differs from the full kernel's"


@pytest.mark.parametrize("ambient_vcol", [False, True])
def test_float_remainder_rows_are_read(ambient_vcol):
    """Gradient totals in fixed point carry components of magnitude >= 2^30 in float remainder rows, which the
    vertex-gradient gathers read only once k_bwd_fused has flagged one (ctr[CTR_FLT]). Upstream gradients scaled
    by 2^44 (exact in float: the backward is linear in them) push most run totals into the remainder rows: the
    vertex and pose gradients must still be 2^44 times the unscaled ones (to float rounding). ambient_vcol: ambient
    light and vertex colours (mesh_deformer.py's C5 shading: no normal chain, k_rt_vgrad_b, colour gradients too)."""
    N, H = 4, 160
    v0, f0, R, T = _cow_views(N)
    intr = torch.tensor([[2.0, 0.0, 2.0, 0.0]], device=DEV).expand(N, 4).contiguous()
    cfg = Kn.ShadeConfig(H=H, W=H)
    tex, vc0 = None, None
    if ambient_vcol:
        cfg.light_kind = 1
        cfg.light_ambient = (1.0, 1.0, 1.0)
        tex = Kn.TextureArgs(kind=1)
        vc0 = (0.5 + 0.5 * torch.sin(3.0 * v0)).contiguous()
    cc = torch.zeros(1, 3, device=DEV)
    g = torch.Generator().manual_seed(9)
    gD = (torch.rand(N, H, H, generator=g) - 0.5).to(DEV)
    gS = (torch.rand(N, H, H, generator=g) - 0.5).to(DEV)
    gC = (torch.rand(N, H, H, 3, generator=g) - 0.5).to(DEV)

    def run(scale):
        v = v0.clone().requires_grad_(True)
        Rg, Tg = R.clone().requires_grad_(True), T.clone().requires_grad_(True)
        vc = vc0.clone().requires_grad_(True) if vc0 is not None else None
        Kn._RESHADE["entry"] = None
        out = Kn.render_views(v, Rg, Tg, f0, intr, cc, cfg, tex, vcolors=vc)
        ((out["depth"] * gD * scale).sum() + (out["sil"] * gS * scale).sum() + (out["rgb"] * gC * scale).sum()).backward()
        torch.cuda.synchronize()
        return (v.grad, Rg.grad, Tg.grad) + ((vc.grad,) if vc is not None else ())

    s = 2.0 ** 44
    small, big = run(1.0), run(s)
    assert big[0].abs().max() > 2.0 ** 31  # the remainder rows were in play
    for a, b, nm in zip(small, big, ("verts", "R", "T", "colours")):
        err = (b / s - a).abs().max().item()
        tol = 1e-5 * max(a.abs().max().item(), 1e-30)
        assert err <= tol, f"{nm}: scaled gradient off by {err:.3e} (tolerance {tol:.3e})"
