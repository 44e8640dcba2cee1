"""Round-6 GPU checks (VERDICT r5 "next" #3):

* No render graph outlives its step: after a fused fwd+bwd and ``del`` of the outputs the leaves' AccumulateGrad
  nodes are gone, and a HIP graph captured after eager steps on the default stream (bench.py's sequence) runs
  without torch's AccumulateGrad stream-mismatch warning — the precondition of round 5's capture crash — and
  replays the eager step's gradients bitwise.
* A reshade of one raster with another texture kind (a depth render, then a vertex-colour Phong render of the
  same geometry, backward through the Phong output only) gives the gradients of a fresh render: the forward
  clears all 27 face-total columns, whatever the first call's texture.
* Run totals beyond the fixed-point cutoff (upstream gradients scaled so that per-(view, tile) runs reach ~2^28)
  take the float rows: the scaled gradients equal the unscaled ones times the scale.
* With vertex colours (corner-major 27-column face rows) the geometry-only backward equals the full kernel's.
"""
import warnings

import pytest
import torch

from tests.helpers import canonical_views, mesh_arrays
from torch_renderer_amd import kernels as Kn
from torch_renderer_amd.structures import Meshes, TexturesUV
from torch_renderer_amd.torch_renderer import DepthColorRender

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _acc_node(t):
    v = t.view_as(t)
    return v.grad_fn.next_functions[0][0]


def _cow(N, H, W):
    verts, faces, d = mesh_arrays("cow")
    img = torch.from_numpy(d["texture_u8"].astype("float32") / 255.0)
    vuv = torch.from_numpy(d["verts_uvs"]).float()
    fuv = torch.from_numpy(d["faces_uvs"]).long()
    tex = TexturesUV(maps=[img.to(DEV)], faces_uvs=[fuv.to(DEV)], verts_uvs=[vuv.to(DEV)])
    _, _, _, (R_cv, t_cv, K) = canonical_views(verts, N, H, W, dist=0.5)
    return verts, faces, tex, R_cv, t_cv, K


def _grads(N, H, W, seed=1, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return [((torch.rand(*s, generator=g) * 2 - 1) * scale).to(DEV) for s in ((N, H, W), (N, H, W), (N, H, W, 3))]


def test_no_autograd_graph_outlives_the_step():
    N, H = 4, 128
    verts, faces, tex, R_cv, t_cv, K = _cow(N, H, H)
    v = verts.to(DEV).requires_grad_(True)
    R = R_cv.to(DEV).contiguous().requires_grad_(True)
    t = t_cv.to(DEV).contiguous().requires_grad_(True)
    ren = DepthColorRender(K.to(DEV), (H, H), device=DEV)
    bm = Meshes([v], [faces.to(DEV)], tex).extend(N)
    g = _grads(N, H, H)
    leaves = {"verts": v, "R": R, "t": t}
    outs = ren.render(bm, R, t)
    for k, x in leaves.items():  # tag the nodes this graph holds
        _acc_node(x).metadata["r6"] = k
    torch.autograd.backward(list(outs), g)
    del outs
    alive = [k for k, x in leaves.items() if _acc_node(x).metadata.get("r6") == k]
    assert not alive, f"the render's autograd graph is still alive after del (AccumulateGrad of {alive})"


def test_hip_graph_capture_after_default_stream_steps():
    """bench.py's sequence: eager warm-up steps on the default stream, two on a side stream, one captured
    fwd+bwd, replays; then an eager step with the static outputs detached. No AccumulateGrad stream-mismatch
    warning anywhere, and the replay's gradients equal the eager step's bitwise."""
    N, H = 8, 128
    verts, faces, tex, R_cv, t_cv, K = _cow(N, H, H)
    v = verts.to(DEV).requires_grad_(True)
    R = R_cv.to(DEV).contiguous().requires_grad_(True)
    t = t_cv.to(DEV).contiguous().requires_grad_(True)
    ren = DepthColorRender(K.to(DEV), (H, H), device=DEV)
    bm = Meshes([v], [faces.to(DEV)], tex).extend(N)
    g = _grads(N, H, H)

    def step():
        v.grad = R.grad = t.grad = None
        torch.autograd.backward(list(ren.render(bm, R, t)), g)

    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        for _ in range(3):
            step()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                step()
        torch.cuda.current_stream().wait_stream(side)
        v.grad = R.grad = t.grad = None
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=torch.cuda.graph_pool_handle()):
            outs = ren.render(bm, R, t)
            torch.autograd.backward(list(outs), g)
        outs = tuple(o.detach() for o in outs)
        for _ in range(2):
            graph.replay()
        torch.cuda.synchronize()
        got = (v.grad.clone(), R.grad.clone(), t.grad.clone())
        step()
        torch.cuda.synchronize()
    bad = [str(x.message)[:120] for x in w if "AccumulateGrad" in str(x.message)]
    assert not bad, bad
    for a, b in zip(got, (v.grad, R.grad, t.grad)):
        assert torch.equal(a, b)
    del graph, outs


def test_reshade_with_another_texture_kind():
    """a depth render (TextureArgs(0): 18 face-total columns in use) followed by a Phong render
    of the same geometry with vertex colours (TextureArgs(1): 27 columns) re-shades the first call's raster; the
    Phong node's backward (the first over that workspace, MR_GRAD_ROWS_CLEARED) adds 27 columns. Its gradients
    equal those of a fresh render of the Phong call alone."""
    N, H = 3, 96
    verts, faces, _, R_cv, t_cv, K = _cow(N, H, H)
    Rp, Tp, intr, _ = canonical_views(verts, N, H, H, dist=0.5)
    gen = torch.Generator().manual_seed(7)
    vcol0 = torch.rand(verts.shape, generator=gen)
    gC = _grads(N, H, H, seed=9)[2]
    cc = torch.zeros(1, 3, device=DEV)
    R, T, it, f = Rp.to(DEV).contiguous(), Tp.to(DEV).contiguous(), intr.to(DEV).contiguous(), faces.to(DEV)
    cfg_d = Kn.ShadeConfig(H=H, W=H, want_depth=True, want_sil=False, want_rgb=False)
    cfg_c = Kn.ShadeConfig(H=H, W=H, want_depth=False, want_sil=False, want_rgb=True)

    def run(reshade):
        Kn._RESHADE["entry"] = None
        Kn._RESHADE["enabled"] = reshade
        try:
            v = verts.to(DEV).requires_grad_(True)
            vc = vcol0.to(DEV).requires_grad_(True)
            Rg, Tg = R.clone().requires_grad_(True), T.clone().requires_grad_(True)
            depth = None
            if reshade:
                depth = Kn.render_views(v, Rg, Tg, f, it, cc, cfg_d)["depth"]
                assert len(Kn._RESHADE["entry"]["served"]) == 1
            rgb = Kn.render_views(v, Rg, Tg, f, it, cc, cfg_c, Kn.TextureArgs(1), vcolors=vc)["rgb"]
            if reshade:  # the Phong call re-shaded the depth call's raster
                assert len(Kn._RESHADE["entry"]["served"]) == 2
            (rgb * gC).sum().backward()
            torch.cuda.synchronize()
            del depth
            return rgb.detach(), v.grad, vc.grad, Rg.grad, Tg.grad
        finally:
            Kn._RESHADE["enabled"] = True
            Kn._RESHADE["entry"] = None

    a, b = run(True), run(False)
    for nm, x, y in zip(("rgb", "grad verts", "grad vcolors", "grad R", "grad T"), a, b):
        assert torch.equal(x, y), f"reshade {nm} differs from a fresh render (max {(x - y).abs().max().item():.3e})"


def test_large_run_totals_take_the_float_rows():
    """upstream gradients scaled by 2^24 put per-(view, tile) run totals around 2^28 and
    face totals far beyond the fixed-point range (+-2^31; with round 5's 2^30 cutoff they wrapped): runs past
    the cutoff (2^24) are added in float, and the scaled vertex / pose gradients equal the unscaled ones times
    2^24 (float rounding apart)."""
    N, H = 8, 256
    verts, faces, tex, R_cv, t_cv, K = _cow(N, H, H)
    scale = 2.0 ** 24

    def run(sc):
        v = verts.to(DEV).requires_grad_(True)
        R = R_cv.to(DEV).contiguous().requires_grad_(True)
        t = t_cv.to(DEV).contiguous().requires_grad_(True)
        outs = DepthColorRender(K.to(DEV), (H, H), device=DEV).render(Meshes([v], [faces.to(DEV)], tex).extend(N), R, t)
        torch.autograd.backward(list(outs), _grads(N, H, H, seed=5, scale=sc))
        return v.grad, R.grad, t.grad

    base = run(1.0)
    big = run(scale)
    assert float(base[0].abs().max()) * scale > 2.0 ** 33, "the scaled totals do not leave the fixed-point range"
    for nm, a, b in zip(("verts", "R", "t"), big, base):
        err = (a / scale - b).abs().max().item()
        tol = 1e-5 * b.abs().max().item()
        print(f"[parity] scaled x2^24 grad {nm}: max |g/2^24 - g| = {err:.3e} (tol {tol:.3e})")
        assert torch.isfinite(a).all() and err <= tol, nm


@pytest.mark.parametrize("clip", [False, True])
def test_geometry_only_backward_equals_full_vertex_colours(clip):
    """With vertex colours (27-column face rows, corner-major since round 6: col_pos / col_rgb / col_nrm) the
    geometry-only backward places its 9 position values at the full kernel's position columns: vertex and pose
    gradients equal, bitwise, those of the full kernel given an all-zero RGB gradient, and no colour gradient
    arrives from either (as test_gpu_round5's untextured case)."""
    from tests.test_gpu_round5 import _cow_views

    N, H = 4, 160
    v0, f0, R, T = _cow_views(N, dist=0.4 if clip else 0.7)
    intr = torch.tensor([[2.0, 0.0, 2.0, 0.0]], device=DEV).expand(N, 4).contiguous()
    cfg = Kn.ShadeConfig(H=H, W=H, clip=False, z_clip=0.3 if clip else None)
    cc = torch.zeros(1, 3, device=DEV)
    g = torch.Generator().manual_seed(5)
    gD = (torch.rand(N, H, H, generator=g) - 0.5).to(DEV)
    gS = (torch.rand(N, H, H, generator=g) - 0.5).to(DEV)
    col0 = torch.rand(v0.shape[0], 3, generator=g).to(DEV)

    def run(zero_rgb):
        v = v0.clone().requires_grad_(True)
        col = col0.clone().requires_grad_(True)
        Rg, Tg = R.clone().requires_grad_(True), T.clone().requires_grad_(True)
        Kn._RESHADE["entry"] = None
        out = Kn.render_views(v, Rg, Tg, f0, intr, cc, cfg, Kn.TextureArgs(1), vcolors=col)
        loss = (out["depth"] * gD).sum() + (out["sil"] * gS).sum()
        if zero_rgb:
            loss = loss + (out["rgb"] * 0.0).sum()
        loss.backward()
        torch.cuda.synchronize()
        return v.grad, Rg.grad, Tg.grad, col.grad

    geo, full = run(False), run(True)
    assert geo[0].abs().max() > 0
    for a, b, nm in zip(geo[:3], full[:3], ("verts", "R", "T")):
        assert torch.equal(a, b), f"{nm}: geometry-only backward differs from the full kernel's"
    assert geo[3] is None or geo[3].abs().max() == 0
    assert full[3] is None or full[3].abs().max() == 0
