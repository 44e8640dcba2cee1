"""Shared test scaffolding: canonical camera batches for any asset."""
import math

import numpy as np
import torch

from torch_renderer_amd.assets import load_asset_arrays
from torch_renderer_amd.transforms import opencv_look_at, opencv_to_pytorch3d


def mesh_arrays(name):
    d = load_asset_arrays(name)
    return torch.from_numpy(d["verts"]).float(), torch.from_numpy(d["faces"]).long(), d


def canonical_views(verts, N, H, W, dist=None, fov_deg=60.0, seed=0, elev_range=(-20.0, 60.0)):
    """OpenCV look-at cameras around the mesh centroid (azimuth 360*i/N, elevation ~U[range]),
    fx = fy from the FoV at width W, principal point at the image centre.
    Returns PyTorch3D-convention R (N,3,3), T (N,3), intr (N,4) and OpenCV (R_cv, t_cv, K)."""
    g = torch.Generator().manual_seed(seed)
    c = verts.mean(0)
    ext = (verts.max(0).values - verts.min(0).values).max().item()
    dist = dist if dist is not None else 2.2 * ext
    az = torch.arange(N, dtype=torch.float64) * (2 * math.pi / N)
    el = torch.empty(N, dtype=torch.float64).uniform_(math.radians(elev_range[0]), math.radians(elev_range[1]),
                                                      generator=g)
    C = torch.stack([dist * torch.cos(el) * torch.sin(az), dist * torch.sin(el), dist * torch.cos(el) * torch.cos(az)],
                    dim=1) + c.double()
    R_cv, t_cv = opencv_look_at(C, c.double())
    f = (W / 2.0) / math.tan(math.radians(fov_deg) / 2.0)
    K = torch.tensor([[f, 0.0, W / 2.0], [0.0, f, H / 2.0], [0.0, 0.0, 1.0]])
    R, T = opencv_to_pytorch3d(R_cv, t_cv)
    s = min(H, W) / 2.0
    intr = torch.tensor([[f / s, (W / 2.0 - K[0, 2].item()) / s, f / s, (H / 2.0 - K[1, 2].item()) / s]]).expand(N, 4)
    return R.float(), T.float(), intr.float().contiguous(), (R_cv, t_cv, K)


def cv_to_p3d(R, t):
    """torch_renderer.py:73-80 restated for the oracle side (R^T, negate columns 0,1; negate t0,t1)."""
    Rp = R.transpose(1, 2).clone()
    Rp[:, :, :2] = -Rp[:, :, :2]
    Tp = t.clone()
    Tp[:, :2] = -Tp[:, :2]
    return Rp, Tp


def intr_from_K(K, H, W, N):
    """(N,4) ax, bx, ay, by of PerspectiveCameras(in_ndc=False) for a pixel K (torch_renderer.py:61-71)."""
    s = min(H, W) / 2.0
    return torch.tensor([[K[0, 0] / s, (W / 2.0 - K[0, 2]) / s, K[1, 1] / s,
                          (H / 2.0 - K[1, 2]) / s]]).expand(N, 4).contiguous()


def fragment_grad_sensitivity(run_oracle, eps=1e-6, seeds=4):
    """How far float32 rounding can move the oracle's own gradients. `run_oracle()` runs the oracle
    forward + backward and returns a tuple of gradient tensors; it is re-run with the gradients
    reaching the fragments (zbuf, bary, dists of oracle.RasterizeRef) multiplied by (1 + eps * n),
    n ~ N(0,1) per entry (eps = 1e-6 is ~8 ulp). Returns (baseline grads, per-entry max |change|
    over the seeds). Sliver faces (projected area ~1e-5 px^2 on the teapot at 40x40) make the
    vertex gradient a difference of ~1/area^2-sized terms: there an 8-ulp change of an upstream
    gradient moves the result by more than the result itself, and neither side's f32 value is
    meaningful beyond that spread."""
    from oracle import oracle as O

    base = [g.detach().clone() for g in run_oracle()]
    sens = [torch.zeros_like(g) for g in base]
    orig = O.RasterizeRef.apply
    for seed in range(seeds):
        gen = torch.Generator().manual_seed(1000 + seed)

        def noisy(*a):
            out = orig(*a)
            for t in out[1:]:
                if t.requires_grad:
                    n = torch.randn(t.shape, generator=gen)
                    t.register_hook(lambda gr, n=n: None if gr is None else gr * (1 + eps * n))
            return out

        O.RasterizeRef.apply = noisy
        try:
            grads = run_oracle()
        finally:
            O.RasterizeRef.apply = orig
        for s, g, b in zip(sens, grads, base):
            torch.maximum(s, (g.detach() - b).abs(), out=s)
    return base, sens


def oracle_runs(run, seeds=4):
    """run(precision) -> flat tuple of tensors (oracle outputs and leaf gradients, in a fixed order).
    Returns (ref, ref64, spread): the f32 oracle, its float64 shadow (oracle.render_ref(precision=
    "f64"): same decisions, float64 arithmetic) and the per-entry conditioning spread = max of
    |ref - ref64| and of |ref' - ref| over `seeds` f32 runs under oracle.perturbed (fragment values
    moved by ~1 ulp, the gradients entering fragments and outputs by ~8 ulp). One sample of the f32
    error can be small by chance where the entry is ill-conditioned; the perturbed runs sample it
    again."""
    from oracle import oracle as O

    ref = [t.detach().clone() for t in run("f32")]
    r64 = [t.detach().clone() for t in run("f64")]
    spread = [(a.double() - b.double()).abs().float() for a, b in zip(ref, r64)]
    for sd in range(seeds):
        with O.perturbed(sd):
            rr = run("f32")
        spread = [torch.maximum(s, (x.detach().float() - a.float()).abs()) for s, x, a in zip(spread, rr, ref)]
    return ref, r64, spread


def report(name, got, ref, tol=1e-4, rel_above_one=True, sens=None, sens_factor=10.0, ref64=None):
    """Compare a GPU tensor with the oracle's, ENTRY BY ENTRY (north_star: 1e-4 on float depths,
    colours and vertex gradients).

    Bar per entry: |got_i - ref_i| <= bar_i = tol * max(1, |ref_i|) (rel_above_one; else tol
    absolute). Values of magnitude <= 1 (images, most gradient entries) are held to tol absolute;
    larger gradient entries (the 1/sigma = 1e4 factor of the soft blends) to tol relative to
    themselves.
    Conditioning: the f32 oracle is itself only f32-accurate. ref64 (the oracle's float64 shadow,
    oracle.render_ref(precision="f64") — same decisions, every value in float64) gives its own
    error spread_i = |ref_i - ref64_i|; sens (fragment_grad_sensitivity) the movement of its value
    under an 8-ulp perturbation of the fragment gradients. An entry whose spread exceeds a tenth
    of its bar is ill-conditioned in f32 (a difference of much larger terms, or a saturated
    sigmoid's 1 - p): it must lie within bar_i + sens_factor * spread_i instead, i.e. the GPU
    must be as accurate as the f32 reference there, within a factor. Prints the max error, the
    worst entry's error / its limit, the ill-conditioned count and, with ref64, how far the GPU
    and the f32 oracle each are from the float64 values."""
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    assert torch.isfinite(got).all(), f"{name}: non-finite values"
    d = (got - ref).abs()
    bar = tol * ref.abs().clamp(min=1.0) if rel_above_one else torch.full_like(ref, tol)
    lim = bar
    n_ill = 0
    spread = None
    if sens is not None:
        spread = sens.detach().float().cpu()
    if ref64 is not None:
        r64 = ref64.detach().double().cpu()
        assert r64.shape == ref.shape, (name, r64.shape, ref.shape)
        s64 = (ref.double() - r64).abs().float()
        spread = s64 if spread is None else torch.maximum(spread, s64)
    if spread is not None:
        ill = spread > 0.1 * bar
        n_ill = int(ill.sum())
        lim = torch.where(ill, bar + sens_factor * spread, bar)
    ratio = d / lim
    if ref64 is not None:
        # an entry within the bar of the float64 value is correct whatever the f32 oracle's own error
        d64 = (got.double() - r64).abs()
        ok64 = d64 <= tol * (r64.abs().clamp(min=1.0) if rel_above_one else torch.ones_like(r64))
        ratio = torch.where(ok64, torch.minimum(ratio, torch.ones_like(ratio)), ratio)
    n = ref.numel()
    err = d.max().item() if n else 0.0
    scale = ref.abs().max().item() if n else 0.0
    worst = ratio.max().item() if n else 0.0
    over = int((ratio > 1.0).sum()) if n else 0
    msg = (f"[parity] {name}: n = {n}, max|err| = {err:.3e}, scale = {scale:.3e}, worst err/limit = {worst:.3f}"
           + (f", ill-conditioned = {n_ill}" if spread is not None else ""))
    if ref64 is not None and n:
        g64 = ((got.double() - r64).abs() / bar.double()).max().item()
        o64 = ((ref.double() - r64).abs() / bar.double()).max().item()
        msg += f", vs f64: GPU {g64:.3f} / f32 oracle {o64:.3f} of the bar"
    if n:
        i = int(ratio.reshape(-1).argmax())
        idx = tuple(int(x) for x in np.unravel_index(i, tuple(got.shape)))
        msg += f" at {idx} (got {got.reshape(-1)[i].item():.6e}, ref {ref.reshape(-1)[i].item():.6e})"
    if over:
        msg += f"; {over} entries over their bar"
    print(msg)
    if over:  # the worst offenders, with the float64 value and the conditioning spread
        top = torch.topk(ratio.reshape(-1), min(over, 5)).indices
        for i in top.tolist():
            idx = tuple(int(x) for x in np.unravel_index(i, tuple(got.shape)))
            extra = f", f64 {r64.reshape(-1)[i].item():.7e}" if ref64 is not None else ""
            extra += f", spread {spread.reshape(-1)[i].item():.3e}" if spread is not None else ""
            print(f"[parity]     {idx}: got {got.reshape(-1)[i].item():.7e}, ref {ref.reshape(-1)[i].item():.7e}"
                  f"{extra}, err/limit {ratio.reshape(-1)[i].item():.3f}")
    assert over == 0, f"{name}: {over} entries exceed |err| <= {tol:g} * max(1, |ref|) (worst ratio {worst:.3f})"
    return err, scale
