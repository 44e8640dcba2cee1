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


def report(name, got, ref, tol=1e-4, rel_above_one=True, sens=None, sens_factor=10.0):
    """Compare a GPU tensor with the oracle's. Prints the absolute error next to the value scale.
    Bar: |err| <= tol absolute for values of scale <= 1; for larger values (vertex / pose gradients,
    which carry the 1/sigma = 1e4 factor of the soft blends and sum thousands of f32 terms in a
    different order on each side) |err| <= tol * scale.
    sens (from fragment_grad_sensitivity): entries whose oracle value moves by more than a tenth of
    the bar under an 8-ulp perturbation of the fragment gradients are ill-conditioned; the scale
    and bar are taken over the well-conditioned entries, and an ill-conditioned entry must lie
    within bar + sens_factor * sens (its count and spread are printed)."""
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    assert torch.isfinite(got).all(), f"{name}: non-finite values"
    if sens is not None:
        sens = sens.detach().float().cpu()
        ill = sens > 0.1 * tol * ref.abs().clamp(min=1.0)
        well_scale = ref[~ill].abs().max().item() if bool((~ill).any()) else 0.0
        bar = tol * max(1.0, well_scale) if rel_above_one else tol
        ill |= sens > 0.1 * bar
        d = (got - ref).abs()
        n_ill = int(ill.sum())
        if n_ill:
            lim = bar + sens_factor * sens
            over = ill & (d > lim)
            print(f"[parity] {name}: {n_ill} ill-conditioned entries (oracle spread up to {sens[ill].max():.3e}, "
                  f"max|err| there {d[ill].max():.3e}); {int(over.sum())} outside bar + {sens_factor:g} x spread")
            assert not bool(over.any()), f"{name}: ill-conditioned entries beyond the oracle's own spread"
        got = torch.where(ill, ref, got)
    err = (got - ref).abs().max().item() if got.numel() else 0.0
    scale = ref.abs().max().item() if ref.numel() else 0.0
    if sens is not None:
        scale = well_scale
    bar = tol * max(1.0, scale) if rel_above_one else tol
    print(f"[parity] {name}: max|err| = {err:.3e}, scale = {scale:.3e}, bar = {bar:.3e}")
    if err > bar:
        i = int((got - ref).abs().reshape(-1).argmax())
        idx = np.unravel_index(i, tuple(got.shape))
        print(f"[parity]   worst at {tuple(int(x) for x in idx)}: got {got.reshape(-1)[i].item():.6e} "
              f"ref {ref.reshape(-1)[i].item():.6e}; #entries over bar: {int(((got - ref).abs() > bar).sum())}")
    assert err <= bar, f"{name}: max abs err {err:.3e} > {bar:.3e} (scale {scale:.3e})"
    return err, scale
