"""Shared test scaffolding: canonical camera batches for any asset."""
import math

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
