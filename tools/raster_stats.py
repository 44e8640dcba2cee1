"""Workload statistics of the raster pass on CPU (no GPU): per view, tile-list entries,
(face, pixel) pairs after clipping each face's pixel bbox to its 8x8 tile, and non-empty
64x8 strips. python tools/raster_stats.py [--mesh cow --views 8 --size 512 --dist 0.5]"""
import argparse
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402
from torch_renderer_amd.assets import load_asset_arrays  # noqa: E402
from torch_renderer_amd.transforms import opencv_to_pytorch3d  # noqa: E402


def pix_range(lo, hi, S1, S2):
    rng = 2.0 * S1 / S2 if S1 > S2 else 2.0
    off = rng / 2
    i_hi = ((hi + off) * S1 - off) / rng
    i_lo = ((lo + off) * S1 - off) / rng
    p0 = np.floor(np.clip(S1 - 1 - i_hi - 0.05, -2, S1 + 1)).astype(int)
    p1 = np.ceil(np.clip(S1 - 1 - i_lo + 0.05, -2, S1 + 1)).astype(int)
    return np.maximum(p0, 0), np.minimum(p1, S1 - 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mesh", default="cow")
    ap.add_argument("--views", type=int, default=8)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--dist", type=float, default=0.5)
    a = ap.parse_args()
    d = load_asset_arrays(a.mesh)
    verts = torch.from_numpy(d["verts"]).float()
    faces = torch.from_numpy(d["faces"]).long()
    H = W = a.size
    R_cv, t_cv, K = bench.canonical_views(verts, a.views, H, W, dist_m=a.dist)
    R, T = opencv_to_pytorch3d(R_cv, t_cv)
    s = min(H, W) / 2
    intr = torch.tensor([[K[0, 0] / s, 0.0, K[1, 1] / s, 0.0]]).expand(a.views, 4).contiguous()
    fv = O.project_faces_torch(verts, faces, R, T, intr).numpy().reshape(a.views, -1, 3, 3)
    tot = {"entries": 0, "pairs": 0, "strips": 0, "pairs_hist": np.zeros(65, int), "max_tile": 0}
    for n in range(a.views):
        v = fv[n]
        x0, x1 = pix_range(v[:, :, 0].min(1), v[:, :, 0].max(1), W, H)
        y0, y1 = pix_range(v[:, :, 1].min(1), v[:, :, 1].max(1), H, W)
        tile = np.zeros((math.ceil(H / 8), math.ceil(W / 8)), int)
        for f in range(v.shape[0]):
            if x0[f] > x1[f] or y0[f] > y1[f] or v[f, :, 2].max() < 0:
                continue
            for ty in range(y0[f] // 8, y1[f] // 8 + 1):
                for tx in range(x0[f] // 8, x1[f] // 8 + 1):
                    w = min(x1[f], tx * 8 + 7) - max(x0[f], tx * 8) + 1
                    h = min(y1[f], ty * 8 + 7) - max(y0[f], ty * 8) + 1
                    tot["entries"] += 1
                    tot["pairs"] += w * h
                    tot["pairs_hist"][w * h] += 1
                    tile[ty, tx] += 1
        strips = tile.reshape(tile.shape[0], -1, 8).sum(2)
        tot["strips"] += int((strips > 0).sum())
        tot["max_tile"] = max(tot["max_tile"], int(tile.max()))
    V = a.views
    print(f"{a.mesh} {H}x{W} dist {a.dist}: per view entries {tot['entries'] / V:.0f}, pairs {tot['pairs'] / V:.0f} "
          f"({tot['pairs'] / max(tot['entries'], 1):.1f}/entry), non-empty strips {tot['strips'] / V:.1f} of "
          f"{math.ceil(H / 8) * math.ceil(W / 64)}, max faces in a tile {tot['max_tile']}")
    h = tot["pairs_hist"]
    print("pairs/entry histogram (1,2,3-4,5-8,9-16,17-64):", h[1], h[2], h[3:5].sum(), h[5:9].sum(), h[9:17].sum(),
          h[17:].sum())


if __name__ == "__main__":
    main()
