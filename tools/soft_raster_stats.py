"""Work counts of the soft bench's K-deep raster (bench.py --mode soft: cow, 128^2, K = 50, the deform blur),
per occupied 8x8 tile: listed faces (padded bbox overlaps the tile), (face, pixel) pairs the kernel evaluates
(padded bbox clipped to the tile) and kept candidates (squared NDC distance to the triangle < blur, or inside).
CPU, torch; approximate camera model (NDC pinhole, focal 1) — counts, not parity.
Usage: python tools/soft_raster_stats.py [--views 64] [--size 128]"""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.transforms import look_at_view_transform  # noqa: E402


def seg_d2(px, py, ax, ay, bx, by):
    dx, dy = bx - ax, by - ay
    l2 = (dx * dx + dy * dy).clamp_min(1e-30)
    t = (((px - ax) * dx + (py - ay) * dy) / l2).clamp(0, 1)
    ex, ey = ax + t * dx - px, ay + t * dy - py
    return ex * ex + ey * ey


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=64)
    ap.add_argument("--size", type=int, default=128)
    a = ap.parse_args()
    H = W = a.size
    blur = math.log(1.0 / 1e-4 - 1.0) * 1e-4
    pad = math.sqrt(blur)
    m = load_asset("cow", textures=False)
    v0 = m.shared_verts().double()
    c = v0.mean(0)
    v = (v0 - c) / (v0 - c).abs().max()
    f = m.shared_faces().long()
    nv = a.views
    R, T = look_at_view_transform(dist=2.7, elev=torch.linspace(0, 360, nv), azim=torch.linspace(-180, 180, nv))
    tot = dict(tiles=0, faces=0, pairs=0, kept=0, px=0, over_k=0)
    per_tile_pairs, per_tile_kept, per_pix_kept, per_tile_faces = [], [], [], []
    for n in range(nv):
        vc = v @ R[n].double() + T[n].double()
        x, y = vc[:, 0] / vc[:, 2], vc[:, 1] / vc[:, 2]
        fx, fy = x[f], y[f]  # F x 3
        # pixel centres in NDC: col c -> 1 - (2c + 1) / W (sign irrelevant for counts)
        cx0 = ((1 - (fx.max(1).values + pad)) * W / 2 - 0.5).ceil().clamp(0, W - 1).long()
        cx1 = ((1 - (fx.min(1).values - pad)) * W / 2 - 0.5).floor().clamp(-1, W - 1).long()
        cy0 = ((1 - (fy.max(1).values + pad)) * H / 2 - 0.5).ceil().clamp(0, H - 1).long()
        cy1 = ((1 - (fy.min(1).values - pad)) * H / 2 - 0.5).floor().clamp(-1, H - 1).long()
        ok = (cx0 <= cx1) & (cy0 <= cy1)
        tiles = {}
        kept_img = torch.zeros(H, W, dtype=torch.int64)
        for i in torch.nonzero(ok).flatten().tolist():
            xs = torch.arange(cx0[i], cx1[i] + 1)
            ys = torch.arange(cy0[i], cy1[i] + 1)
            PY, PX = torch.meshgrid(ys, xs, indexing="ij")
            pxn = 1 - (2 * PX.double() + 1) / W
            pyn = 1 - (2 * PY.double() + 1) / H
            ax, ay, bx, by, qx, qy = fx[i, 0], fy[i, 0], fx[i, 1], fy[i, 1], fx[i, 2], fy[i, 2]
            d2 = torch.minimum(torch.minimum(seg_d2(pxn, pyn, ax, ay, bx, by), seg_d2(pxn, pyn, bx, by, qx, qy)),
                               seg_d2(pxn, pyn, qx, qy, ax, ay))
            e0 = (bx - ax) * (pyn - ay) - (by - ay) * (pxn - ax)
            e1 = (qx - bx) * (pyn - by) - (qy - by) * (pxn - bx)
            e2 = (ax - qx) * (pyn - qy) - (ay - qy) * (pxn - qx)
            inside = ((e0 >= 0) & (e1 >= 0) & (e2 >= 0)) | ((e0 <= 0) & (e1 <= 0) & (e2 <= 0))
            keep = inside | (d2 < blur)
            kept_img[PY[keep], PX[keep]] += 1
            for ty in range(int(cy0[i]) // 8, int(cy1[i]) // 8 + 1):
                for tx in range(int(cx0[i]) // 8, int(cx1[i]) // 8 + 1):
                    sel = (PY // 8 == ty) & (PX // 8 == tx)
                    t = tiles.setdefault((ty, tx), [0, 0, 0])
                    t[0] += 1
                    t[1] += int(sel.sum())
                    t[2] += int((sel & keep).sum())
        for t in tiles.values():
            tot["tiles"] += 1
            tot["faces"] += t[0]
            tot["pairs"] += t[1]
            tot["kept"] += t[2]
            per_tile_pairs.append(t[1])
            per_tile_faces.append(t[0])
            per_tile_kept.append(t[2])
        kp = kept_img[kept_img > 0]
        tot["px"] += int(kp.numel())
        tot["over_k"] += int((kp > 50).sum())
        per_pix_kept.append(kp)
    pp = torch.tensor(per_tile_pairs, dtype=torch.float64)
    ff = torch.tensor(per_tile_faces, dtype=torch.float64)
    kk = torch.tensor(per_tile_kept, dtype=torch.float64)
    px = torch.cat(per_pix_kept).double()
    print(f"views {nv}  occupied tiles {tot['tiles']} ({tot['tiles'] / nv:.1f}/view)")
    print(f"listed faces / tile  mean {tot['faces'] / tot['tiles']:.1f}  p90 {ff.quantile(0.9):.0f}  max {ff.max():.0f}"
          f"  tiles > 1536: {int((ff > 1536).sum())}  > 2048: {int((ff > 2048).sum())}")
    print(f"pairs / tile  mean {pp.mean():.0f}  p90 {pp.quantile(0.9):.0f}  max {pp.max():.0f}")
    print(f"kept / tile  mean {kk.mean():.0f}  p90 {kk.quantile(0.9):.0f}  max {kk.max():.0f}")
    print(f"covered px {tot['px']}  kept / px mean {px.mean():.1f}  p90 {px.quantile(0.9):.0f}  max {px.max():.0f}"
          f"  > K=50: {tot['over_k']}")


if __name__ == "__main__":
    main()
