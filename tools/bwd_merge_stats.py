"""How many per-face gradient rows the fused backward's atomics carry, and how many a wider merge would
leave (bench workload: cow, 64 views, 512x512). Rows today = runs of equal faces along the 8x8 tiles'
row-major pixel order; alternatives: distinct faces per tile, per group of G consecutive non-empty tiles
of a view (slot order), per (view, face)."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from torch_renderer_amd import distributed as D  # noqa: E402
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.cameras import PerspectiveCameras, view_batch  # noqa: E402
from torch_renderer_amd.kernels import RasterizeMeshesWorld, mesh_topology  # noqa: E402
from torch_renderer_amd.transforms import opencv_to_pytorch3d  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    H = W = 512
    nv = 64
    meshes = load_asset("cow", device=dev, textures=False)
    verts, faces = meshes.shared_verts(), meshes.shared_faces()
    R_all, t_all, K = bench.canonical_views(verts.cpu(), nv, H, W, dist_m=bench.view_distance("cow", verts.cpu()))
    Rp, Tp = opencv_to_pytorch3d(R_all.to(dev), t_all.to(dev))
    cams = PerspectiveCameras(focal_length=((float(K[0, 0]), float(K[1, 1])),),
                              principal_point=((float(K[0, 2]), float(K[1, 2])),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]), device=dev)
    Rb, Tb, intr = view_batch(cams, (H, W), Rp, Tp, n_views=nv)
    mesh_topology(faces, verts.shape[0])
    with torch.no_grad():
        out = RasterizeMeshesWorld.apply(verts, Rb.contiguous(), Tb.contiguous(), faces, intr.contiguous(), nv, H, W,
                                         1, 0.0, True, False, False, None)
    p2f = out[0][..., 0]  # (N, H, W) packed ids, -1 background
    T = (H // 8) * (W // 8)
    tiles = p2f.reshape(nv, H // 8, 8, W // 8, 8).permute(0, 1, 3, 2, 4).reshape(nv, T, 64)
    nonempty = (tiles >= 0).any(-1)
    covered = int((tiles >= 0).sum())
    slots = int(nonempty.sum())
    # runs of equal faces in lane order (lane = 8 * row + col) among covered lanes
    prev = torch.cat([torch.full_like(tiles[..., :1], -2), tiles[..., :-1]], -1)
    runs = int(((tiles >= 0) & (tiles != prev)).sum())
    # distinct faces per tile
    srt = tiles.sort(-1).values
    sprev = torch.cat([torch.full_like(srt[..., :1], -2), srt[..., :-1]], -1)
    per_tile = int(((srt >= 0) & (srt != sprev)).sum())
    print(f"covered {covered}, slots {slots} ({covered / slots / 64:.3f} lane use), rows: runs {runs}, "
          f"distinct per tile {per_tile}")
    # runs under other lane -> tile-pixel orders (lane L handles tile pixel perm[L])
    def morton(L):
        x = (L & 1) | ((L >> 1) & 2) | ((L >> 2) & 4)
        y = ((L >> 1) & 1) | ((L >> 2) & 2) | ((L >> 3) & 4)
        return 8 * y + x

    def hilbert(L):
        x = y = 0
        t, s = L, 1
        while s < 8:
            rx = 1 & (t // 2)
            ry = 1 & (t ^ rx)
            if ry == 0:
                if rx == 1:
                    x, y = s - 1 - x, s - 1 - y
                x, y = y, x
            x += s * rx
            y += s * ry
            t //= 4
            s *= 2
        return 8 * y + x

    orders = {"morton": [morton(L) for L in range(64)], "hilbert": [hilbert(L) for L in range(64)],
              "snake": [8 * (L // 8) + ((L % 8) if (L // 8) % 2 == 0 else 7 - L % 8) for L in range(64)],
              "col-major": [8 * (L % 8) + L // 8 for L in range(64)]}
    for name, perm in orders.items():
        assert sorted(perm) == list(range(64)), name
        tp = tiles[..., torch.tensor(perm, device=dev)]
        pv = torch.cat([torch.full_like(tp[..., :1], -2), tp[..., :-1]], -1)
        print(f"  runs in {name} order: {int(((tp >= 0) & (tp != pv)).sum())}")
    # distinct per group of G consecutive non-empty tiles of a view
    for G in (2, 4, 8, 16, 32):
        tot = 0
        for n in range(nv):
            t = tiles[n][nonempty[n]]  # (slots_n, 64)
            ns = t.shape[0]
            pad = (-ns) % G
            if pad:
                t = torch.cat([t, torch.full((pad, 64), -1, device=dev, dtype=t.dtype)], 0)
            g = t.reshape(-1, G * 64).sort(-1).values
            gp = torch.cat([torch.full_like(g[:, :1], -2), g[:, :-1]], -1)
            tot += int(((g >= 0) & (g != gp)).sum())
        print(f"  distinct per group of {G} slots: {tot}")
    vf = int(sum(int(torch.unique(p2f[n][p2f[n] >= 0]).numel()) for n in range(nv)))
    print(f"  distinct (view, face): {vf}; 18-float rows: runs {runs * 72 / 1e6:.1f} MB, per tile "
          f"{per_tile * 72 / 1e6:.1f} MB, per (view, face) {vf * 72 / 1e6:.1f} MB")


if __name__ == "__main__":
    main()
