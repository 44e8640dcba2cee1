"""Print the pixels where the HIP raster and the C oracle disagree, with both candidates."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import canonical_views, mesh_arrays  # noqa: E402
from oracle import oracle as O  # noqa: E402
from torch_renderer_amd import kernels as Kn  # noqa: E402

name, H, W, N = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
verts, faces, _ = mesh_arrays(name)
R, T, intr, _ = canonical_views(verts, N, H, W)
views = O.views_tensor(R, T, intr)
fv = O.project_faces_c(verts, faces, views)
F = faces.shape[0]
first = torch.arange(N) * F
count = torch.full((N,), F)
ref = O.raster_fwd(fv, first, count, H, W, 1, 0.0, True)
dev = torch.device("cuda:0")
got = [t.cpu() for t in Kn.rasterize_meshes_fwd(fv.to(dev), first.to(dev), count.to(dev), H, W, 1, 0.0, True)]
bad = (got[0] != ref[0]).nonzero()
print("mismatches", len(bad))
for n, y, x, k in bad[:10].tolist():
    fg, fr = got[0][n, y, x, 0].item(), ref[0][n, y, x, 0].item()
    print(f"view {n} px ({y},{x}) got f={fg} z={got[1][n,y,x,0].item()!r} ref f={fr} z={ref[1][n,y,x,0].item()!r}")
    for f in (fg, fr):
        if f >= 0:
            print("   face", f, fv[f].tolist())
