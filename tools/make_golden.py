"""Generate tests/golden/*.npz from the C oracle (restated PyTorch3D CPU rasterizer).
Inputs (face_verts) are produced by the oracle projection from the bundled assets, so the
GPU parity tests can feed bit-identical floats. python tools/make_golden.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from tests.helpers import canonical_views, mesh_arrays  # noqa: E402

CASES = [  # name, mesh, views, H, W, K, blur, persp, seed
    ("sphere_32x32_k1", "sphere", 1, 32, 32, 1, 0.0, True, 0),
    ("teapot_40x56_k1_2v", "teapot", 2, 40, 56, 1, 0.0, True, 1),
    ("teapot_32x32_k3_affine", "teapot", 1, 32, 32, 3, 0.0, False, 2),
    ("cow_48x48_k1", "cow", 1, 48, 48, 1, 0.0, True, 3),
    ("dolphin_24x40_k2_blur", "dolphin", 1, 24, 40, 2, 1e-4, True, 4),
]

out = os.path.join(ROOT, "tests", "golden")
os.makedirs(out, exist_ok=True)
for name, mesh, N, H, W, K, blur, persp, seed in CASES:
    verts, faces, _ = mesh_arrays(mesh)
    R, T, intr, _ = canonical_views(verts, N, H, W, seed=seed)
    fv = O.project_faces_c(verts, faces, O.views_tensor(R, T, intr))
    Fn = faces.shape[0]
    first, count = torch.arange(N) * Fn, torch.full((N,), Fn)
    p2f, zbuf, bary, dists = O.raster_fwd(fv, first, count, H, W, K, blur, persp)
    np.savez_compressed(os.path.join(out, name + ".npz"), face_verts=fv.numpy(), first=first.numpy(),
                        count=count.numpy(), hwk=np.array([H, W, K]), blur=np.float32(blur), persp=np.bool_(persp),
                        views=O.views_tensor(R, T, intr).numpy(), mesh=np.array(mesh),
                        pix_to_face=p2f.numpy(), zbuf=zbuf.numpy(), bary=bary.numpy(), dists=dists.numpy())
    print(name, "covered", int((p2f[..., 0] >= 0).sum()))
