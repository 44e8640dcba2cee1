#!/usr/bin/env python3
"""How much does the projection's floating-point ORDER matter?

The build projects a vertex as ax * (X_view / Z_view) + bx (one affine per axis). Upstream
PyTorch3D composes 4x4 Transform3d matrices and divides the homogeneous product by w
(oracle.project_faces_upstream: v0.5/0.6 order "v06" and v0.7+ order "v07"). The two differ by
ulps in the NDC vertices; this tool rasterizes the same views with every variant on the C oracle
and counts the pixels whose pix_to_face differs, on the metric workload (cow, 512x512, 64 views,
PerspectiveCameras(in_ndc=False)) and on C3 (cow, 512x512, FoVPerspectiveCameras, near-plane clip).

    python tools/projection_flips.py [--views 64] [--threads 8] [--out profiles/r3_projection_flips.json]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from tests.helpers import mesh_arrays  # noqa: E402


def ulp_diff(a, b):
    ai = a.contiguous().view(torch.int32).long()
    bi = b.contiguous().view(torch.int32).long()
    ai = torch.where(ai < 0, -(ai & 0x7fffffff), ai)
    bi = torch.where(bi < 0, -(bi & 0x7fffffff), bi)
    return (ai - bi).abs()


def raster(fv, N, F, H, W, z_clip=None):
    first = torch.arange(N, dtype=torch.int64) * F
    count = torch.full((N,), F, dtype=torch.int64)
    if z_clip is None:
        return O.raster_fwd(fv, first, count, H, W)
    cf = O.clip_faces_ref(fv, first, count, z_clip, True)
    p2f, zbuf, bary, dists = O.raster_fwd(cf["face_verts"], cf["first"], cf["count"], H, W, neighbor=cf["neighbor"])
    p2f, bary = O.unclip_fragments(p2f, bary, cf)
    return p2f, zbuf, bary, dists


def compare(tag, fvs, N, F, H, W, z_clip=None):
    res = {}
    t0 = time.time()
    frags = {k: raster(v, N, F, H, W, z_clip) for k, v in fvs.items()}
    base = frags["build"]
    covered = int((base[0] >= 0).sum())
    for k in fvs:
        if k == "build":
            continue
        u = ulp_diff(fvs[k][..., :2], fvs["build"][..., :2])
        p2f_diff = int((frags[k][0] != base[0]).sum())
        same = (frags[k][0] == base[0]) & (base[0] >= 0)
        dz = (frags[k][1] - base[1])[same].abs().max().item() if bool(same.any()) else 0.0
        db = (frags[k][2] - base[2])[same].abs().max().item() if bool(same.any()) else 0.0
        dxy = (fvs[k][..., :2] - fvs["build"][..., :2]).abs()
        res[k] = {"ndc_xy_verts_differing": int((u > 0).sum()), "ndc_xy_max_abs_diff": dxy.max().item(),
                  "ndc_xy_max_ulp_away_from_zero": int(u[fvs["build"][..., :2].abs() > 1e-3].max()),
                  "ndc_xy_total": int(u.numel()), "p2f_flips": p2f_diff, "covered_pixels": covered,
                  "pixels": N * H * W, "flip_fraction_of_covered": p2f_diff / max(covered, 1),
                  "max_abs_zbuf_diff_same_face": dz, "max_abs_bary_diff_same_face": db}
        print(f"[{tag}] build vs {k}: {res[k]}", flush=True)
    if "upstream_v06" in frags and "upstream_v07" in frags:  # the two upstream versions against each other
        a, b = frags["upstream_v06"][0], frags["upstream_v07"][0]
        res["v06_vs_v07_p2f_flips"] = int((a != b).sum())
        print(f"[{tag}] upstream_v06 vs upstream_v07: {res['v06_vs_v07_p2f_flips']} p2f flips", flush=True)
    print(f"[{tag}] {time.time() - t0:.1f} s", flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=64)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r3_projection_flips.json"))
    args = ap.parse_args()
    O.set_threads(args.threads)
    torch.set_num_threads(args.threads)
    from bench import canonical_views
    from torch_renderer_amd.cameras import PerspectiveCameras
    from torch_renderer_amd.transforms import (look_at_view_transform, matrix_to_quaternion, opencv_to_pytorch3d,
                                               quaternion_to_matrix)

    verts, faces, _ = mesh_arrays("cow")
    F = faces.shape[0]
    H = W = 512
    out = {}
    # ---- metric workload: PerspectiveCameras(in_ndc=False), fx = fy for 60 deg at 512, centred pp
    N = args.views
    R_cv, t_cv, K = canonical_views(verts, N, H, W, dist_m=0.5)
    R, T = opencv_to_pytorch3d(R_cv.float(), t_cv.float())
    R, T = R.contiguous(), T.contiguous()
    cams = PerspectiveCameras(focal_length=((float(K[0, 0]), float(K[1, 1])),),
                              principal_point=((float(K[0, 2]), float(K[1, 2])),), in_ndc=False,
                              image_size=torch.tensor([[H, W]]))
    intr = cams.ndc_affine((H, W)).expand(N, 4).contiguous()
    cam = {"kind": "perspective", "fx": float(K[0, 0]), "fy": float(K[1, 1]), "px": float(K[0, 2]),
           "py": float(K[1, 2]), "in_ndc": False, "image_size": (H, W)}
    fvs = {"build": O.project_faces_torch(verts, faces, R, T, intr),
           "upstream_v06": O.project_faces_upstream(verts, faces, R, T, cam, "v06"),
           "upstream_v07": O.project_faces_upstream(verts, faces, R, T, cam, "v07")}
    out["metric"] = {"config": f"cow F={F}, {H}x{W}, {N} views, PerspectiveCameras(in_ndc=False)",
                     **compare("metric", fvs, N, F, H, W)}
    # ---- C3: FoVPerspectiveCameras(fov 60, znear 1, zfar 100), look_at_view_transform(0.7, 30, 60) + noise
    R0, T0 = look_at_view_transform(0.7, 30.0, 60.0)
    q = torch.cat((T0, matrix_to_quaternion(R0)), -1)
    q = q + torch.randn(1, 7, generator=torch.Generator().manual_seed(0)) * 0.03
    Rc = quaternion_to_matrix(q[:, 3:]).detach()
    Tc = q[:, :3].detach().contiguous()
    t = 1.0 / math.tan(math.radians(30.0))
    intr_c = torch.tensor([[t, 0.0, t, 0.0]])
    camc = {"kind": "fov", "znear": 1.0, "zfar": 100.0, "fov": 60.0, "aspect_ratio": 1.0, "degrees": True}
    fvc = {"build": O.project_faces_torch(verts, faces, Rc, Tc, intr_c),
           "upstream_v06": O.project_faces_upstream(verts, faces, Rc, Tc, camc, "v06"),
           "upstream_v07": O.project_faces_upstream(verts, faces, Rc, Tc, camc, "v07")}
    out["C3"] = {"config": f"cow F={F}, {H}x{W}, 1 view, FoVPerspectiveCameras, z_clip=0.5",
                 **compare("C3", fvc, 1, F, H, W, z_clip=0.5)}
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
