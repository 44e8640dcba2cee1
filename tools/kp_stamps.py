"""Per-tile timing of the fused soft silhouette raster (experiment build -DMR_XP_STAMP: each tile's wave
writes its start / end wall clock (100 MHz), pass and drain counts into the R channel of its first four
pixels). Run: MI355R_LIB=exp/stamp.so python tools/kp_stamps.py"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torch_renderer_amd.assets import load_asset  # noqa: E402
from torch_renderer_amd.cameras import PerspectiveCameras  # noqa: E402
from torch_renderer_amd.mesh_renderer import (BlendParams, MeshRasterizer, MeshRenderer,  # noqa: E402
                                              RasterizationSettings, SoftSilhouetteShader)
from torch_renderer_amd.structures import Meshes  # noqa: E402
from torch_renderer_amd.transforms import look_at_view_transform  # noqa: E402

dev = torch.device("cuda:0")
H = W = 128
nv = 64
m = load_asset("cow", device=dev, textures=False)
v0 = m.shared_verts().detach()
c = v0.mean(0)
verts = ((v0 - c) / (v0 - c).abs().max()).contiguous()
faces = m.shared_faces()
R, T = look_at_view_transform(dist=2.7, elev=torch.linspace(0, 360, nv), azim=torch.linspace(-180, 180, nv))
R, T = R.to(dev).contiguous(), T.to(dev).contiguous()
cams = PerspectiveCameras(device=dev, R=R, T=T)
rs = RasterizationSettings(image_size=H, blur_radius=math.log(1.0 / 1e-4 - 1.0) * 1e-4, faces_per_pixel=50,
                           perspective_correct=False)
renderer = MeshRenderer(rasterizer=MeshRasterizer(cameras=cams, raster_settings=rs),
                        shader=SoftSilhouetteShader(blend_params=BlendParams(sigma=1e-4)))
with torch.no_grad():
    for _ in range(3):
        img = renderer(Meshes([verts], [faces]).extend(nv), cameras=cams, R=R, T=T)
    torch.cuda.synchronize()
    img = renderer(Meshes([verts], [faces]).extend(nv), cameras=cams, R=R, T=T)
    torch.cuda.synchronize()
cov = img[..., 3] > 0
r = img[..., 0].contiguous().view(torch.int32).cpu()
covt = cov.view(nv, H // 8, 8, W // 8, 8).any(4).any(2).cpu()
rows = []
for n, ty, tx in covt.nonzero().tolist():
    y0, x0 = ty * 8, tx * 8
    v = r[n, y0, x0:x0 + 4].tolist()
    rows.append((n, ty, tx, v[0] & 0xffffffff, v[1] & 0xffffffff, v[2], v[3]))
t0 = min(x[3] for x in rows)
d = sorted(((x[4] - x[3]) & 0xffffffff) / 100.0 for x in rows)  # us
print(f"tiles {len(rows)}  span {(max(x[4] for x in rows) - t0) / 100.0:.1f} us")
q = lambda a, f: a[min(len(a) - 1, int(f * len(a)))]
print(f"tile us: mean {sum(d) / len(d):.1f} p50 {q(d, .5):.1f} p90 {q(d, .9):.1f} p99 {q(d, .99):.1f} max {d[-1]:.1f}")
st = sorted((x[3] - t0) / 100.0 for x in rows)
print(f"start us: p50 {q(st, .5):.1f} p90 {q(st, .9):.1f} max {st[-1]:.1f}")
top = sorted(rows, key=lambda x: -((x[4] - x[3]) & 0xffffffff))[:12]
for x in top:
    print(f"  view {x[0]:2d} tile ({x[1]:2d},{x[2]:2d}) start {(x[3] - t0) / 100.0:7.1f} us  dur {((x[4] - x[3]) & 0xffffffff) / 100.0:7.1f} us  passes {x[5]}  drains {x[6]}")
sp = sorted(x[5] for x in rows)
dr = sorted(x[6] for x in rows)
print(f"passes mean {sum(sp) / len(sp):.1f} max {sp[-1]}  drains mean {sum(dr) / len(dr):.1f} max {dr[-1]}")
tot = sum(d)
print(f"sum of tile us {tot:.0f}  -> / 1024 SIMDs {tot / 1024:.1f} us, / 2048 wave slots {tot / 2048:.1f} us")
