"""The HIP soft shader over stored fragments (mr_shade_fragments_forward / _backward: SoftPhongShader
and SoftSilhouetteShader for any faces_per_pixel) fed the oracle's OWN
fragments, so the shading is isolated from rasterization: images within 1e-4 of the oracle's
torch restatement of phong_shading + softmax_rgb_blend / sigmoid_alpha_blend, and gradients
w.r.t. zbuf, barycentrics, dists, vertex positions (interpolated points and normals), vertex
colours and the texture map within the bars of tests/helpers.report. Fragments: K-deep with
deform_mesh_with_color.py's blur = ln(1/1e-4 - 1) * 1e-4 and barycentric clipping."""
import math

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests.helpers import canonical_views, mesh_arrays, oracle_runs, report
from torch_renderer_amd import Meshes, TexturesUV, TexturesVertex
from torch_renderer_amd.cameras import PerspectiveCameras
from torch_renderer_amd.mesh_renderer import (BlendParams, Fragments, HardPhongShader, Materials, PointLights,
                                              SoftPhongShader, SoftSilhouetteShader)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
BLUR = math.log(1.0 / 1e-4 - 1.0) * 1e-4


def _leaf(t):
    return t.detach().clone().requires_grad_(True)


@pytest.mark.parametrize("K", [1, 3, 8, 50])
@pytest.mark.parametrize("texture", ["vertex", "uv"])
@pytest.mark.parametrize("shader", ["phong", "silhouette", "hard"])
def test_hip_shader_on_oracle_fragments(K, texture, shader):
    H, W, N = 40, 48, 2
    name = "teapot" if texture == "vertex" else "cow"
    verts, faces, d = mesh_arrays(name)
    R, T, intr, _ = canonical_views(verts, N, H, W)
    ref = O.render_ref(verts, faces, R, T, intr, H, W, K=K, blur=BLUR, clip=True)
    assert (ref["p2f"][..., min(K, 3) - 1] >= 0).any()
    p2f = ref["p2f"]
    g = torch.Generator().manual_seed(K)
    light = {"kind": "point", "location": (0.3, 0.8, -2.5), "ambient": (0.5, 0.4, 0.3), "diffuse": (0.3, 0.4, 0.5),
             "specular": (0.2, 0.25, 0.3)}
    mat = {"ambient": (1.0, 0.9, 0.8), "diffuse": (1.0, 1.0, 0.7), "specular": (0.6, 1.0, 1.0), "shininess": 32.0}
    cc = torch.tensor([[0.1, -0.2, 0.3]])
    bg = (0.1, 0.2, 0.3)
    vcol0 = torch.rand(verts.shape, generator=g) if texture == "vertex" else None
    if texture == "uv":
        img = torch.from_numpy(d["texture_u8"].astype(np.float32) / 255.0)
        map0 = img * 0.9 + 0.05
        vuv = torch.from_numpy(d["verts_uvs"]).float()
        fuv = torch.from_numpy(d["faces_uvs"]).long()
    local = p2f.clone()
    local[p2f >= 0] = p2f[p2f >= 0] % faces.shape[0]

    def oracle(dt):  # oracle shading on leaves; float64: its shadow (tests.helpers.report's conditioning)
        L = {k: _leaf(ref[k].to(dt)) for k in ("zbuf", "bary", "dists")}
        zbf, bry, dst = (O._jitter(L[k]) for k in ("zbuf", "bary", "dists"))  # probe (inside O.perturbed only)
        L["verts"] = _leaf(verts.to(dt))
        if texture == "vertex":
            L["tex"] = _leaf(vcol0.to(dt))
            texels = O.sample_textures_vertex(local, bry, L["tex"], faces)
        else:
            L["tex"] = _leaf(map0.to(dt))
            texels = O.sample_textures_uv(local, bry, vuv.to(dt), fuv, L["tex"])
        if shader == "phong":
            colors = O.phong_colors(local, bry, L["verts"], faces, texels, light, mat, cc.to(dt))
            o = O.softmax_rgb_blend(colors, p2f, zbf, dst, 1e-4, 1e-4, bg)
        elif shader == "hard":  # HardPhongShader: hard_rgb_blend of the same Phong colours
            colors = O.phong_colors(local, bry, L["verts"], faces, texels, light, mat, cc.to(dt))
            o = O.hard_rgb_blend(colors, p2f, bg)
        else:
            sil = O.sigmoid_alpha(p2f, dst, 1e-4)
            o = torch.cat([torch.ones(sil.shape + (3,), dtype=dt), sil[..., None]], -1)
        return O._jitter(o, False), L

    out_ref, Lr = oracle(torch.float32)
    go = torch.rand(out_ref.shape, generator=g) - 0.5
    (out_ref * go).sum().backward()
    zb, ba, di, vr = Lr["zbuf"], Lr["bary"], Lr["dists"], Lr["verts"]
    tex_gpu_src = Lr["tex"]
    if texture == "vertex":
        vcr = Lr["tex"]
    else:
        mr = Lr["tex"]
    keys = ("out", "zbuf", "bary", "dists", "verts", "tex")

    def flat(precision):
        o, L = oracle(torch.float32 if precision == "f32" else torch.float64)
        (o * go.to(o.dtype)).sum().backward()
        z = torch.zeros(1)
        return (o,) + tuple(L[k].grad if L[k].grad is not None else z for k in keys[1:])

    _, r64l, spl = oracle_runs(flat)
    out64 = r64l[0]

    def g64(k):
        return r64l[keys.index(k)] if Lr[k].grad is not None else None

    def spread(k):
        return spl[keys.index(k)] if Lr[k].grad is not None else None
    # HIP shader on the same fragments
    zg, bgp, dg = (_leaf(t.to(DEV)) for t in (ref["zbuf"], ref["bary"], ref["dists"]))
    vg = _leaf(verts.to(DEV))
    if texture == "vertex":
        vcg = _leaf(tex_gpu_src.detach().to(DEV))
        tex = TexturesVertex([vcg])
    else:
        mg = _leaf(mr.detach().to(DEV))
        tex = TexturesUV(maps=[mg], faces_uvs=[fuv.to(DEV)], verts_uvs=[vuv.to(DEV)])
    meshes = Meshes([vg], [faces.to(DEV)], tex).extend(N)
    cams = PerspectiveCameras(device=DEV, R=torch.eye(3)[None], T=-cc @ torch.eye(3))
    blend = BlendParams(sigma=1e-4, gamma=1e-4, background_color=bg)
    frags = Fragments(p2f.to(DEV), zg, bgp, dg)
    if shader in ("phong", "hard"):
        lights = PointLights(location=[light["location"]], ambient_color=[light["ambient"]],
                             diffuse_color=[light["diffuse"]], specular_color=[light["specular"]])
        mats = Materials(ambient_color=[mat["ambient"]], diffuse_color=[mat["diffuse"]],
                         specular_color=[mat["specular"]], shininess=mat["shininess"])
        cls = SoftPhongShader if shader == "phong" else HardPhongShader
        out = cls(device=DEV, cameras=cams, lights=lights, materials=mats, blend_params=blend)(frags, meshes)
    else:
        out = SoftSilhouetteShader(blend_params=blend)(frags, meshes, cameras=cams)
    tag = f"K={K} {texture} {shader}"
    report(f"{tag} rgba", out, out_ref, ref64=out64, sens=spl[0])
    (out * go.to(DEV)).sum().backward()
    if shader == "hard":  # no depth / distance dependence
        assert zg.grad is None and dg.grad is None  # no depth / distance dependence: no gradient tensors
        assert zb.grad is None or not zb.grad.any()
    else:
        report(f"{tag} grad dists", dg.grad, di.grad, ref64=g64("dists"), sens=spread("dists"))
    if shader == "silhouette":  # the silhouette blend reads only the distances
        assert zg.grad is None and bgp.grad is None
    if shader in ("phong", "hard"):
        if shader == "phong":
            report(f"{tag} grad zbuf", zg.grad, zb.grad, ref64=g64("zbuf"), sens=spread("zbuf"))
        report(f"{tag} grad bary", bgp.grad, ba.grad, ref64=g64("bary"), sens=spread("bary"))
        report(f"{tag} grad verts", vg.grad, vr.grad, ref64=g64("verts"), sens=spread("verts"))
        if texture == "vertex":
            report(f"{tag} grad vcolors", vcg.grad, vcr.grad, ref64=g64("tex"), sens=spread("tex"))
        else:
            report(f"{tag} grad map", mg.grad, mr.grad, ref64=g64("tex"), sens=spread("tex"))
    # the same fragments flagged sorted (MR_FRAG_SORTED, as this library's rasterizer marks its own):
    # the kernels stop at each pixel's first empty slot; outputs and fragment gradients are bitwise the
    # full-K ones, the mesh gradients (float atomics: summation order varies run to run) within 1e-6
    leaves = [zg, bgp, dg, vg] + ([vcg] if texture == "vertex" else [mg])
    first = [x.grad.clone() if x.grad is not None else None for x in leaves]
    for x in leaves:
        x.grad = None
    frags_s = Fragments(p2f.to(DEV), zg, bgp, dg, sorted_slots=True)
    if shader in ("phong", "hard"):
        out_s = cls(device=DEV, cameras=cams, lights=lights, materials=mats, blend_params=blend)(frags_s, meshes)
    else:
        out_s = SoftSilhouetteShader(blend_params=blend)(frags_s, meshes, cameras=cams)
    assert torch.equal(out_s, out)
    (out_s * go.to(DEV)).sum().backward()
    for i, (a, b) in enumerate(zip(leaves, first)):
        assert (a.grad is None) == (b is None)
        if b is None:
            continue
        if i < 3:
            assert torch.equal(a.grad, b)
        else:
            report(f"{tag} sorted vs full-K mesh grad {i}", a.grad, b, tol=1e-6)
