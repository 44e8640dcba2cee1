"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

CPU restatement of the reference's render path:
  * rasterizer: C restatement of PyTorch3D ``RasterizeMeshesNaiveCpu`` /
    ``RasterizeMeshesBackwardCpu`` (oracle/raster_cpu.c, built by oracle/Makefile);
  * everything around it — MeshRasterizer.transform, Meshes.verts_normals_packed,
    interpolate_face_attributes (python fallback), TexturesUV/TexturesVertex
    sampling, PointLights/AmbientLights/Materials, phong_shading,
    softmax_rgb_blend, sigmoid_alpha_blend — restated with plain torch CPU ops,
    following the upstream PyTorch3D Python (the reference's call sites:
    torch_renderer.py:61-159, renderer.py:47-101, camera_pose_optimizer.py:105-158,
    mesh_deformer.py:113-145). Autograd of these torch ops + the C backward gives
    the reference gradients.

PyTorch3D itself is absent from this container, so this oracle is
pinned by analytic known-answer tests and a float64 NumPy spec (oracle/spec_np.py),
not by reference-produced vectors. Nothing here is imported by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import torch
import torch.nn.functional as F

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None


def build_oracle(force: bool = False) -> str:
    src = os.path.join(_HERE, "raster_cpu.c")
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        build_oracle()
        L = ctypes.CDLL(_LIB)
        vp, i32, i64, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
        L.orc_raster_fwd.argtypes = [vp, vp, vp, i32, i32, i32, i32, f32, i32, i32, i32, vp, vp, vp, vp]
        L.orc_raster_fwd.restype = None
        L.orc_raster_fwd_ex.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, f32, i32, i32, i32, i32, i32, i32, i32,
                                        vp, vp, vp, vp]
        L.orc_raster_fwd_ex.restype = None
        L.orc_raster_fwd_pairs.argtypes = [vp, vp, vp, vp, i32, i32, i32, i32, f32, i32, i32, i32, vp, vp, vp, vp]
        L.orc_raster_fwd_pairs.restype = None
        L.orc_raster_bwd.argtypes = [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp]
        L.orc_raster_bwd.restype = None
        L.orc_set_threads.argtypes = [i32]
        L.orc_set_threads.restype = None
        L.orc_project_faces.argtypes = [vp, vp, i64, vp, i32, vp]
        L.orc_project_faces.restype = None
        _lib = L
    return _lib


def set_threads(n: int) -> None:
    """Threads of the C rasterizer (OpenMP) — the CPU baseline's core count."""
    lib().orc_set_threads(int(n))


def _p(t):
    assert t.is_contiguous() and t.device.type == "cpu"
    return ctypes.c_void_p(t.data_ptr())


# ---------------------------------------------------------------- rasterizer
def raster_fwd(face_verts, first, count, H, W, K=1, blur=0.0, persp=True, clip=False, cull=False, neighbor=None,
               window=None, pair_mode=0):
    """window = (y0, y1, x0, x1): rasterize only those pixels (others stay background).
    pair_mode = 1: split faces resolved as one candidate per pair (the MI355X rule; see
    orc_raster_fwd_pairs) instead of the CPU's order-dependent neighbour rule."""
    fv = face_verts.detach().float().contiguous().cpu()
    first = first.to(torch.int64).contiguous().cpu()
    count = count.to(torch.int64).contiguous().cpu()
    N = first.numel()
    p2f = torch.empty((N, H, W, K), dtype=torch.int64)
    zbuf = torch.empty((N, H, W, K))
    bary = torch.empty((N, H, W, K, 3))
    dists = torch.empty((N, H, W, K))
    nb = None if neighbor is None else neighbor.to(torch.int64).contiguous().cpu()
    if pair_mode:
        assert window is None
        lib().orc_raster_fwd_pairs(_p(fv), _p(first), _p(count), None if nb is None else _p(nb), N, H, W, K,
                                   float(blur), int(persp), int(clip), int(cull), _p(p2f), _p(zbuf), _p(bary),
                                   _p(dists))
        return p2f, zbuf, bary, dists
    wy0, wy1, wx0, wx1 = window if window is not None else (0, 0, 0, 0)
    lib().orc_raster_fwd_ex(_p(fv), _p(first), _p(count), None if nb is None else _p(nb), N, H, W, K, float(blur),
                            int(persp), int(clip), int(cull), wy0, wy1, wx0, wx1, _p(p2f), _p(zbuf), _p(bary),
                            _p(dists))
    return p2f, zbuf, bary, dists


def raster_bwd(face_verts, p2f, gz, gb, gd, persp=True, clip=False):
    fv = face_verts.detach().float().contiguous().cpu()
    N, H, W, K = p2f.shape
    g = torch.zeros_like(fv)
    lib().orc_raster_bwd(_p(fv), _p(p2f.contiguous()), _p(gz.float().contiguous()), _p(gb.float().contiguous()),
                         _p(gd.float().contiguous()), N, H, W, K, int(persp), int(clip), _p(g))
    return g


class RasterizeRef(torch.autograd.Function):
    """_RasterizeFaceVerts restated on the C oracle."""

    @staticmethod
    def forward(ctx, face_verts, first, count, H, W, K, blur, persp, clip, cull, neighbor=None, window=None,
                pair_mode=0):
        p2f, zbuf, bary, dists = raster_fwd(face_verts, first, count, H, W, K, blur, persp, clip, cull, neighbor,
                                            window, pair_mode)
        ctx.save_for_backward(face_verts, p2f)
        ctx.persp, ctx.clip = persp, clip
        ctx.mark_non_differentiable(p2f)
        return p2f, zbuf, bary, dists

    @staticmethod
    def backward(ctx, _gp, gz, gb, gd):
        fv, p2f = ctx.saved_tensors
        g = raster_bwd(fv, p2f, gz, gb, gd, ctx.persp, ctx.clip)
        return g, None, None, None, None, None, None, None, None, None, None, None, None


def project_faces_c(verts, faces, views):
    """Bit-exact restatement of the MI355X projection (orc_project_faces)."""
    v = verts.detach().float().contiguous().cpu()
    f = faces.to(torch.int32).contiguous().cpu()
    vw = views.detach().float().contiguous().cpu()
    N = vw.shape[0]
    out = torch.empty((N * f.shape[0], 3, 3))
    lib().orc_project_faces(_p(v), _p(f), f.shape[0], _p(vw), N, _p(out))
    return out


def project_faces_torch(verts, faces, R, T, intr):
    """Same projection with torch elementwise ops (autograd). intr: (N,4) ax, bx, ay, by.
    Operand order identical to orc_project_faces, so values are bitwise equal."""
    X = verts[faces.long()]  # (F,3,3)
    Xb = X[None]
    Rb = R[:, None, None]
    Tb = T[:, None, None]
    vx = ((Xb[..., 0] * Rb[..., 0, 0] + Xb[..., 1] * Rb[..., 1, 0]) + Xb[..., 2] * Rb[..., 2, 0]) + Tb[..., 0]
    vy = ((Xb[..., 0] * Rb[..., 0, 1] + Xb[..., 1] * Rb[..., 1, 1]) + Xb[..., 2] * Rb[..., 2, 1]) + Tb[..., 1]
    vz = ((Xb[..., 0] * Rb[..., 0, 2] + Xb[..., 1] * Rb[..., 1, 2]) + Xb[..., 2] * Rb[..., 2, 2]) + Tb[..., 2]
    ax, bx, ay, by = (intr[:, i][:, None, None] for i in range(4))
    nx = ax * (vx / vz) + bx
    ny = ay * (vy / vz) + by
    fv = torch.stack([nx, ny, vz], dim=-1)  # (N,F,3,3)
    return fv.reshape(-1, 3, 3)


# ---------------------------------------------------------------- near-plane clipping
def _clip_point(a, b, w, c, persp):
    """Point on edge a->b (rows (x_ndc, y_ndc, z_view)) at view z = c, w = (c - za) / (zb - za).
    Perspective: interpolate the view-linear ndc*z and divide by c (upstream clip.py
    _find_verts_intersecting_clipping_plane); otherwise interpolate ndc linearly. z = c."""
    if persp:
        axw, ayw = a[:, 0] * a[:, 2], a[:, 1] * a[:, 2]
        bxw, byw = b[:, 0] * b[:, 2], b[:, 1] * b[:, 2]
        x = (axw + w * (bxw - axw)) / c
        y = (ayw + w * (byw - ayw)) / c
    else:
        x = a[:, 0] + w * (b[:, 0] - a[:, 0])
        y = a[:, 1] + w * (b[:, 1] - a[:, 1])
    return torch.stack([x, y, torch.full_like(x, c)], dim=1)


def clip_faces_ref(face_verts, first, count, z_clip, persp=True):
    """upstream mesh/clip.py clip_faces restated (z plane only; cull_to_frustum off).

    Per face (corners ordered i, j = i+1, k = i+2 mod 3) with b = #corners at view z < z_clip:
      b = 0 -> unchanged; b = 3 -> culled;
      b = 2 (front corner i) -> one triangle: slot i = p_i, slot j = p_ij, slot k = p_ik;
      b = 1 (behind corner i) -> the quadrilateral p_ij, p_j, p_k, p_ik split into
        t1 = (slot i = p_ij, j = p_j, k = p_k) and t2 = (slot i = p_ik, j = p_ij, k = p_k),
        consecutive packed ids, each the other's clipped_faces_neighbor_idx;
    p_ij is the point on edge i->j at z_clip. Sub-triangles keep the original orientation and
    take the original's place in the packed order (culled faces drop out). conversion[t] (3,3):
    row s = original-face barycentrics of the sub-triangle's slot-s vertex, so the original
    barycentrics of a fragment are sum_s b_sub[s] * conversion[t][s].

    Returns dict(face_verts (Fc,3,3), first (N), count (N), neighbor (Fc) i64, orig (Fc) i64,
    conversion (Fc,3,3)). Differentiable w.r.t. face_verts (autograd through the torch ops)."""
    fv = face_verts
    F = fv.shape[0]
    c = float(z_clip)
    z = fv[:, :, 2]
    behind = z < c
    nb = behind.sum(1)
    eye = torch.eye(3, dtype=fv.dtype)
    ar = torch.arange(F)
    # corner i per face: the single front corner (b = 2) or the single behind corner (b = 1)
    i_front = torch.argmax((~behind).to(torch.int64), dim=1)
    i_back = torch.argmax(behind.to(torch.int64), dim=1)
    i = torch.where(nb == 2, i_front, i_back)
    j, k = (i + 1) % 3, (i + 2) % 3
    pi, pj, pk = fv[ar, i], fv[ar, j], fv[ar, k]
    zi, zj, zk = pi[:, 2], pj[:, 2], pk[:, 2]
    # only clipped faces use wj / wk; elsewhere the denominators may be 0 (and a masked NaN would
    # still poison autograd), so they divide by 1 there
    clipped = (nb == 1) | (nb == 2)
    one = torch.ones_like(zi)
    wj = (c - zi) / torch.where(clipped, zj - zi, one)
    wk = (c - zi) / torch.where(clipped, zk - zi, one)
    wj = torch.where(clipped, wj, torch.zeros_like(wj))
    wk = torch.where(clipped, wk, torch.zeros_like(wk))
    pij = _clip_point(pi, pj, wj, c, persp)
    pik = _clip_point(pi, pk, wk, c, persp)
    ei, ej, ek = eye[i], eye[j], eye[k]
    cij = (1.0 - wj)[:, None] * ei + wj[:, None] * ej
    cik = (1.0 - wk)[:, None] * ei + wk[:, None] * ek

    def slots(a, b_, c_):  # rows placed at slots (i, j, k)
        out = torch.zeros(F, 3, a.shape[1], dtype=fv.dtype)
        out = out.index_put((ar, i), a).index_put((ar, j), b_).index_put((ar, k), c_)
        return out

    t_case2 = slots(pi, pij, pik)
    c_case2 = slots(ei, cij, cik)
    t1 = slots(pij, pj, pk)
    c1 = slots(cij, ej, ek)
    t2 = slots(pik, pij, pk)
    c2 = slots(cik, cij, ek)
    eye3 = eye.expand(F, 3, 3)
    first_t = torch.where((nb == 2)[:, None, None], t_case2, torch.where((nb == 1)[:, None, None], t1, fv))
    first_c = torch.where((nb == 2)[:, None, None], c_case2, torch.where((nb == 1)[:, None, None], c1, eye3))
    keep = nb < 3
    quad = nb == 1
    verts_out, conv_out, orig, nbr = [], [], [], []
    n_out = torch.zeros(len(first), dtype=torch.int64)
    mesh = torch.zeros(F, dtype=torch.int64)
    for m in range(len(first)):
        mesh[int(first[m]):int(first[m]) + int(count[m])] = m
    pos = 0
    idx_first, idx_second = [], []
    for f in range(F):
        if not bool(keep[f]):
            continue
        idx_first.append((f, pos))
        orig.append(f)
        nbr.append(pos + 1 if bool(quad[f]) else -1)
        n_out[mesh[f]] += 1
        pos += 1
        if bool(quad[f]):
            idx_second.append((f, pos))
            orig.append(f)
            nbr.append(pos - 1)
            n_out[mesh[f]] += 1
            pos += 1
    Fc = pos
    order = torch.empty(Fc, dtype=torch.int64)
    which = torch.zeros(Fc, dtype=torch.bool)
    for f, p_ in idx_first:
        order[p_] = f
    for f, p_ in idx_second:
        order[p_] = f
        which[p_] = True
    verts = torch.where(which[:, None, None], t2[order], first_t[order])
    conv = torch.where(which[:, None, None], c2[order], first_c[order])
    cnt = n_out
    fst = torch.cumsum(cnt, 0) - cnt
    return {"face_verts": verts, "first": fst, "count": cnt, "neighbor": torch.tensor(nbr, dtype=torch.int64),
            "orig": torch.tensor(orig, dtype=torch.int64), "conversion": conv}


def unclip_fragments(p2f, bary, clip):
    """convert_clipped_rasterization_to_original_faces: packed ids of the original faces and the
    original-face barycentrics sum_s b_sub[s] * conversion[s] (explicit (s0 + s1) + s2 order)."""
    valid = p2f >= 0
    idx = p2f.clamp(min=0)
    conv = clip["conversion"][idx]  # (..., 3, 3)
    b = bary
    ob = (b[..., 0:1] * conv[..., 0, :] + b[..., 1:2] * conv[..., 1, :]) + b[..., 2:3] * conv[..., 2, :]
    ob = torch.where(valid[..., None], ob, bary)
    op2f = torch.where(valid, clip["orig"][idx], p2f)
    return op2f, ob


# ---------------------------------------------------------------- mesh / shading restatement
def vertex_normals(verts, faces):
    """Meshes._compute_vertex_normals (upstream structures/meshes.py)."""
    faces = faces.long()
    vf = verts[faces]
    fn = torch.cross(vf[:, 2] - vf[:, 1], vf[:, 0] - vf[:, 1], dim=1)
    vn = torch.zeros_like(verts)
    vn = vn.index_add(0, faces[:, 0], fn)
    vn = vn.index_add(0, faces[:, 1], fn)
    vn = vn.index_add(0, faces[:, 2], fn)
    return F.normalize(vn, eps=1e-6, dim=1)


def interpolate_face_attributes(pix_to_face, bary, face_attrs):
    """interpolate_face_attributes_python (upstream ops/interp_face_attrs.py)."""
    Fn, FV, D = face_attrs.shape
    N, H, W, K, _ = bary.shape
    mask = pix_to_face < 0
    p2f = pix_to_face.clone()
    p2f[mask] = 0
    idx = p2f.view(N * H * W * K, 1, 1).expand(N * H * W * K, 3, D)
    vals = face_attrs.gather(0, idx).view(N, H, W, K, 3, D)
    out = (bary[..., None] * vals).sum(dim=-2)
    out = out.masked_fill(mask[..., None], 0.0)
    return out


def sample_textures_uv(p2f, bary, verts_uvs, faces_uvs_packed, tex_map):
    """TexturesUV.sample_textures (align_corners=True, padding 'border', bilinear).
    tex_map: (Ht, Wt, C) shared by all meshes of the batch."""
    N, H, W, K = p2f.shape
    fvu = verts_uvs[faces_uvs_packed.long()]  # (Ftot,3,2)
    uvs = interpolate_face_attributes(p2f, bary, fvu)  # (N,H,W,K,2)
    uvs = uvs.permute(0, 3, 1, 2, 4).reshape(N * K, H, W, 2)
    C = tex_map.shape[-1]
    maps = tex_map.permute(2, 0, 1)[None].expand(N * K, C, tex_map.shape[0], tex_map.shape[1])
    uvs = uvs * 2.0 - 1.0
    maps = torch.flip(maps, [2])
    texels = F.grid_sample(maps, uvs, mode="bilinear", align_corners=True, padding_mode="border")
    return texels.reshape(N, K, C, H, W).permute(0, 3, 4, 1, 2)


def sample_textures_vertex(p2f, bary, vcolors_packed, faces_packed):
    return interpolate_face_attributes(p2f, bary, vcolors_packed[faces_packed.long()])


def _normalize(x):
    return F.normalize(x, p=2, dim=-1, eps=1e-6)


def phong_colors(p2f, bary, verts, faces, texels, light, mat, cam_center):
    """phong_shading + _apply_lighting with PointLights / AmbientLights."""
    vn = vertex_normals(verts, faces)
    fverts = verts[faces.long()]
    fnorms = vn[faces.long()]
    coords = interpolate_face_attributes(p2f, bary, fverts)
    normals = interpolate_face_attributes(p2f, bary, fnorms)
    amb = torch.tensor(mat["ambient"]) * torch.tensor(light["ambient"])
    if light["kind"] == "ambient":
        return amb * texels
    loc = torch.tensor(light["location"], dtype=torch.float32)
    direction = loc - coords
    nh = _normalize(normals)
    lh = _normalize(direction)
    angle = F.relu(torch.sum(nh * lh, dim=-1))
    diffuse = torch.tensor(mat["diffuse"]) * (torch.tensor(light["diffuse"]) * angle[..., None])
    # specular (PointLights.specular)
    nh2 = _normalize(normals)
    lh2 = _normalize(direction)
    cos_angle = torch.sum(nh2 * lh2, dim=-1)
    mask = (cos_angle > 0).to(torch.float32)
    cc = cam_center.view(-1, 1, 1, 1, 3)
    view_direction = _normalize(cc - coords)
    reflect = -lh2 + 2 * (cos_angle[..., None] * nh2)
    alpha = F.relu(torch.sum(view_direction * reflect, dim=-1)) * mask
    specular = torch.tensor(mat["specular"]) * (torch.tensor(light["specular"]) *
                                                torch.pow(alpha, mat["shininess"])[..., None])
    return (amb + diffuse) * texels + specular


def softmax_rgb_blend(colors, p2f, zbuf, dists, sigma, gamma, bg, znear=1.0, zfar=100.0):
    eps = 1e-10
    mask = p2f >= 0
    prob_map = torch.sigmoid(-dists / sigma) * mask
    alpha = torch.prod((1.0 - prob_map), dim=-1)
    z_inv = (zfar - zbuf) / (zfar - znear) * mask
    z_inv_max = torch.max(z_inv, dim=-1).values[..., None].clamp(min=eps)
    weights_num = prob_map * torch.exp((z_inv - z_inv_max) / gamma)
    delta = torch.exp((eps - z_inv_max) / gamma).clamp(min=eps)
    denom = weights_num.sum(dim=-1)[..., None] + delta
    weighted_colors = (weights_num[..., None] * colors).sum(dim=-2)
    background = torch.tensor(bg, dtype=torch.float32)
    rgb = (weighted_colors + delta * background) / denom
    return torch.cat([rgb, (1.0 - alpha)[..., None]], dim=-1)


def hard_rgb_blend(colors, p2f, bg):
    """upstream blending.py hard_rgb_blend (PyTorch3D >= 0.5; HardPhongShader, myrenderer.py:88):
    the nearest fragment's colour where a face covers the pixel, the background elsewhere;
    alpha = ~is_background. Restated from the published source as recalled (no copy here to check
    against; parity unpinned beyond this restatement)."""
    is_bg = p2f[..., 0] < 0
    bgc = torch.as_tensor(bg, dtype=colors.dtype)
    rgb = torch.where(is_bg[..., None], bgc.expand(colors[..., 0, :].shape), colors[..., 0, :])
    alpha = (~is_bg).to(colors.dtype)[..., None]
    return torch.cat([rgb, alpha], dim=-1)


def sigmoid_alpha(p2f, dists, sigma):
    mask = p2f >= 0
    prob = torch.sigmoid(-dists / sigma) * mask
    alpha = torch.prod((1.0 - prob), dim=-1)
    return 1.0 - alpha


DEFAULT_LIGHT = {"kind": "point", "location": (0.0, 0.0, -3.0), "ambient": (0.5, 0.5, 0.5),
                 "diffuse": (0.3, 0.3, 0.3), "specular": (0.2, 0.2, 0.2)}
DEFAULT_MAT = {"ambient": (1.0, 1.0, 1.0), "diffuse": (1.0, 1.0, 1.0), "specular": (1.0, 1.0, 1.0),
               "shininess": 64.0}


def render_ref(verts, faces, R, T, intr, H, W, *, texture=None, light=DEFAULT_LIGHT, mat=DEFAULT_MAT,
               cam_center=(0.0, 0.0, 0.0), sigma=1e-4, gamma=1e-4, bg=(1.0, 1.0, 1.0), sigma_sil=1e-4,
               znear=1.0, zfar=100.0, persp=True, K=1, blur=0.0, clip=False, z_clip=None, window=None):
    """The reference CPU render path for one mesh shared by N views:
    depth = relu(zbuf[...,0]); sil = sigmoid_alpha_blend alpha; rgba = softmax_rgb_blend(phong).
    texture: None (white), ("vertex", vcolors (V,3)), ("uv", verts_uvs, faces_uvs, map (Ht,Wt,C)).
    Returns dict with depth, sil, rgba, fragments."""
    N = R.shape[0]
    Fn = faces.shape[0]
    fv = project_faces_torch(verts, faces, R, T, intr)
    first = torch.arange(N, dtype=torch.int64) * Fn
    count = torch.full((N,), Fn, dtype=torch.int64)
    if z_clip is None:
        p2f, zbuf, bary, dists = RasterizeRef.apply(fv, first, count, H, W, K, blur, persp, clip, False, None, window)
    else:  # MeshRasterizer with a znear camera: clip_faces -> raster -> convert back (upstream clip.py)
        cf = clip_faces_ref(fv, first, count, z_clip, persp)
        p2f_c, zbuf, bary_c, dists = RasterizeRef.apply(cf["face_verts"], cf["first"], cf["count"], H, W, K, blur,
                                                        persp, clip, False, cf["neighbor"], window)
        p2f, bary = unclip_fragments(p2f_c, bary_c, cf)
    faces_packed = faces.long().repeat(N, 1)
    verts_packed_faces = faces_packed  # faces index the shared verts
    local = p2f.clone()
    local[p2f >= 0] = p2f[p2f >= 0] % Fn
    if texture is None:
        texels = torch.ones(N, H, W, K, 3)
    elif texture[0] == "vertex":
        texels = sample_textures_vertex(local, bary, texture[1], faces)
    else:
        texels = sample_textures_uv(local, bary, texture[1], texture[2], texture[3])
    cc = torch.as_tensor(cam_center, dtype=torch.float32).view(-1, 3)
    colors = phong_colors(local, bary, verts, faces, texels, light, mat, cc)
    rgba = softmax_rgb_blend(colors, p2f, zbuf, dists, sigma, gamma, bg, znear, zfar)
    sil = sigmoid_alpha(p2f, dists, sigma_sil)
    depth = torch.relu(zbuf[..., 0])
    del verts_packed_faces
    return {"depth": depth, "sil": sil, "rgba": rgba, "p2f": p2f, "zbuf": zbuf, "bary": bary, "dists": dists,
            "face_verts": fv}


def views_tensor(R, T, intr):
    """(N,16) view records {R row-major, T, ax, bx, ay, by} as in include/mi355r.h."""
    return torch.cat([R.reshape(-1, 9), T.reshape(-1, 3), intr.reshape(-1, 4)], dim=1).float().contiguous()


__all__ = ["raster_fwd", "raster_bwd", "RasterizeRef", "project_faces_c", "project_faces_torch", "render_ref",
           "vertex_normals", "views_tensor", "np"]
