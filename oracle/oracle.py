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


# ---------------------------------------------------------------- upstream-order projection
# PyTorch3D's MeshRasterizer.transform does not compute ax * (x / z) + bx: it composes 4x4
# Transform3d matrices (row-vector convention) and applies one homogeneous product + divide:
#   v0.5/0.6 ("v06", cameras.transform_points_ndc):  [X, 1] @ (((R4 @ T4) @ K4) @ (FIX4 @ S2N4)) / w
#   v0.7+    ("v07", projection_transform.compose(to_ndc) on verts_view):  [Xv, 1] @ (K4 @ (FIX4 @ S2N4)) / w
# with R4 = Rotate(R), T4 = Translate(T) (get_world_to_view_transform), K4 = K^T of the camera's
# calibration matrix (_get_sfm_calibration_matrix / FoV compute_projection_matrix), FIX4 the
# principal-point fix and S2N4 = inverse(ndc -> screen) of get_ndc_camera_transform (in_ndc=False
# only; identity otherwise); then verts_ndc[..., 2] = verts_view[..., 2]. Restated from the published
# PyTorch3D sources as recalled (the package is absent here: parity unpinned); every 4x4 product is
# evaluated as torch's small-bmm CPU kernel does, sum over k = 0..3 in order, float32, no FMA. The
# float32 tan of the FoV camera and LAPACK's 4x4 inverse are taken as correctly rounded (exact for
# the power-of-two image sizes of every BASELINE config).
def _mm4(A, B):
    """(..., 4, 4) float32 matrix product, k summed in order 0..3, one rounding per operation."""
    A = np.asarray(A, np.float32)
    B = np.asarray(B, np.float32)
    shp = np.broadcast_shapes(A.shape, B.shape)
    C = np.zeros(shp, np.float32)
    for i in range(4):
        for j in range(4):
            acc = A[..., i, 0] * B[..., 0, j]
            for k in range(1, 4):
                acc = (acc + A[..., i, k] * B[..., k, j]).astype(np.float32)
            C[..., i, j] = acc
    return C


def _apply4(P, M):
    """[P, 1] @ M then divide by w (Transform3d.transform_points, eps=None). P (..., 3), M (..., 4, 4)."""
    P = np.asarray(P, np.float32)
    out = []
    for j in range(4):
        acc = P[..., 0] * M[..., 0, j]
        acc = (acc + P[..., 1] * M[..., 1, j]).astype(np.float32)
        acc = (acc + P[..., 2] * M[..., 2, j]).astype(np.float32)
        acc = (acc + np.float32(1.0) * M[..., 3, j]).astype(np.float32)
        out.append(acc)
    w = out[3]
    return np.stack([(out[0] / w).astype(np.float32), (out[1] / w).astype(np.float32),
                     (out[2] / w).astype(np.float32)], -1)


def upstream_camera_mats(cam, N):
    """(K4, NDC4) (N,4,4) float32 row-vector matrices of a camera spec:
    {"kind": "perspective", "fx", "fy", "px", "py", "in_ndc", "image_size": (H, W)} or
    {"kind": "fov", "znear", "zfar", "fov", "aspect_ratio", "degrees"}."""
    f32 = np.float32
    Kc = np.zeros((N, 4, 4), np.float32)  # column-vector K, transposed at the end
    ndc = np.tile(np.eye(4, dtype=np.float32), (N, 1, 1))
    if cam["kind"] == "fov":
        zn, zf = f32(cam.get("znear", 1.0)), f32(cam.get("zfar", 100.0))
        ar = f32(cam.get("aspect_ratio", 1.0))
        fov = f32(cam.get("fov", 60.0))
        if cam.get("degrees", True):
            fov = f32(f32(np.pi / 180) * fov)
        tanh = f32(np.tan(fov / f32(2.0)))
        max_y = f32(tanh * zn)
        min_y = f32(-max_y)
        max_x = f32(max_y * ar)
        min_x = f32(-max_x)
        Kc[:, 0, 0] = f32(f32(f32(2.0) * zn) / f32(max_x - min_x))
        Kc[:, 1, 1] = f32(f32(f32(2.0) * zn) / f32(max_y - min_y))
        Kc[:, 0, 2] = f32(f32(max_x + min_x) / f32(max_x - min_x))
        Kc[:, 1, 2] = f32(f32(max_y + min_y) / f32(max_y - min_y))
        Kc[:, 3, 2] = 1.0
        Kc[:, 2, 2] = f32(zf / f32(zf - zn))
        Kc[:, 2, 3] = f32(-f32(zf * zn) / f32(zf - zn))
    else:
        fx, fy = f32(cam["fx"]), f32(cam["fy"])
        px, py = f32(cam["px"]), f32(cam["py"])
        Kc[:, 0, 0], Kc[:, 1, 1], Kc[:, 0, 2], Kc[:, 1, 2] = fx, fy, px, py
        Kc[:, 3, 2] = 1.0
        Kc[:, 2, 3] = 1.0
        if not cam.get("in_ndc", True):
            H, W = cam["image_size"]
            s = f32(f32(min(H, W)) / f32(2.0))
            fix = np.tile(np.eye(4, dtype=np.float32), (N, 1, 1))
            fix[:, 3, 0] = f32(-2.0) * px  # pr_point_fix[:, :2, 3] = -2 * pp, transposed
            fix[:, 3, 1] = f32(-2.0) * py
            inv_s = f32(f32(1.0) / s)
            s2n = np.tile(np.eye(4, dtype=np.float32), (N, 1, 1))
            s2n[:, 0, 0] = inv_s
            s2n[:, 1, 1] = inv_s
            s2n[:, 3, 0] = f32(f32(f32(W) / f32(2.0)) * inv_s)  # inverse of the -W/2 translation
            s2n[:, 3, 1] = f32(f32(f32(H) / f32(2.0)) * inv_s)
            ndc = _mm4(fix, s2n)
    return np.ascontiguousarray(np.transpose(Kc, (0, 2, 1))), ndc


def project_faces_upstream(verts, faces, R, T, cam, version="v06"):
    """face_verts (N*F, 3, 3) as upstream MeshRasterizer.transform computes them (see above): NDC
    x, y from the composed homogeneous product and divide, view z kept. R (N,3,3) row-vector
    convention, T (N,3). Returns a float32 torch tensor (no autograd)."""
    v = verts.detach().float().cpu().numpy()
    f = faces.detach().long().cpu().numpy()
    Rn = R.detach().float().cpu().numpy().reshape(-1, 3, 3)
    Tn = T.detach().float().cpu().numpy().reshape(-1, 3)
    N = max(Rn.shape[0], Tn.shape[0])
    Rn = np.broadcast_to(Rn, (N, 3, 3))
    Tn = np.broadcast_to(Tn, (N, 3))
    R4 = np.tile(np.eye(4, dtype=np.float32), (N, 1, 1))
    R4[:, :3, :3] = Rn
    T4 = np.tile(np.eye(4, dtype=np.float32), (N, 1, 1))
    T4[:, 3, :3] = Tn
    K4, ndc = upstream_camera_mats(cam, N)
    W2V = _mm4(R4, T4)
    X = v[f]  # (F,3,3)
    view = _apply4(X[None], W2V[:, None, None])  # (N,F,3,3) verts_view
    if version == "v06":
        M = _mm4(_mm4(W2V, K4), ndc)
        out = _apply4(X[None], M[:, None, None])
    elif version == "v07":
        P = _mm4(K4, ndc)
        out = _apply4(view, P[:, None, None])
    else:
        raise ValueError(version)
    out[..., 2] = view[..., 2]
    return torch.from_numpy(np.ascontiguousarray(out.reshape(-1, 3, 3)))


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
               znear=1.0, zfar=100.0, persp=True, K=1, blur=0.0, clip=False, z_clip=None, window=None,
               precision="f32"):
    """The reference CPU render path for one mesh shared by N views:
    depth = relu(zbuf[...,0]); sil = sigmoid_alpha_blend alpha; rgba = softmax_rgb_blend(phong).
    texture: None (white), ("vertex", vcolors (V,3)), ("uv", verts_uvs, faces_uvs, map (Ht,Wt,C)).
    precision="f64": the float64 shadow (same decisions, every value and gradient in float64; see
    frag_eval_t), which measures the f32 oracle's own rounding error.
    Returns dict with depth, sil, rgba, fragments."""
    N = R.shape[0]
    Fn = faces.shape[0]
    if precision == "f64":
        p2f, zbuf, bary, dists, fv = _shadow_fragments(verts, faces, R, T, intr, H, W, K, blur, persp, clip, z_clip,
                                                       window)
        verts = verts.double()
        if texture is not None:
            texture = tuple(t.double() if torch.is_tensor(t) and t.is_floating_point() else t for t in texture)
        cam_center = torch.as_tensor(cam_center).double()
    else:
        fv = project_faces_torch(verts, faces, R, T, intr)
        first = torch.arange(N, dtype=torch.int64) * Fn
        count = torch.full((N,), Fn, dtype=torch.int64)
        if z_clip is None:
            p2f, zbuf, bary, dists = RasterizeRef.apply(fv, first, count, H, W, K, blur, persp, clip, False, None,
                                                        window)
        else:  # MeshRasterizer with a znear camera: clip_faces -> raster -> convert back (upstream clip.py)
            cf = clip_faces_ref(fv, first, count, z_clip, persp)
            p2f_c, zbuf, bary_c, dists = RasterizeRef.apply(cf["face_verts"], cf["first"], cf["count"], H, W, K,
                                                            blur, persp, clip, False, cf["neighbor"], window)
            p2f, bary = unclip_fragments(p2f_c, bary_c, cf)
        zbuf, bary, dists = _jitter(zbuf), _jitter(bary), _jitter(dists)  # conditioning probe (if active)
    local = p2f.clone()
    local[p2f >= 0] = p2f[p2f >= 0] % Fn
    if texture is None:
        texels = torch.ones(N, H, W, K, 3, dtype=zbuf.dtype)
    elif texture[0] == "vertex":
        texels = sample_textures_vertex(local, bary, texture[1], faces)
    else:
        texels = sample_textures_uv(local, bary, texture[1], texture[2], texture[3])
    cc = torch.as_tensor(cam_center, dtype=zbuf.dtype).view(-1, 3)
    colors = phong_colors(local, bary, verts, faces, texels, light, mat, cc)
    rgba = softmax_rgb_blend(colors, p2f, zbuf, dists, sigma, gamma, bg, znear, zfar)
    sil = sigmoid_alpha(p2f, dists, sigma_sil)
    depth = torch.relu(zbuf[..., 0])
    depth, sil, rgba = _jitter(depth, False), _jitter(sil, False), _jitter(rgba, False)
    return {"depth": depth, "sil": sil, "rgba": rgba, "p2f": p2f, "zbuf": zbuf, "bary": bary, "dists": dists,
            "face_verts": fv}


# ---------------------------------------------------------------- conditioning probe
# Under `with perturbed(seed):` render_ref (f32) scales the values of its fragments (zbuf, bary,
# dists) by 1 + eps_val * n and every gradient entering its fragments and its outputs (depth,
# silhouette, rgba) by 1 + eps_grad * n, n ~ N(0, 1) per entry (1e-7 ~ 1 ulp, 1e-6 ~ 8 ulp). How far
# a result moves under that is how far float32 rounding can move it: the per-entry conditioning that
# tests.helpers.report allows for (a gradient that is a difference of much larger per-pixel terms,
# a saturated sigmoid's 1 - p, a sliver face's 1 / area^2).
_PERTURB = None


class perturbed:
    def __init__(self, seed, eps_val=1e-7, eps_grad=1e-6):
        self.gen = torch.Generator().manual_seed(1000 + int(seed))
        self.eps_val, self.eps_grad = eps_val, eps_grad

    def __enter__(self):
        global _PERTURB
        _PERTURB = self
        return self

    def __exit__(self, *exc):
        global _PERTURB
        _PERTURB = None
        return False


class _Jitter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, nv, ng, eps_val, eps_grad):
        ctx.save_for_backward(ng)
        ctx.eps_grad = eps_grad
        return x * (1 + eps_val * nv)

    @staticmethod
    def backward(ctx, g):
        (ng,) = ctx.saved_tensors
        return g * (1 + ctx.eps_grad * ng), None, None, None, None


def _jitter(x, value=True):
    P = _PERTURB
    if P is None or not torch.is_tensor(x) or not x.is_floating_point():
        return x
    nv = torch.randn(x.shape, generator=P.gen, dtype=x.dtype) if value else torch.zeros_like(x)
    ng = torch.randn(x.shape, generator=P.gen, dtype=x.dtype)
    return _Jitter.apply(x, nv, ng, P.eps_val if value else 0.0, P.eps_grad)


# ---------------------------------------------------------------- float64 shadow
# The f32 oracle is itself only as accurate as float32 allows: a vertex gradient that is a
# difference of large per-pixel terms (the 1/sigma = 1e4 factor of the soft blends, 1/area^2 of
# slivers), or sigmoid(x)(1 - sigmoid(x)) near saturation, carries the oracle's own rounding error.
# The shadow evaluates the same formulas in float64 at the same decisions (the f32 run's
# pix_to_face and near-plane split structure), differentiable end to end by torch autograd:
# |oracle_f32 - shadow_f64| is the f32 oracle's own error, entry by entry (tests.helpers.report).
def _pix_ndc_t(i, S1, S2, dtype):
    rng = 2.0 * S1 / S2 if S1 > S2 else 2.0
    off = rng / 2.0
    return -off + (rng * i.to(dtype) + off) / S1


def _edge_t(px, py, ax, ay, bx, by):
    return (px - ax) * (by - ay) - (py - ay) * (bx - ax)


def _seg_dist2_t(px, py, ax, ay, bx, by):
    dx, dy = bx - ax, by - ay
    l2 = dx * dx + dy * dy
    degen = l2 <= 1e-8
    t = (dx * (px - ax) + dy * (py - ay)) / torch.where(degen, torch.ones_like(l2), l2)
    t = t.clamp(0.0, 1.0)
    qx, qy = ax + t * dx, ay + t * dy
    d_line = (px - qx) ** 2 + (py - qy) ** 2
    d_pt = (px - bx) ** 2 + (py - by) ** 2
    return torch.where(degen, d_pt, d_line)


def frag_eval_t(face_verts, p2f, H, W, persp=True, clip=False):
    """zbuf, bary, dists of the fragments named by p2f (N,H,W,K) from face_verts (differentiable,
    in face_verts' dtype): RasterizeMeshesNaiveCpu's per-(pixel, face) formulas
    at decisions already taken; background entries are -1."""
    N, H_, W_, K = p2f.shape
    dt = face_verts.dtype
    valid = p2f >= 0
    v = face_verts[p2f.clamp(min=0)]  # (N,H,W,K,3,3)
    yi = torch.arange(H).view(1, H, 1, 1)
    xi = torch.arange(W).view(1, 1, W, 1)
    py = _pix_ndc_t(H - 1 - yi, H, W, dt)
    px = _pix_ndc_t(W - 1 - xi, W, H, dt)
    x0, y0, z0 = v[..., 0, 0], v[..., 0, 1], v[..., 0, 2]
    x1, y1, z1 = v[..., 1, 0], v[..., 1, 1], v[..., 1, 2]
    x2, y2, z2 = v[..., 2, 0], v[..., 2, 1], v[..., 2, 2]
    area = _edge_t(x2, y2, x0, y0, x1, y1) + 1e-8
    w0 = _edge_t(px, py, x1, y1, x2, y2) / area
    w1 = _edge_t(px, py, x2, y2, x0, y0) / area
    w2 = _edge_t(px, py, x0, y0, x1, y1) / area
    if persp:
        t0, t1, t2 = w0 * z1 * z2, w1 * z0 * z2, w2 * z0 * z1
        d = (t0 + t1 + t2).clamp(min=1e-8)
        c0, c1, c2 = t0 / d, t1 / d, t2 / d
    else:
        c0, c1, c2 = w0, w1, w2
    if clip:
        u0, u1, u2 = c0.clamp(min=0.0), c1.clamp(min=0.0), c2.clamp(min=0.0)
        s = (u0 + u1 + u2).clamp(min=1e-5)
        b0, b1, b2 = u0 / s, u1 / s, u2 / s
    else:
        b0, b1, b2 = c0, c1, c2
    pz = b0 * z0 + b1 * z1 + b2 * z2
    dist = torch.minimum(torch.minimum(_seg_dist2_t(px, py, x0, y0, x1, y1), _seg_dist2_t(px, py, x0, y0, x2, y2)),
                         _seg_dist2_t(px, py, x1, y1, x2, y2))
    inside = (c0 > 0) & (c1 > 0) & (c2 > 0)
    sd = torch.where(inside, -dist, dist)
    m1 = torch.full_like(pz, -1.0)
    zbuf = torch.where(valid, pz, m1)
    dists = torch.where(valid, sd, m1)
    bary = torch.where(valid[..., None], torch.stack([b0, b1, b2], -1), m1[..., None].expand(*m1.shape, 3))
    return zbuf, bary, dists


def _shadow_fragments(verts, faces, R, T, intr, H, W, K, blur, persp, clip, z_clip, window):
    """f32 decisions (projection + near-plane split + C raster), then the float64 differentiable
    re-evaluation of the kept fragments. Returns (p2f, zbuf, bary, dists, face_verts64)."""
    N = R.shape[0]
    Fn = faces.shape[0]
    first = torch.arange(N, dtype=torch.int64) * Fn
    count = torch.full((N,), Fn, dtype=torch.int64)
    with torch.no_grad():
        fv32 = project_faces_torch(verts.detach().float(), faces, R.detach().float(), T.detach().float(),
                                   intr.detach().float())
        if z_clip is not None:
            cf32 = clip_faces_ref(fv32, first, count, z_clip, persp)
            p2f_c = raster_fwd(cf32["face_verts"], cf32["first"], cf32["count"], H, W, K, blur, persp, clip, False,
                               cf32["neighbor"], window)[0]
        else:
            p2f_c = raster_fwd(fv32, first, count, H, W, K, blur, persp, clip, False, None, window)[0]
    fv = project_faces_torch(verts.double(), faces, R.double(), T.double(), intr.double())
    if z_clip is None:
        zbuf, bary, dists = frag_eval_t(fv, p2f_c, H, W, persp, clip)
        return p2f_c, zbuf, bary, dists, fv
    cf = clip_faces_ref(fv, first, count, z_clip, persp)
    if not torch.equal(cf["orig"], cf32["orig"]):
        raise RuntimeError("f64 shadow: the near-plane split differs from the f32 run's")
    zbuf, bary_c, dists = frag_eval_t(cf["face_verts"], p2f_c, H, W, persp, clip)
    p2f, bary = unclip_fragments(p2f_c, bary_c, cf)
    return p2f, zbuf, bary, dists, fv


def views_tensor(R, T, intr):
    """(N,16) view records {R row-major, T, ax, bx, ay, by} as in include/mi355r.h."""
    return torch.cat([R.reshape(-1, 9), T.reshape(-1, 3), intr.reshape(-1, 4)], dim=1).float().contiguous()


__all__ = ["raster_fwd", "raster_bwd", "RasterizeRef", "project_faces_c", "project_faces_torch", "render_ref",
           "vertex_normals", "views_tensor", "np"]
