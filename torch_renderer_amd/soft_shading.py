"""Shading of stored ``Fragments`` (faces_per_pixel >= 1, blur >= 0): the modular soft path.

The fused kernels (``mr_render_forward`` / ``k_bwd_fused``) shade the single nearest face of
every pixel inside the raster launch; that covers the reference's default settings
(``faces_per_pixel=1``, ``blur_radius=0``, torch_renderer.py:90-95,136-140). Soft rasterization
(``deform_mesh_with_color.py:153-159`` with K=50,
``renderer_comparison_with_pyrender.py:174-179``) keeps K faces per pixel, so shading becomes a
per-(pixel, k) pass over the fragments that ``mr_rasterize_meshes`` (HIP, any K) produced.

This module is that pass, written as device tensor expressions that follow upstream PyTorch3D
term by term, so autograd carries gradients back into ``Fragments`` (and from there through
``mr_rasterize_meshes_backward``) and into vertex positions, colours and texture maps:

* ``interpolate_face_attributes`` — upstream ops/interp_face_attrs.py (python form);
* ``sample_textures`` — upstream mesh/textures.py ``TexturesVertex`` / ``TexturesUV``
  (bilinear ``grid_sample``, ``align_corners=True``, ``padding_mode="border"``, y-flipped map);
* ``phong_shading`` — upstream mesh/shading.py ``phong_shading`` + ``_apply_lighting`` with
  ``PointLights`` / ``AmbientLights`` and ``Materials`` (normals from ``verts_normals_packed``,
  area-weighted, ``normalize(eps=1e-6)``);
* ``softmax_rgb_blend`` / ``sigmoid_alpha_blend`` — upstream mesh/blending.py.

Everything runs on the tensors' device (the fragments come from the HIP rasterizer, which
refuses CPU tensors), so there is no CPU fallback in the render path.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def interpolate_face_attributes(pix_to_face: torch.Tensor, bary: torch.Tensor, face_attrs: torch.Tensor):
    """out[n,h,w,k] = sum_i bary[n,h,w,k,i] * face_attrs[p2f, i]; background (p2f < 0) -> 0."""
    N, H, W, K = pix_to_face.shape
    D = face_attrs.shape[-1]
    mask = pix_to_face < 0
    idx = pix_to_face.clamp(min=0).reshape(-1)
    vals = face_attrs.index_select(0, idx).view(N, H, W, K, 3, D)
    out = (bary[..., None] * vals).sum(dim=-2)
    return out.masked_fill(mask[..., None], 0.0)


def face_vertex_normals(verts_packed: torch.Tensor, faces_packed: torch.Tensor):
    """Meshes.verts_normals_packed (area-weighted face normals summed per vertex), differentiable."""
    f = faces_packed.long()
    vf = verts_packed[f]
    fn = torch.cross(vf[:, 2] - vf[:, 1], vf[:, 0] - vf[:, 1], dim=1)
    vn = torch.zeros_like(verts_packed)
    vn = vn.index_add(0, f[:, 0], fn).index_add(0, f[:, 1], fn).index_add(0, f[:, 2], fn)
    return F.normalize(vn, eps=1e-6, dim=1)


def _packed_per_mesh(list_, counts, name):
    """Concatenate per-mesh tensors; a single entry shared by a batch (Meshes.extend) repeats."""
    if len(list_) == len(counts):
        return list_
    if len(list_) == 1:
        return list_ * len(counts)
    raise ValueError(f"{name}: {len(list_)} entries for a batch of {len(counts)} meshes")


def sample_textures(meshes, fragments):
    """Meshes.sample_textures(fragments) -> texels (N,H,W,K,C)."""
    from .structures import TexturesUV, TexturesVertex

    p2f, bary = fragments.pix_to_face, fragments.bary_coords
    N, H, W, K = p2f.shape
    tex = meshes.textures
    if tex is None:
        raise ValueError("Meshes does not have textures")  # upstream Meshes.sample_textures
    faces_packed = meshes.faces_packed().to(p2f.device)
    if isinstance(tex, TexturesVertex):
        feats = _packed_per_mesh(tex.verts_features_list(), meshes.verts_list(), "TexturesVertex")
        vc = torch.cat([f.to(p2f.device) for f in feats], 0)
        return interpolate_face_attributes(p2f, bary, vc[faces_packed.long()])
    if isinstance(tex, TexturesUV):
        n_mesh = len(meshes)
        fuv = _packed_per_mesh(tex.faces_uvs_list(), range(n_mesh), "TexturesUV.faces_uvs")
        vuv = _packed_per_mesh(tex.verts_uvs_list(), range(n_mesh), "TexturesUV.verts_uvs")
        maps = _packed_per_mesh(tex.maps_list(), range(n_mesh), "TexturesUV.maps")
        face_uvs = torch.cat([v.to(p2f.device)[f.to(p2f.device).long()] for v, f in zip(vuv, fuv)], 0)
        uvs = interpolate_face_attributes(p2f, bary, face_uvs)                    # (N,H,W,K,2)
        uvs = uvs.permute(0, 3, 1, 2, 4).reshape(N * K, H, W, 2) * 2.0 - 1.0
        if any(m.shape != maps[0].shape for m in maps):
            raise NotImplementedError("TexturesUV: maps of different sizes in one batch")
        if all(m is maps[0] for m in maps):
            mp = maps[0].to(p2f.device).permute(2, 0, 1)[None].expand(N * K, -1, -1, -1)
        else:
            mp = torch.stack([m.to(p2f.device) for m in maps], 0).permute(0, 3, 1, 2)
            mp = mp[:, None].expand(-1, K, -1, -1, -1).reshape(N * K, *mp.shape[1:])
        mp = torch.flip(mp, [2])
        C = mp.shape[1]
        texels = F.grid_sample(mp, uvs, mode="bilinear", align_corners=True, padding_mode="border")
        return texels.reshape(N, K, C, H, W).permute(0, 3, 4, 1, 2)
    raise NotImplementedError(f"textures of type {type(tex).__name__}")


def _col(t, dev):
    return torch.tensor(t, dtype=torch.float32, device=dev)


def phong_shading(meshes, fragments, texels, lights, materials, camera_center):
    """upstream shading.py phong_shading -> (N,H,W,K,3) colours."""
    from .mesh_renderer import AmbientLights, PointLights

    p2f, bary = fragments.pix_to_face, fragments.bary_coords
    dev = p2f.device
    amb = _col(materials.ambient_color, dev) * _col(lights.ambient_color, dev)
    if isinstance(lights, AmbientLights):
        return amb * texels
    if not isinstance(lights, PointLights):
        raise NotImplementedError(f"lights of type {type(lights).__name__}")
    verts = meshes.verts_packed().to(dev)
    faces = meshes.faces_packed().to(dev).long()
    vn = face_vertex_normals(verts, faces)
    coords = interpolate_face_attributes(p2f, bary, verts[faces])
    normals = interpolate_face_attributes(p2f, bary, vn[faces])
    direction = _col(lights.location_tuple(), dev) - coords
    nh = F.normalize(normals, p=2, dim=-1, eps=1e-6)
    lh = F.normalize(direction, p=2, dim=-1, eps=1e-6)
    cos_angle = torch.sum(nh * lh, dim=-1)
    diffuse = _col(materials.diffuse_color, dev) * (_col(lights.diffuse_color, dev) * F.relu(cos_angle)[..., None])
    mask = (cos_angle > 0).to(torch.float32)
    cc = camera_center.to(dev).reshape(-1, 1, 1, 1, 3)
    view_direction = F.normalize(cc - coords, p=2, dim=-1, eps=1e-6)
    reflect = -lh + 2 * (cos_angle[..., None] * nh)
    alpha = F.relu(torch.sum(view_direction * reflect, dim=-1)) * mask
    specular = _col(materials.specular_color, dev) * (_col(lights.specular_color, dev) *
                                                      torch.pow(alpha, materials.shininess)[..., None])
    return (amb + diffuse) * texels + specular


def softmax_rgb_blend(colors, fragments, blend_params, znear=1.0, zfar=100.0):
    """upstream blending.py softmax_rgb_blend -> (N,H,W,4)."""
    eps = 1e-10
    p2f, zbuf, dists = fragments.pix_to_face, fragments.zbuf, fragments.dists
    mask = p2f >= 0
    prob_map = torch.sigmoid(-dists / blend_params.sigma) * mask
    alpha = torch.prod(1.0 - prob_map, dim=-1)
    z_inv = (zfar - zbuf) / (zfar - znear) * mask
    z_inv_max = torch.max(z_inv, dim=-1).values[..., None].clamp(min=eps)
    weights_num = prob_map * torch.exp((z_inv - z_inv_max) / blend_params.gamma)
    delta = torch.exp((eps - z_inv_max) / blend_params.gamma).clamp(min=eps)
    denom = weights_num.sum(dim=-1)[..., None] + delta
    weighted_colors = (weights_num[..., None] * colors).sum(dim=-2)
    bg = _col(tuple(blend_params.background_color), colors.device)
    rgb = (weighted_colors + delta * bg) / denom
    return torch.cat([rgb, (1.0 - alpha)[..., None]], dim=-1)


def sigmoid_alpha_blend(fragments, blend_params):
    """upstream blending.py sigmoid_alpha_blend -> (N,H,W,4) with RGB = 1."""
    mask = fragments.pix_to_face >= 0
    prob = torch.sigmoid(-fragments.dists / blend_params.sigma) * mask
    alpha = 1.0 - torch.prod(1.0 - prob, dim=-1)
    return torch.cat([torch.ones(alpha.shape + (3,), device=alpha.device, dtype=alpha.dtype), alpha[..., None]], -1)
