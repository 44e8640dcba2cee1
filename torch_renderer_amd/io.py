"""OBJ / MTL / PNG loading — drop-in for the ``pytorch3d.io`` calls of the reference
(``load_objs_as_meshes`` at torch_renderer.py:8, renderer.py:75-76,
camera_pose_optimizer.py:102, mesh_deformer.py:93; ``load_obj`` at
camera_pose_optimizer.py:~80).

Semantics follow upstream pytorch3d/io/obj_io.py:
  * ``v``/``vt``/``vn``/``f`` records, 1-based (negative = relative) indices;
  * polygons fan-triangulated (v0, vi, vi+1);
  * missing texture / normal indices become -1;
  * ``mtllib`` + ``usemtl`` + ``map_Kd``: texture image read as RGB float32 / 255;
  * ``load_objs_as_meshes`` builds TexturesUV from the first material image
    (textures=None when the image is missing, e.g. data/sphere.mtl:12).
"""
from __future__ import annotations

import os
from collections import namedtuple

import numpy as np
import torch

Faces = namedtuple("Faces", "verts_idx normals_idx textures_idx materials_idx")
Aux = namedtuple("Aux", "normals verts_uvs material_colors texture_images texture_atlas")


def _parse_index(tok: str, n: int) -> int:
    i = int(tok)
    return i - 1 if i > 0 else n + i


def _read_image(path: str) -> torch.Tensor:
    from PIL import Image

    with Image.open(path) as im:
        arr = np.asarray(im.convert("RGB")).astype(np.float32) / 255.0
    return torch.from_numpy(arr)


def _load_mtl(path: str):
    mats, cur = {}, None
    if not os.path.exists(path):
        return mats
    with open(path, "r", errors="replace") as fh:
        for line in fh:
            tok = line.strip().split()
            if not tok or tok[0].startswith("#"):
                continue
            if tok[0] == "newmtl":
                cur = " ".join(tok[1:])
                mats[cur] = {}
            elif cur is not None and tok[0] in ("Ka", "Kd", "Ks") and len(tok) >= 4:
                mats[cur][tok[0]] = [float(x) for x in tok[1:4]]
            elif cur is not None and tok[0] == "Ns":
                mats[cur]["Ns"] = float(tok[1])
            elif cur is not None and tok[0] == "map_Kd":
                mats[cur]["map_Kd"] = " ".join(tok[1:])
    return mats


def load_obj(f, load_textures: bool = True, device="cpu"):
    """Returns (verts (V,3), Faces, Aux) like pytorch3d.io.load_obj."""
    path = os.fspath(f)
    base = os.path.dirname(path)
    verts, uvs, normals = [], [], []
    fv, fn, ft, fm = [], [], [], []
    mtl_files, mat_names, cur_mat = [], [], -1
    with open(path, "r", errors="replace") as fh:
        for line in fh:
            tok = line.split()
            if not tok:
                continue
            t = tok[0]
            if t == "v":
                verts.append([float(x) for x in tok[1:4]])
            elif t == "vt":
                uvs.append([float(x) for x in tok[1:3]])
            elif t == "vn":
                normals.append([float(x) for x in tok[1:4]])
            elif t == "f":
                corners = []
                for c in tok[1:]:
                    parts = c.split("/")
                    vi = _parse_index(parts[0], len(verts))
                    ti = _parse_index(parts[1], len(uvs)) if len(parts) > 1 and parts[1] else -1
                    ni = _parse_index(parts[2], len(normals)) if len(parts) > 2 and parts[2] else -1
                    corners.append((vi, ti, ni))
                if len(corners) < 3:
                    raise ValueError(f"Face with fewer than 3 vertices in {path}: {line.strip()}")
                for i in range(1, len(corners) - 1):
                    tri = (corners[0], corners[i], corners[i + 1])
                    fv.append([c[0] for c in tri])
                    ft.append([c[1] for c in tri])
                    fn.append([c[2] for c in tri])
                    fm.append(cur_mat)
            elif t == "mtllib":
                mtl_files.append(" ".join(tok[1:]))
            elif t == "usemtl":
                name = " ".join(tok[1:])
                if name not in mat_names:
                    mat_names.append(name)
                cur_mat = mat_names.index(name)
    verts_t = torch.tensor(verts, dtype=torch.float32).reshape(-1, 3)
    faces_idx = torch.tensor(fv, dtype=torch.int64).reshape(-1, 3)
    if faces_idx.numel() and (faces_idx.min() < 0 or faces_idx.max() >= verts_t.shape[0]):
        raise ValueError("Faces have invalid indices")
    textures_idx = torch.tensor(ft, dtype=torch.int64).reshape(-1, 3)
    normals_idx = torch.tensor(fn, dtype=torch.int64).reshape(-1, 3)
    materials_idx = torch.tensor(fm, dtype=torch.int64)
    texture_images, material_colors = {}, {}
    if load_textures:
        for mf in mtl_files:
            mats = _load_mtl(os.path.join(base, mf))
            for name, props in mats.items():
                material_colors[name] = {
                    "ambient_color": torch.tensor(props.get("Ka", [1.0, 1.0, 1.0])),
                    "diffuse_color": torch.tensor(props.get("Kd", [1.0, 1.0, 1.0])),
                    "specular_color": torch.tensor(props.get("Ks", [1.0, 1.0, 1.0])),
                    "shininess": torch.tensor(props.get("Ns", 10.0)),
                }
                img = props.get("map_Kd")
                if img is not None:
                    p = img if os.path.isabs(img) else os.path.join(base, img)
                    if os.path.exists(p):
                        texture_images[name] = _read_image(p)
    aux = Aux(
        normals=torch.tensor(normals, dtype=torch.float32).reshape(-1, 3) if normals else None,
        verts_uvs=torch.tensor(uvs, dtype=torch.float32).reshape(-1, 2) if uvs else None,
        material_colors=material_colors or None,
        texture_images=texture_images or None,
        texture_atlas=None,
    )
    dev = torch.device(device)
    faces = Faces(faces_idx.to(dev), normals_idx.to(dev), textures_idx.to(dev), materials_idx.to(dev))
    return verts_t.to(dev), faces, aux


def load_objs_as_meshes(files, device=None, load_textures: bool = True, **_unused):
    """Meshes with TexturesUV from the first texture image of each file (or no textures)."""
    from .structures import Meshes, TexturesUV

    verts_list, faces_list, tex_maps, fuvs, vuvs = [], [], [], [], []
    for f in files:
        verts, faces, aux = load_obj(f, load_textures=load_textures)
        verts_list.append(verts)
        faces_list.append(faces.verts_idx)
        if load_textures and aux.texture_images and aux.verts_uvs is not None:
            tex_maps.append(next(iter(aux.texture_images.values())))
            fuvs.append(faces.textures_idx.clamp(min=0))
            vuvs.append(aux.verts_uvs)
    textures = None
    if tex_maps and len(tex_maps) == len(files):
        textures = TexturesUV(maps=tex_maps, faces_uvs=fuvs, verts_uvs=vuvs)
    m = Meshes(verts=verts_list, faces=faces_list, textures=textures)
    return m.to(device) if device is not None else m
