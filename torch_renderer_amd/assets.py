"""Bundled mesh assets (converted from the reference's data/ by tools/make_assets.py)."""
from __future__ import annotations

import os

import numpy as np
import torch

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")


def asset_path(name: str) -> str:
    return os.path.join(ASSET_DIR, name + ".npz")


def load_asset_arrays(name: str) -> dict:
    with np.load(asset_path(name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def load_asset(name: str, device="cpu", textures: bool = True):
    """Meshes for `name` (sphere, teapot, dolphin, cow); TexturesUV when a map is present
    (texture = uint8 / 255 in float32, exactly what pytorch3d.io produces)."""
    from .structures import Meshes, TexturesUV

    d = load_asset_arrays(name)
    verts = torch.from_numpy(d["verts"]).float()
    faces = torch.from_numpy(d["faces"]).long()
    tex = None
    if textures and "texture_u8" in d:
        img = torch.from_numpy(d["texture_u8"].astype(np.float32) / 255.0)
        tex = TexturesUV(maps=[img], faces_uvs=[torch.from_numpy(d["faces_uvs"]).long()],
                         verts_uvs=[torch.from_numpy(d["verts_uvs"]).float()])
    return Meshes([verts], [faces], tex).to(device)
