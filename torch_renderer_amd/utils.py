"""Mesh construction helpers the reference's callers need.

* ``SubdivideMeshes`` — upstream ``pytorch3d.ops.SubdivideMeshes`` (no feature subdivision):
  every triangle (v0, v1, v2) becomes four, using one new vertex at the midpoint of each unique
  edge. Edges are numbered as upstream ``Meshes.edges_packed``: the per-face edges
  (v1,v2), (v2,v0), (v0,v1) sorted and made unique by ``min*V + max``; the midpoint of edge e is
  vertex ``V + e``. New faces, in order: all [v0, m01, m20], then all [v1, m12, m01], then all
  [v2, m20, m12], then all [m12, m20, m01] (orientation preserved).
* ``ico_sphere(level)`` — upstream ``pytorch3d.utils.ico_sphere``: the icosahedron subdivided
  ``level`` times, vertices projected back onto the unit sphere after every level.
* ``subdivided_sphere(levels)`` — the C5 workload of BASELINE.json (``mesh_deformer.py`` scale):
  ``data/sphere.obj`` (an ico-level-4 sphere, F=5120) subdivided twice with re-projection →
  F=81,920, V=40,962.

Faithful to upstream's documented construction; the exact edge numbering is restated from the
upstream source as recalled, without a copy to check against (parity of this generator is
unpinned — it only builds benchmark inputs).
"""
from __future__ import annotations

import math

import torch

from .structures import Meshes


def _unique_edges(faces: torch.Tensor, V: int):
    """(edges (E,2) sorted (min,max), face_to_edge (F,3)) with columns = edges opposite v0, v1, v2."""
    f = faces.long()
    e12 = torch.stack([f[:, 1], f[:, 2]], 1)
    e20 = torch.stack([f[:, 2], f[:, 0]], 1)
    e01 = torch.stack([f[:, 0], f[:, 1]], 1)
    edges = torch.cat([e12, e20, e01], 0)
    edges, _ = edges.sort(dim=1)
    h = edges[:, 0] * V + edges[:, 1]
    u, inv = torch.unique(h, return_inverse=True)
    uniq = torch.stack([u // V, u % V], 1)
    F = f.shape[0]
    f2e = inv.view(3, F).t().contiguous()
    return uniq, f2e


def subdivide(verts: torch.Tensor, faces: torch.Tensor):
    """One SubdivideMeshes step on a single mesh: (new_verts (V+E,3), new_faces (4F,3))."""
    V = verts.shape[0]
    edges, f2e = _unique_edges(faces, V)
    mid = verts[edges].mean(dim=1)
    new_verts = torch.cat([verts, mid], 0)
    f = faces.long()
    m = f2e + V  # midpoint vertex ids: column 0 = m12, 1 = m20, 2 = m01
    f0 = torch.stack([f[:, 0], m[:, 2], m[:, 1]], 1)
    f1 = torch.stack([f[:, 1], m[:, 0], m[:, 2]], 1)
    f2 = torch.stack([f[:, 2], m[:, 1], m[:, 0]], 1)
    f3 = m
    return new_verts, torch.cat([f0, f1, f2, f3], 0)


class SubdivideMeshes(torch.nn.Module):
    """upstream ops/subdivide_meshes.py SubdivideMeshes (geometry only)."""

    def forward(self, meshes: Meshes) -> Meshes:
        vl, fl = [], []
        for v, f in zip(meshes.verts_list(), meshes.faces_list()):
            nv, nf = subdivide(v, f)
            vl.append(nv)
            fl.append(nf)
        return Meshes(vl, fl)


def _icosahedron(device="cpu"):
    t = (1.0 + math.sqrt(5.0)) / 2.0
    verts = torch.tensor([[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t],
                          [0, 1, -t], [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]], dtype=torch.float32,
                         device=device)
    faces = torch.tensor([[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4],
                          [11, 10, 2], [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8],
                          [3, 8, 9], [4, 9, 5], [2, 4, 11], [6, 2, 10], [8, 6, 7], [9, 8, 1]], dtype=torch.int64,
                         device=device)
    return verts, faces


def _project_unit(v):
    return v / v.norm(p=2, dim=1, keepdim=True)


def ico_sphere(level: int = 0, device="cpu") -> Meshes:
    """Unit ico-sphere: 20 * 4**level faces."""
    if level < 0:
        raise ValueError("level must be >= 0")
    v, f = _icosahedron(device)
    v = _project_unit(v)
    for _ in range(level):
        v, f = subdivide(v, f)
        v = _project_unit(v)
    return Meshes([v], [f])


def subdivided_sphere(levels: int = 2, device="cpu") -> Meshes:
    """C5: the reference's data/sphere.obj (assets/sphere.npz, F=5120) subdivided `levels` times
    with re-projection onto the unit sphere (levels=2: F=81,920, V=40,962)."""
    from .assets import load_asset_arrays

    d = load_asset_arrays("sphere")
    v = torch.from_numpy(d["verts"]).float().to(device)
    f = torch.from_numpy(d["faces"]).long().to(device)
    for _ in range(levels):
        v, f = subdivide(v, f)
        v = _project_unit(v)
    return Meshes([v], [f])
