"""PyTorch3D-free ``Meshes`` and textures (the reference passes
``pytorch3d.structures.Meshes`` into every render call: torch_renderer.py:111,156).

A batch built with ``Meshes.extend(N)`` (batch_rendering_test.py:326,
pose_optimizer.py:104) is kept as ONE shared mesh + a repeat count: the MI355X
renderer projects and rasterizes that single copy for all N views instead of
materialising N copies (the upstream extend copies verts, faces and the 12 MB
texture map per view). Gradients reach the source vertices exactly as they do
through upstream's ``clone`` (sum over the views).
"""
from __future__ import annotations

import torch


class TexturesVertex:
    """Per-vertex colours (upstream renderer/mesh/textures.py TexturesVertex)."""

    def __init__(self, verts_features):
        if torch.is_tensor(verts_features):
            if verts_features.dim() != 3:
                raise ValueError("verts_features must be (N, V, C) or a list of (V, C)")
            verts_features = list(verts_features.unbind(0))
        self._feats = list(verts_features)

    def verts_features_list(self):
        return self._feats

    def verts_features_packed(self):
        return torch.cat(self._feats, 0)

    def extend(self, N):
        return TexturesVertex([f for f in self._feats for _ in range(N)])

    def to(self, device):
        return TexturesVertex([f.to(device) for f in self._feats])

    def __getitem__(self, i):
        return TexturesVertex([self._feats[i]])

    def requires_grad(self) -> bool:
        return False  # vertex colours are a differentiable input of the fused kernels


class TexturesUV:
    """UV texture (upstream TexturesUV; defaults align_corners=True,
    padding_mode='border', sampling_mode='bilinear' are the only ones supported)."""

    def __init__(self, maps, faces_uvs, verts_uvs, align_corners=True, padding_mode="border",
                 sampling_mode="bilinear"):
        if (align_corners, padding_mode, sampling_mode) != (True, "border", "bilinear"):
            raise NotImplementedError("TexturesUV: only align_corners=True, padding 'border', bilinear")
        if torch.is_tensor(maps):
            maps = list(maps.unbind(0)) if maps.dim() == 4 else [maps]
        if torch.is_tensor(faces_uvs):
            faces_uvs = list(faces_uvs.unbind(0)) if faces_uvs.dim() == 3 else [faces_uvs]
        if torch.is_tensor(verts_uvs):
            verts_uvs = list(verts_uvs.unbind(0)) if verts_uvs.dim() == 3 else [verts_uvs]
        self._maps, self._faces_uvs, self._verts_uvs = list(maps), list(faces_uvs), list(verts_uvs)
        self._rgba_cache = None
        self._idx_cache = None

    def maps_list(self):
        return self._maps

    def maps_padded(self):
        return torch.stack(self._maps, 0)

    def faces_uvs_list(self):
        return self._faces_uvs

    def verts_uvs_list(self):
        return self._verts_uvs

    def extend(self, N):
        t = TexturesUV([m for m in self._maps for _ in range(N)], [f for f in self._faces_uvs for _ in range(N)],
                       [v for v in self._verts_uvs for _ in range(N)])
        return t

    def to(self, device):
        return TexturesUV([m.to(device) for m in self._maps], [f.to(device) for f in self._faces_uvs],
                          [v.to(device) for v in self._verts_uvs])

    def __getitem__(self, i):
        return TexturesUV([self._maps[i]], [self._faces_uvs[i]], [self._verts_uvs[i]])

    def requires_grad(self) -> bool:
        """True when a map or verts_uvs tensor requires grad (deform_mesh_with_color.py:269-271,329):
        the fused K=1 kernels sample a cached copy and carry no gradient to them, so such renders
        take the modular path (HIP raster + differentiable shading over the fragments)."""
        return any(t.requires_grad for t in self._maps + self._verts_uvs)

    def kernel_uvs(self, i=0):
        """(verts_uvs float32, faces_uvs int32) of mesh i, contiguous, as the kernels read them.
        Cached per source tensor version, so a steady render loop (or a captured HIP graph)
        launches no per-step cast/copy kernels."""
        vu, fu = self._verts_uvs[i], self._faces_uvs[i]
        key = (vu.data_ptr(), fu.data_ptr(), vu.device, getattr(vu, "_version", 0), getattr(fu, "_version", 0))
        if self._idx_cache is None or self._idx_cache[0] != key:
            self._idx_cache = (key, vu.float().contiguous(), fu.to(torch.int32).contiguous())
        return self._idx_cache[1], self._idx_cache[2]

    def rgba_map(self, i=0):
        """(Ht, Wt, 4) float32 copy of map i, padded for 16-byte texel loads (cached)."""
        m = self._maps[i]
        key = (m.data_ptr(), m.device, getattr(m, "_version", 0))
        if self._rgba_cache is None or self._rgba_cache[0] != key:
            Ht, Wt, C = m.shape
            rgba = torch.zeros((Ht, Wt, 4), dtype=torch.float32, device=m.device)
            rgba[..., :min(C, 3)] = m[..., :3].float()
            self._rgba_cache = (key, rgba.contiguous())
            self._u8_cache = None
        return self._rgba_cache[1]

    def u8_map(self, i=0):
        """(8-bit (Ht, Wt, 4) copy, (256,) f32 table) of rgba_map(i) when every value is exactly
        table[k] = float32(k) / 255 for some k (a PNG read as uint8 / 255), else None. The samplers
        then read 4-B texels, bitwise the same values. Checked once per map version (cached)."""
        rgba = self.rgba_map(i)
        if getattr(self, "_u8_cache", None) is not None and self._u8_cache[0] is rgba:
            return self._u8_cache[1]
        lut_cpu = torch.arange(256, dtype=torch.float32) / 255.0  # IEEE float32 division
        lut = lut_cpu.to(rgba.device)
        q = torch.round(rgba * 255.0).clamp(0, 255).to(torch.uint8)
        exact = bool(torch.equal(lut[q.long()], rgba))
        res = (q.contiguous(), lut) if exact else None
        self._u8_cache = (rgba, res)
        return res


class Meshes:
    """Batch of triangle meshes (subset of upstream structures/meshes.py used by the reference)."""

    def __init__(self, verts=None, faces=None, textures=None):
        if torch.is_tensor(verts):
            verts = list(verts.unbind(0))
        if torch.is_tensor(faces):
            faces = list(faces.unbind(0))
        if verts is None or faces is None or len(verts) != len(faces):
            raise ValueError("Meshes: verts and faces must be lists of equal length")
        self._verts_list = list(verts)
        self._faces_list = [f.to(torch.int64) for f in faces]
        self.textures = textures
        self._shared = None  # (src_index, N): all meshes are views of mesh 0 (extend)
        self._adj = None

    # --- construction helpers
    @classmethod
    def _shared_batch(cls, verts, faces, textures, N):
        m = cls.__new__(cls)
        m._verts_list = [verts]
        m._faces_list = [faces]
        m.textures = textures
        m._shared = N
        m._adj = None
        return m

    def extend(self, N: int):
        if not isinstance(N, int) or N < 1:
            raise ValueError("N must be a positive integer")
        if len(self) == 1:
            base_tex = self.textures
            return Meshes._shared_batch(self._verts_list[0], self._faces_list[0], base_tex, N * self.num_shared())
        verts = [v for v in self.verts_list() for _ in range(N)]
        faces = [f for f in self.faces_list() for _ in range(N)]
        tex = self.textures.extend(N) if self.textures is not None else None
        return Meshes(verts, faces, tex)

    # --- shared-batch introspection (MI355X renderer)
    def num_shared(self) -> int:
        return self._shared or 1

    def is_shared(self) -> bool:
        """True when every mesh of the batch is the same mesh (single or extended)."""
        return self._shared is not None or len(self._verts_list) == 1

    def shared_verts(self):
        return self._verts_list[0]

    def shared_faces(self):
        return self._faces_list[0]

    # --- upstream API
    def __len__(self):
        return self._shared if self._shared is not None else len(self._verts_list)

    @property
    def device(self):
        return self._verts_list[0].device

    def isempty(self):
        return len(self) == 0 or all(f.numel() == 0 for f in self._faces_list)

    def verts_list(self):
        if self._shared is not None:
            return [self._verts_list[0].clone() for _ in range(self._shared)]
        return self._verts_list

    def faces_list(self):
        if self._shared is not None:
            return [self._faces_list[0] for _ in range(self._shared)]
        return self._faces_list

    def num_verts_per_mesh(self):
        return torch.tensor([v.shape[0] for v in self.verts_list()], device=self.device)

    def num_faces_per_mesh(self):
        return torch.tensor([f.shape[0] for f in self.faces_list()], device=self.device)

    def verts_packed(self):
        if self._shared is not None:
            return self._verts_list[0].repeat(self._shared, 1)
        return torch.cat(self._verts_list, 0)

    def faces_packed(self):
        fl = self.faces_list()
        off = 0
        out = []
        for v, f in zip(self.verts_list(), fl):
            out.append(f + off)
            off += v.shape[0]
        return torch.cat(out, 0)

    def verts_padded(self):
        vl = self.verts_list()
        Vmax = max(v.shape[0] for v in vl)
        out = vl[0].new_zeros((len(vl), Vmax, 3))
        for i, v in enumerate(vl):
            out[i, : v.shape[0]] = v
        return out

    def mesh_to_faces_packed_first_idx(self):
        counts = self.num_faces_per_mesh()
        return torch.cumsum(counts, 0) - counts

    def verts_normals_packed(self):
        from .kernels import vertex_normals

        if self._shared is not None or len(self._verts_list) == 1:
            vn, _ = vertex_normals(self._verts_list[0], self._faces_list[0])
            return vn.repeat(len(self), 1)
        return torch.cat([vertex_normals(v, f)[0] for v, f in zip(self._verts_list, self._faces_list)], 0)

    def offset_verts(self, vert_offsets_packed):
        if self._shared is not None:
            V = self._verts_list[0].shape[0]
            off = vert_offsets_packed.view(self._shared, V, 3)
            verts = [self._verts_list[0] + off[i] for i in range(self._shared)]
            return Meshes(verts, self.faces_list(), self.textures)
        sizes = [v.shape[0] for v in self._verts_list]
        offs = vert_offsets_packed.split(sizes, 0)
        return Meshes([v + o for v, o in zip(self._verts_list, offs)], self._faces_list, self.textures)

    def offset_verts_(self, vert_offsets_packed):
        """In-place offset (mesh_deformer.py:103): a (3,) offset applies to every vertex, a
        (sum V, 3) one per packed vertex (a shared/extended batch takes a per-source-vertex (V,3)
        offset, which keeps it shared)."""
        off = torch.as_tensor(vert_offsets_packed, dtype=self._verts_list[0].dtype, device=self.device)
        if off.dim() == 1 or off.shape[0] == 1:
            self._verts_list = [v + off.reshape(1, 3) for v in self._verts_list]
            return self
        if self._shared is not None:
            V = self._verts_list[0].shape[0]
            if off.shape[0] == V:
                self._verts_list = [self._verts_list[0] + off]
                return self
            raise ValueError("offset_verts_ on an extended batch needs one (V,3) offset shared by all meshes")
        sizes = [v.shape[0] for v in self._verts_list]
        if off.shape[0] != sum(sizes):
            raise ValueError("Verts offsets must have dimension (all_v, 3).")
        self._verts_list = [v + o for v, o in zip(self._verts_list, off.split(sizes, 0))]
        return self

    def scale_verts_(self, scale):
        """In-place uniform scale per mesh (mesh_deformer.py:104): a float or an (N,) tensor."""
        sc = torch.as_tensor(scale, dtype=self._verts_list[0].dtype, device=self.device).reshape(-1)
        if sc.numel() == 1:
            self._verts_list = [v * sc for v in self._verts_list]
            return self
        if self._shared is not None or sc.numel() != len(self._verts_list):
            raise ValueError("scale_verts_: one scale per mesh (a shared batch takes a single scale)")
        self._verts_list = [v * sc[i] for i, v in enumerate(self._verts_list)]
        return self

    def scale_verts(self, scale):
        return self.clone().scale_verts_(scale)

    def update_padded(self, new_verts_padded):
        vl = [new_verts_padded[i, : v.shape[0]] for i, v in enumerate(self.verts_list())]
        return Meshes(vl, self.faces_list(), self.textures)

    def to(self, device):
        dev = torch.device(device) if device is not None else self.device
        m = Meshes.__new__(Meshes)
        m._verts_list = [v.to(dev) for v in self._verts_list]
        m._faces_list = [f.to(dev) for f in self._faces_list]
        m.textures = self.textures.to(dev) if self.textures is not None else None
        m._shared = self._shared
        m._adj = None
        return m

    def cuda(self):
        return self.to("cuda")

    def clone(self):
        m = Meshes.__new__(Meshes)
        m._verts_list = [v.clone() for v in self._verts_list]
        m._faces_list = [f.clone() for f in self._faces_list]
        m.textures = self.textures
        m._shared = self._shared
        m._adj = None
        return m

    def detach(self):
        m = self.clone()
        m._verts_list = [v.detach() for v in m._verts_list]
        return m

    def __getitem__(self, i):
        if self._shared is not None:
            return Meshes([self._verts_list[0]], [self._faces_list[0]], self.textures)
        tex = self.textures[i] if self.textures is not None else None
        return Meshes([self._verts_list[i]], [self._faces_list[i]], tex)
