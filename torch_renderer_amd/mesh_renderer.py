"""PyTorch3D-style rendering API on the MI355X kernels.

The reference reaches the render path through PyTorch3D's classes
(torch_renderer.py:87-108,132-153; renderer.py:71-101; camera_pose_optimizer.py:131-158,244-250):
``RasterizationSettings``, ``MeshRasterizer`` -> ``Fragments``, ``PointLights`` /
``AmbientLights`` / ``Materials`` / ``BlendParams``, ``SoftPhongShader``,
``SoftSilhouetteShader`` and ``MeshRenderer``. This module mirrors their constructors,
argument meaning and outputs:

* ``MeshRasterizer(meshes)`` runs the modular path — ``mr_project_faces`` then
  ``mr_rasterize_meshes`` (the ``pytorch3d._C.rasterize_meshes`` boundary), or for one mesh shared
  by every view both in one call (``mr_rasterize_meshes_world``, bitwise the same) — and returns
  ``Fragments`` in PyTorch3D layout (int64 packed ``pix_to_face`` (N,H,W,K), zbuf, bary_coords,
  dists), differentiable w.r.t. vertex positions and R, T.
* ``MeshRenderer(meshes)`` with a Soft* shader runs ONE fused launch (project + bin +
  raster + shade + blend, ``mr_render_forward``) and returns the shader's (N,H,W,4) image,
  differentiable w.r.t. vertex positions, R, T and vertex colours.

* With ``faces_per_pixel > 1`` or ``blur_radius > 0`` (soft rasterization),
  or a texture map that needs gradients, ``MeshRenderer`` runs the K-deep HIP rasterizer and then
  the shader over the stored fragments on the HIP kernels (``mr_shade_fragments_*``: per-fragment
  Phong, softmax_rgb_blend / sigmoid_alpha_blend, analytic backward), as upstream composes them.

Rasterization always runs on the HIP kernels; there is no CPU fallback. Near-plane clipping
(``z_clip_value``, znear / 2 for FoV cameras: upstream clip_faces) runs inside the HIP binning. The
one setting the MI355X path does not implement (cull_to_frustum) raises ``NotImplementedError``
rather than returning different numbers.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field

import torch

from .cameras import CamerasBase, view_batch
from .kernels import ProjectFaces, ProjectFacesMeshes, RasterizeFaceVerts, RasterizeMeshesWorld, ShadeConfig
from .structures import Meshes


# --------------------------------------------------------------------------- settings / params
@dataclass
class RasterizationSettings:
    """upstream mesh/rasterizer.py RasterizationSettings (image_size int -> square)."""
    image_size: int | tuple = 256
    blur_radius: float = 0.0
    faces_per_pixel: int = 1
    bin_size: int | None = None           # accepted; the MI355X binning uses fixed 8x8 tiles
    max_faces_per_bin: int | None = None  # list-pool reservation; overflow stays exact
    perspective_correct: bool | None = None
    clip_barycentric_coords: bool | None = None
    cull_backfaces: bool = False
    z_clip_value: float | None = None
    cull_to_frustum: bool = False

    def hw(self):
        s = self.image_size
        if isinstance(s, int):
            return s, s
        return int(s[0]), int(s[1])


@dataclass
class BlendParams:
    """upstream blending.py BlendParams."""
    sigma: float = 1e-4
    gamma: float = 1e-4
    background_color: tuple = (1.0, 1.0, 1.0)


def _bg_triple(bp):
    """background_color as floats. Upstream reads the field on every call, so a colour mutated in
    place or reassigned takes effect: cached only for an unchanged tensor (same storage and
    version; its conversion is a host read), re-read for lists / tuples (three floats, no device
    work)."""
    bc = bp.background_color
    if not torch.is_tensor(bc):
        if type(bc) in (tuple, list) and len(bc) == 3 and all(type(x) in (float, int) for x in bc):
            return (float(bc[0]), float(bc[1]), float(bc[2]))  # the common case: three numbers, no tensor work
        return _triple(bc, None, "BlendParams.background_color")
    key = (bc.data_ptr(), bc._version, tuple(bc.shape), str(bc.device))
    c = bp.__dict__.get("_bg_cache")
    if c is None or c[0] != key:
        c = (key, _triple(bc, None, "BlendParams.background_color"))
        bp.__dict__["_bg_cache"] = c
    return c[1]


def _triple(x, default, what="lights/materials"):
    """One RGB (or xyz) triple as Python floats, converted ONCE at construction (a device tensor
    costs one host read here, never per render call). Differentiable light / material
    parameters are not supported by the fused kernels: refuse them instead of dropping the
    gradient."""
    if x is None:
        x = default
    if torch.is_tensor(x) and x.requires_grad:
        raise NotImplementedError(f"{what}: parameters that require grad are not supported on the MI355X path")
    t = torch.as_tensor(x, dtype=torch.float32).reshape(-1)
    if t.numel() == 1:
        t = t.expand(3)
    if t.numel() != 3:
        raise NotImplementedError(f"{what}: one colour per batch (3 values) is supported")
    return tuple(float(v) for v in t.cpu())


def _tensor_sig(v):
    return (v.data_ptr(), v._version, tuple(v.shape), str(v.device)) if torch.is_tensor(v) else None


def _triple_property(name, what):
    """A light / material field that re-converts on assignment (upstream reads the tensors on every
    call, so e.g. renderer.py:82-83 ``lights.location = ...`` takes effect on the next render) and,
    for a tensor value, again whenever the tensor is edited in place (``lights.location[0, 2] = -5.``:
    its storage or version changes), as _bg_triple does. The getter returns what was assigned;
    _field_triple(obj, name) is the float triple the kernels take."""
    def get(self):
        return self.__dict__["_raw_" + name]

    def set_(self, v):
        self.__dict__["_" + name] = (_tensor_sig(v), _triple(v, None, what))  # validates (grad, shape)
        self.__dict__["_raw_" + name] = v
        self.__dict__["_what_" + name] = what

    return property(get, set_)


def _field_triple(obj, name):
    sig, trip = obj.__dict__["_" + name]
    raw = obj.__dict__["_raw_" + name]
    if sig is not None and _tensor_sig(raw) != sig:  # edited in place since the last conversion
        sig, trip = _tensor_sig(raw), _triple(raw, None, obj.__dict__["_what_" + name])
        obj.__dict__["_" + name] = (sig, trip)
    return trip


class PointLights:
    """upstream lighting.py PointLights (one light shared by the batch)."""

    location = _triple_property("location", "PointLights.location")
    ambient_color = _triple_property("ambient", "PointLights.ambient_color")
    diffuse_color = _triple_property("diffuse", "PointLights.diffuse_color")
    specular_color = _triple_property("specular", "PointLights.specular_color")

    def __init__(self, ambient_color=((0.5, 0.5, 0.5),), diffuse_color=((0.3, 0.3, 0.3),),
                 specular_color=((0.2, 0.2, 0.2),), location=((0, 1, 0),), device="cpu"):
        self.device = device
        self.ambient_color = ambient_color
        self.diffuse_color = diffuse_color
        self.specular_color = specular_color
        self.location = location

    def location_tuple(self):
        return _field_triple(self, "location")

    def color_tuples(self):
        """(ambient, diffuse, specular) as float triples."""
        return _field_triple(self, "ambient"), _field_triple(self, "diffuse"), _field_triple(self, "specular")


class AmbientLights:
    """upstream lighting.py AmbientLights (mesh_deformer.py:113): colour = ambient * texel."""

    ambient_color = _triple_property("ambient", "AmbientLights.ambient_color")

    def __init__(self, ambient_color=((1.0, 1.0, 1.0),), device="cpu"):
        self.device = device
        self.ambient_color = ambient_color

    def ambient_tuple(self):
        return _field_triple(self, "ambient")


class Materials:
    """upstream materials.py Materials."""

    ambient_color = _triple_property("ambient", "Materials.ambient_color")
    diffuse_color = _triple_property("diffuse", "Materials.diffuse_color")
    specular_color = _triple_property("specular", "Materials.specular_color")

    def __init__(self, ambient_color=((1, 1, 1),), diffuse_color=((1, 1, 1),), specular_color=((1, 1, 1),),
                 shininess=64, device="cpu"):
        self.device = device
        self.ambient_color = ambient_color
        self.diffuse_color = diffuse_color
        self.specular_color = specular_color
        self.shininess = shininess

    @property
    def shininess(self):
        return self.__dict__["_raw_shininess"]

    @shininess.setter
    def shininess(self, v):
        if torch.is_tensor(v) and v.requires_grad:
            raise NotImplementedError("Materials.shininess: parameters that require grad are not supported")
        self.__dict__["_shininess"] = float(torch.as_tensor(v).reshape(-1)[0].cpu())
        self.__dict__["_raw_shininess"] = v

    def color_tuples(self):
        return _field_triple(self, "ambient"), _field_triple(self, "diffuse"), _field_triple(self, "specular")

    def shininess_value(self):
        return self.__dict__["_shininess"]


@dataclass
class Fragments:
    """upstream mesh/rasterizer.py Fragments. ``sorted_slots`` (not upstream's): set by this library's
    rasterizer, whose empty slots (pix_to_face = -1) follow each pixel's filled ones, so the shaders
    stop at the first (MR_FRAG_SORTED); Fragments built elsewhere are shaded over all K slots."""
    pix_to_face: torch.Tensor
    zbuf: torch.Tensor
    bary_coords: torch.Tensor
    dists: torch.Tensor
    sorted_slots: bool = field(default=False, repr=False, compare=False)
    _p2f_sig: tuple | None = field(default=None, repr=False, compare=False)

    def __post_init__(self):
        # the slot order holds for pix_to_face as the rasterizer wrote it: an in-place edit (e.g.
        # masking faces with -1) or a replaced tensor turns the early stop off (shade every slot)
        if self.sorted_slots and self._p2f_sig is None:
            self._p2f_sig = _tensor_sig(self.pix_to_face)

    def slots_sorted(self) -> bool:
        if not self.sorted_slots:
            return False
        p2f = self.pix_to_face
        return self._p2f_sig is not None and _tensor_sig(p2f) == self._p2f_sig

    def materialize(self) -> "Fragments":
        """Every field computed now (a no-op here; see _LazyFragments)."""
        return self


class _LazyFragments(Fragments):
    """MeshRasterizer's K = 1 Fragments of one mesh shared by the views, computed on first access.
    ``zbuf`` alone — what camera_pose_optimizer.py:244-246 and batch_rendering_test.py:274 read —
    comes from the fused render in zbuf mode (mr_render_forward with MR_OUT_ZBUF: the nearest face's
    depth, -1 where no face; bitwise the modular rasterizer's zbuf), whose backward is the fused
    depth backward: no (N,H,W,1) pix_to_face / bary_coords / dists tensors written, and no
    per-fragment-slot raster backward. Reading pix_to_face, bary_coords or dists runs the modular
    rasterizer (RasterizeMeshesWorld) once for all three (and zbuf, if not read before)."""

    def __init__(self, zbuf_fn, full_fn):  # noqa: D107 (no dataclass __init__: the fields are lazy)
        self.__dict__["_zbuf_fn"] = zbuf_fn
        self.__dict__["_full_fn"] = full_fn
        self.sorted_slots = True
        self._p2f_sig = None

    def __getattr__(self, name):  # only for fields not computed yet
        d = self.__dict__
        if name == "zbuf":
            d["zbuf"] = d["_zbuf_fn"]()
            return d["zbuf"]
        if name in ("pix_to_face", "bary_coords", "dists"):
            p2f, zbuf, bary, dists = d["_full_fn"]()
            d.update(pix_to_face=p2f, bary_coords=bary, dists=dists)
            d.setdefault("zbuf", zbuf)
            d["_p2f_sig"] = _tensor_sig(p2f)
            return d[name]
        raise AttributeError(name)

    def materialize(self) -> "Fragments":
        _ = self.pix_to_face  # one modular pass for every field (zbuf too, when not read before)
        return self


# --------------------------------------------------------------------------- rasterizer
def _z_clip_value(cameras: CamerasBase, rs: RasterizationSettings):
    """MeshRasterizer: z_clip_value = znear / 2 for perspective cameras that have a znear."""
    if rs.z_clip_value is not None:
        return float(rs.z_clip_value)
    if cameras.is_perspective() and cameras.get_znear() is not None:
        return float(torch.as_tensor(cameras.get_znear()).min()) / 2.0
    return None


def _check_cull_to_frustum(cull_to_frustum):
    """Near-plane clipping (clip_faces) runs inside the HIP binning; frustum culling does not."""
    if cull_to_frustum:
        raise NotImplementedError("cull_to_frustum is not implemented on the MI355X path yet")


def _views(meshes: Meshes, cameras: CamerasBase, hw, kwargs):
    R = kwargs.get("R", None)
    T = kwargs.get("T", None)
    n = max(len(meshes), 1 if R is None else R.reshape(-1, 3, 3).shape[0],
            1 if T is None else T.reshape(-1, 3).shape[0])
    return view_batch(cameras, hw, R, T, n_views=n)


class MeshRasterizer(torch.nn.Module):
    """upstream mesh/rasterizer.py MeshRasterizer: world -> view -> NDC (MeshRasterizer.transform,
    with view z kept as the depth), then _C.rasterize_meshes (mr_rasterize_meshes)."""

    def __init__(self, cameras=None, raster_settings=None):
        super().__init__()
        self.cameras = cameras
        self.raster_settings = raster_settings or RasterizationSettings()

    def transform(self, meshes_world: Meshes, **kwargs):
        """Packed face_verts (sum F_n, 3, 3): NDC xy + view z, packed ids n*F + f."""
        meshes = meshes_world
        cameras = kwargs.get("cameras", self.cameras)
        if cameras is None:
            raise ValueError("Cameras must be specified either at initialization or in the forward pass")
        hw = kwargs.get("raster_settings", self.raster_settings).hw()  # a per-call raster_settings wins
        R, T, intr = _views(meshes, cameras, hw, kwargs)
        if meshes.is_shared():
            return ProjectFaces.apply(meshes.shared_verts(), R, T, meshes.shared_faces(), intr.contiguous())
        if len(meshes) != R.shape[0]:
            raise ValueError(f"Meshes batch ({len(meshes)}) and camera batch ({R.shape[0]}) differ")
        # distinct meshes: their union, view n projecting mesh n, in one launch
        from .torch_renderer import _union_topology
        faces_u, ffirst, _, fmax, vfirst, vmax = _union_topology(meshes)
        return ProjectFacesMeshes.apply(torch.cat(list(meshes.verts_list()), 0), R, T, faces_u, intr.contiguous(),
                                        ffirst, fmax, vfirst, vmax)

    def forward(self, meshes_world: Meshes, **kwargs) -> Fragments:
        """upstream signature: forward(meshes_world, **kwargs) (camera_pose_optimizer.py:175-177,244
        call it as rasterizer(meshes_world=..., R=..., T=...))."""
        meshes = meshes_world
        cameras = kwargs.get("cameras", self.cameras)
        rs = kwargs.get("raster_settings", self.raster_settings)
        H, W = rs.hw()
        _check_cull_to_frustum(rs.cull_to_frustum)
        persp = cameras.is_perspective() if rs.perspective_correct is None else bool(rs.perspective_correct)
        clip = rs.blur_radius > 0.0 if rs.clip_barycentric_coords is None else bool(rs.clip_barycentric_coords)
        if cameras is not None and meshes.is_shared():
            # one mesh for every view (Meshes.extend): transform + rasterize in one native call,
            # bitwise the two-step result below
            R, T, intr = _views(meshes, cameras, (H, W), kwargs)
            zc = _z_clip_value(cameras, rs)
            from .kernels import _require_cuda

            # what the call sees is captured now (the fields may be computed later, on first access): the
            # vertex / face tensors, their versions and the grad mode, as upstream's eager rasterizer
            # would have used them at this call
            verts, faces = meshes.shared_verts(), meshes.shared_faces()
            _require_cuda(verts, faces, R, T)  # fail at the call, not at first use
            grad_mode = torch.is_grad_enabled()
            versions = (verts._version, faces._version)

            def _check_unchanged():
                if (verts._version, faces._version) != versions:
                    raise RuntimeError("MeshRasterizer: the mesh's verts / faces were modified in place between the "
                                       "rasterizer call and the first access of its Fragments")

            def full():
                _check_unchanged()
                with torch.set_grad_enabled(grad_mode):
                    return RasterizeMeshesWorld.apply(
                        verts, R, T, faces, intr, R.shape[0], H, W,
                        int(rs.faces_per_pixel), float(rs.blur_radius), persp, clip, bool(rs.cull_backfaces),
                        rs.max_faces_per_bin, zc)

            if int(rs.faces_per_pixel) == 1 and float(rs.blur_radius) == 0.0:
                def zbuf_only():  # the fused render in zbuf mode (see _LazyFragments)
                    from .kernels import render_views

                    _check_unchanged()
                    cfg = ShadeConfig(H=H, W=W, persp=persp, clip=clip, cull=bool(rs.cull_backfaces),
                                      max_faces_per_bin=rs.max_faces_per_bin, light_kind=1, want_depth=True,
                                      want_sil=False, want_rgb=False, zbuf=True, z_clip=zc)
                    cc = torch.zeros((1, 3), device=R.device)
                    try:
                        with torch.set_grad_enabled(grad_mode):
                            return render_views(verts, R, T, faces, intr, cc, cfg)["depth"].unsqueeze(-1)
                    except NotImplementedError:  # MR_EUNSUPPORTED from the fused path: the modular rasterizer
                        return full()[1]

                return _LazyFragments(zbuf_only, full)
            p2f, zbuf, bary, dists = full()
            return Fragments(pix_to_face=p2f, zbuf=zbuf, bary_coords=bary, dists=dists, sorted_slots=True)
        fv = self.transform(meshes, **{**kwargs, "raster_settings": rs})
        first = meshes.mesh_to_faces_packed_first_idx().to(fv.device)
        count = meshes.num_faces_per_mesh().to(fv.device)
        # near-plane clipping (z_clip_value = znear / 2 for FoV cameras) happens inside the HIP
        # binning: split faces are rasterized and mapped back to the original faces in-kernel
        p2f, zbuf, bary, dists = RasterizeFaceVerts.apply(fv, first, count, H, W, int(rs.faces_per_pixel),
                                                          float(rs.blur_radius), persp, clip,
                                                          bool(rs.cull_backfaces), rs.max_faces_per_bin,
                                                          _z_clip_value(cameras, rs))
        return Fragments(pix_to_face=p2f, zbuf=zbuf, bary_coords=bary, dists=dists, sorted_slots=True)


def rasterize(meshes: Meshes, cameras: CamerasBase, raster_settings: RasterizationSettings, **kwargs) -> Fragments:
    """Functional form used by callers that consume fragments directly
    (camera_pose_optimizer.py:244-246, batch_rendering_test.py:274)."""
    return MeshRasterizer(cameras, raster_settings)(meshes, **kwargs)


# --------------------------------------------------------------------------- shaders / renderer
def _shade_config(sh, cameras, H, W, kwargs):
    """Lighting / material / blend part of a ShadeConfig for shader `sh`. Per-call ``lights=``,
    ``materials=``, ``blend_params=`` override the shader's own, as upstream SoftPhongShader.forward
    does (the reference passes ``lights=`` on every call: mesh_deformer.py:153,197,
    deform_mesh_with_color.py:185,342)."""
    bp = kwargs.get("blend_params", sh.blend_params)
    znear = kwargs.get("znear", getattr(cameras, "znear", 1.0))
    zfar = kwargs.get("zfar", getattr(cameras, "zfar", 100.0))
    cfg = ShadeConfig(H=H, W=W, sigma_rgb=float(bp.sigma), gamma=float(bp.gamma), background=_bg_triple(bp),
                      znear=float(znear), zfar=float(zfar), sigma_sil=float(bp.sigma), want_depth=False)
    if isinstance(sh, SoftSilhouetteShader):
        cfg.want_rgb = False
        cfg.want_sil = True
        return cfg
    if not isinstance(sh, (SoftPhongShader, HardPhongShader)):
        raise NotImplementedError(f"shader {type(sh).__name__} is not implemented on the MI355X path")
    cfg.hard = isinstance(sh, HardPhongShader)
    lights = kwargs.get("lights", sh.lights)
    mats = kwargs.get("materials", sh.materials)
    if isinstance(lights, AmbientLights):
        cfg.light_kind = 1
        cfg.light_ambient = lights.ambient_tuple()
    elif isinstance(lights, PointLights):
        cfg.light_kind = 0
        cfg.light_location = lights.location_tuple()
        cfg.light_ambient, cfg.light_diffuse, cfg.light_specular = lights.color_tuples()
    else:
        raise NotImplementedError(f"lights of type {type(lights).__name__}")
    cfg.mat_ambient, cfg.mat_diffuse, cfg.mat_specular = mats.color_tuples()
    cfg.shininess = mats.shininess_value()
    cfg.want_sil = False
    cfg.rgb_channels = 4
    return cfg


def shade_fragments(fragments: Fragments, meshes: Meshes, cfg: ShadeConfig, cam_center):
    """The shader over stored fragments on the HIP kernels (mr_shade_fragments_*): one launch for a
    batch of one shared mesh or of distinct meshes (their union; per mesh only when their UV maps
    differ). Returns (N,H,W,4)."""
    from .kernels import ShadeFragments
    from .structures import TexturesUV, TexturesVertex

    p2f = fragments.pix_to_face
    N = p2f.shape[0]
    tex = meshes.textures
    if isinstance(fragments, Fragments) and fragments.slots_sorted() and not cfg.frag_sorted:
        cfg = dataclasses.replace(cfg, frag_sorted=True)
    if cfg.want_rgb and tex is None:
        raise ValueError("Meshes does not have textures")  # upstream Meshes.sample_textures
    cc = cam_center.to(p2f.device).float().reshape(-1, 3)

    def one(i0, i1, verts, faces, tex_i, first):
        vc = tmap = vuv = fuv = None
        if cfg.want_rgb and isinstance(tex_i, TexturesVertex):
            vc = tex_i.verts_features_list()[0]
            if vc.shape[-1] != 3:
                raise NotImplementedError("TexturesVertex: only 3-channel features are supported")
        elif cfg.want_rgb and isinstance(tex_i, TexturesUV):
            tmap, fuv, vuv = tex_i.maps_list()[0], tex_i.faces_uvs_list()[0], tex_i.verts_uvs_list()[0]
        elif cfg.want_rgb:
            raise NotImplementedError(f"textures of type {type(tex_i).__name__}")
        whole = i0 == 0 and i1 == N  # the whole batch: no slices (a slice's backward would zero-fill
        sl = (lambda t: t) if whole else (lambda t: t[i0:i1])  # noqa: E731  and copy each fragment grad)
        q = sl(p2f)
        if first:
            q = torch.where(q >= 0, q - first, q)
        c = cc[i0:i1] if cc.shape[0] > 1 else cc
        return ShadeFragments.apply(sl(fragments.zbuf), sl(fragments.bary_coords), sl(fragments.dists),
                                    verts, vc, tmap, vuv, q.contiguous(), faces, fuv, c, cfg)

    if meshes.is_shared():
        return one(0, N, meshes.shared_verts(), meshes.shared_faces(), tex, 0)
    if len(meshes) == N and _union_shading_ok(tex, cfg):
        # distinct meshes: pix_to_face already holds union (packed) face ids
        from .torch_renderer import _union_topology
        faces_u, ffirst, fcount, fmax = _union_topology(meshes)[:4]
        vc = tmap = vuv = fuv = None
        if cfg.want_rgb and isinstance(tex, TexturesVertex):
            vc = torch.cat(list(tex.verts_features_list()), 0)
            if vc.shape[-1] != 3:
                raise NotImplementedError("TexturesVertex: only 3-channel features are supported")
        elif cfg.want_rgb and isinstance(tex, TexturesUV):
            tmap = tex.maps_list()[0]
            offs, o = [], 0
            for vu in tex.verts_uvs_list():
                offs.append(o)
                o += vu.shape[0]
            vuv = torch.cat(list(tex.verts_uvs_list()), 0)
            fuv = torch.cat([fu.to(torch.int64) + off for fu, off in zip(tex.faces_uvs_list(), offs)], 0)
        return ShadeFragments.apply(fragments.zbuf, fragments.bary_coords, fragments.dists,
                                    torch.cat(list(meshes.verts_list()), 0), vc, tmap, vuv, p2f.contiguous(), faces_u,
                                    fuv, cc, cfg, (ffirst, fcount, fmax))
    firsts = meshes.mesh_to_faces_packed_first_idx().tolist()
    outs = []
    for i in range(N):
        mi = meshes[i]
        outs.append(one(i, i + 1, mi.shared_verts(), mi.shared_faces(), mi.textures, int(firsts[i])))
    return torch.cat(outs, 0)


def _union_shading_ok(tex, cfg):
    """Whether a batch of distinct meshes can be shaded as one union mesh: any texture but UV maps
    that differ between the meshes."""
    from .structures import TexturesUV

    if not cfg.want_rgb or not isinstance(tex, TexturesUV):
        return True
    maps = tex.maps_list()
    return all(m is maps[0] for m in maps)


class _SoftShader(torch.nn.Module):
    def __init__(self, device="cpu", cameras=None, lights=None, materials=None, blend_params=None):
        super().__init__()
        self.cameras = cameras
        self.lights = lights if lights is not None else PointLights(device=device)
        self.materials = materials if materials is not None else Materials(device=device)
        self.blend_params = blend_params if blend_params is not None else BlendParams()

    def forward(self, fragments, meshes, **kwargs):
        cameras = kwargs.get("cameras", self.cameras)
        H, W = fragments.pix_to_face.shape[1:3]
        cfg = _shade_config(self, cameras, H, W, kwargs)
        if cfg.want_rgb and cameras is None:
            raise ValueError("Cameras must be specified either at initialization or in the forward pass")
        from .cameras import cached_camera_center

        cc = cached_camera_center(cameras, fragments.pix_to_face.device) if cameras is not None else \
            torch.zeros(1, 3, device=fragments.pix_to_face.device)
        return shade_fragments(fragments, meshes, cfg, cc)


class SoftPhongShader(_SoftShader):
    """upstream mesh/shader.py SoftPhongShader: phong_shading + softmax_rgb_blend -> RGBA, on stored
    Fragments of any faces_per_pixel (HIP: mr_shade_fragments_*); inside MeshRenderer with K = 1 and
    blur = 0 the fused one-launch render shades instead."""


class HardPhongShader(_SoftShader):
    """upstream mesh/shader.py HardPhongShader (myrenderer.py:88): phong_shading + hard_rgb_blend —
    the nearest fragment's colour, the background elsewhere, alpha = 1 where a face covers the
    pixel (PyTorch3D >= 0.5 `alpha = ~is_background`); on stored Fragments (HIP:
    mr_shade_fragments_* with MR_OUT_HARD). Gradients reach the nearest fragment's colour
    (bary, vertex positions / normals / colours, texture) only, as upstream's."""


class SoftSilhouetteShader(_SoftShader):
    """upstream mesh/shader.py SoftSilhouetteShader: sigmoid_alpha_blend -> (1, 1, 1, alpha)."""

    def __init__(self, blend_params=None):
        super().__init__(blend_params=blend_params)


class MeshRenderer(torch.nn.Module):
    """upstream mesh/renderer.py MeshRenderer: rasterizer + shader, here ONE fused launch."""

    def __init__(self, rasterizer: MeshRasterizer, shader):
        super().__init__()
        self.rasterizer = rasterizer
        self.shader = shader

    def _config(self, cameras, rs, H, W, kwargs):
        """ShadeConfig of one fused call: the shader's (and per-call) lighting / blending plus the
        rasterization settings."""
        if rs.cull_to_frustum:
            raise NotImplementedError("cull_to_frustum is not implemented on the MI355X path yet")
        cfg = _shade_config(self.shader, cameras, H, W, kwargs)
        cfg.persp = cameras.is_perspective() if rs.perspective_correct is None else bool(rs.perspective_correct)
        cfg.clip = False if rs.clip_barycentric_coords is None else bool(rs.clip_barycentric_coords)
        cfg.cull = bool(rs.cull_backfaces)
        cfg.max_faces_per_bin = rs.max_faces_per_bin
        cfg.z_clip = _z_clip_value(cameras, rs)
        return cfg

    def _soft_silhouette(self, meshes, cameras, rs, kwargs):
        """SoftSilhouetteWorld for a shared mesh, or None when the grid is one the per-view binning does not
        take (the caller then runs rasterizer + shader)."""
        from .kernels import SoftSilhouetteWorld

        H, W = rs.hw()
        persp = cameras.is_perspective() if rs.perspective_correct is None else bool(rs.perspective_correct)
        clip = rs.blur_radius > 0.0 if rs.clip_barycentric_coords is None else bool(rs.clip_barycentric_coords)
        cfg = _shade_config(self.shader, cameras, H, W, kwargs)
        R, T, intr = _views(meshes, cameras, (H, W), kwargs)
        N, Fn = R.shape[0], meshes.shared_faces().shape[0]
        # the fused pass needs the per-view binning (mr_rasterize_meshes_world's common case: <= 16,384
        # 8x8 tiles, <= 256 per side)
        from . import _lib

        tx, ty = (W + 7) // 8, (H + 7) // 8
        if not _lib.load().mr_per_view_binning(N, N * Fn, H, W):
            return None
        if N * tx * ty * 64 * int(rs.faces_per_pixel) >= 2 ** 31:  # mr_soft_silhouette_forward's slot bound
            return None
        return SoftSilhouetteWorld.apply(meshes.shared_verts(), R, T, meshes.shared_faces(), intr, N, H, W,
                                         int(rs.faces_per_pixel), float(rs.blur_radius), persp, clip,
                                         bool(rs.cull_backfaces), rs.max_faces_per_bin, _z_clip_value(cameras, rs),
                                         cfg.sigma_sil)

    def forward(self, meshes_world: Meshes, **kwargs) -> torch.Tensor:
        """upstream signature: forward(meshes_world, **kwargs) (camera_pose_optimizer.py:177)."""
        from .torch_renderer import render_mesh_batch

        meshes = meshes_world
        cameras = kwargs.get("cameras", self.rasterizer.cameras)
        if cameras is None:
            raise ValueError("Cameras must be specified either at initialization or in the forward pass")
        rs = kwargs.get("raster_settings", self.rasterizer.raster_settings)
        from .torch_renderer import textures_need_modular

        if (type(self.shader) is SoftSilhouetteShader and type(self.rasterizer) is MeshRasterizer and
                1 < int(rs.faces_per_pixel) <= 64 and meshes.is_shared() and not rs.cull_to_frustum):
            # the soft silhouette of deform_mesh_with_color.py: raster + sigmoid_alpha_blend in one pass,
            # the fragments never written (bitwise the two-step result; SoftSilhouetteWorld)
            out = self._soft_silhouette(meshes, cameras, rs, kwargs)
            if out is not None:
                return out
        if int(rs.faces_per_pixel) != 1 or float(rs.blur_radius) != 0.0 or isinstance(self.shader, HardPhongShader) or (
                isinstance(self.shader, SoftPhongShader) and textures_need_modular(meshes)):
            # soft rasterization, or a texture map that needs gradients: the HIP
            # raster, then the shader over the fragments (differentiable w.r.t. the map and uvs)
            return self.shader(self.rasterizer(meshes, **kwargs), meshes, **kwargs)
        H, W = rs.hw()
        cfg = self._config(cameras, rs, H, W, kwargs)
        cfg.sil_rgba = not cfg.want_rgb  # SoftSilhouetteShader's (1, 1, 1, alpha) straight from the kernels
        R, T, intr = _views(meshes, cameras, (H, W), kwargs)
        # specular camera position: cameras.get_camera_center() without the R/T kwargs (upstream
        # shading.py), i.e. from the camera object's own R, T
        out = render_mesh_batch(meshes, cameras, (H, W), R, T, cfg, views=(R, T, intr))
        return out["rgb"] if cfg.want_rgb else out["sil"]
