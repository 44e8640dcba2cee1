"""ctypes binding of the C ABI in ``include/mi355r.h`` (``libmi355r.so``).

The library is the product: there is no CPU or PyTorch fallback. If the shared
object is missing or fails to load, importing a GPU entry point raises
``RuntimeError`` (build it with ``python -m torch_renderer_amd._build`` or
``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  -- must be imported first: the .so shares torch's HIP runtime

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmi355r.so")

c_float_p = ctypes.POINTER(ctypes.c_float)
c_i64_p = ctypes.POINTER(ctypes.c_int64)
c_i32_p = ctypes.POINTER(ctypes.c_int32)

MR_OUT_DEPTH = 1
MR_OUT_SIL = 2
MR_OUT_RGB = 4
MR_OUT_HARD = 8  # hard_rgb_blend (HardPhongShader), fragment-shader path only
MR_OUT_SIL_RGBA = 32  # silhouette as (N,H,W,4) RGBA (1, 1, 1, alpha), fused render path
MR_OUT_ZBUF = 64  # depth output = MeshRasterizer's zbuf[..., 0] (background -1), fused render path
MR_SREC_SLOT_SHIFT = 8  # out_flags bits 8-9: the workspace's ShadeRec slot (mr_render_reshade)
MR_FRAG_SORTED = 1024  # mr_shade_fragments_*: empty slots follow the filled ones (this library's rasterizer)
MR_GRAD_ROWS_CLEARED = 16  # mr_render_backward: first backward over a forward (its face totals are still clear)


class MrView(ctypes.Structure):
    _fields_ = [("R", ctypes.c_float * 9), ("T", ctypes.c_float * 3), ("ax", ctypes.c_float),
                ("bx", ctypes.c_float), ("ay", ctypes.c_float), ("by", ctypes.c_float)]


class MrRasterSettings(ctypes.Structure):
    _fields_ = [("H", ctypes.c_int32), ("W", ctypes.c_int32), ("faces_per_pixel", ctypes.c_int32),
                ("blur_radius", ctypes.c_float), ("perspective_correct", ctypes.c_int32),
                ("clip_barycentric_coords", ctypes.c_int32), ("cull_backfaces", ctypes.c_int32),
                ("max_faces_per_bin", ctypes.c_int32), ("clip_z", ctypes.c_int32), ("z_clip_value", ctypes.c_float)]


F3 = ctypes.c_float * 3


class MrShadeParams(ctypes.Structure):
    _fields_ = [("light_kind", ctypes.c_int32), ("light_location", F3), ("light_ambient", F3),
                ("light_diffuse", F3), ("light_specular", F3), ("mat_ambient", F3), ("mat_diffuse", F3),
                ("mat_specular", F3), ("shininess", ctypes.c_float), ("sigma_rgb", ctypes.c_float),
                ("gamma", ctypes.c_float), ("background", F3), ("znear", ctypes.c_float),
                ("zfar", ctypes.c_float), ("sigma_sil", ctypes.c_float), ("out_flags", ctypes.c_int32),
                ("rgb_channels", ctypes.c_int32)]


class MrOpencvPoses(ctypes.Structure):
    _fields_ = [("R", ctypes.c_void_p), ("R_stride", ctypes.c_int64), ("t", ctypes.c_void_p),
                ("t_stride", ctypes.c_int64), ("intr", ctypes.c_void_p), ("intr_stride", ctypes.c_int64)]


class MrPoses(ctypes.Structure):
    _fields_ = [("R", ctypes.c_void_p), ("R_stride", ctypes.c_int64), ("T", ctypes.c_void_p),
                ("T_stride", ctypes.c_int64), ("intr", ctypes.c_void_p), ("intr_stride", ctypes.c_int64)]


class MrMesh(ctypes.Structure):
    _fields_ = [("verts", ctypes.c_void_p), ("V", ctypes.c_int64), ("faces", ctypes.c_void_p),
                ("F", ctypes.c_int64), ("vadj_ptr", ctypes.c_void_p), ("vadj", ctypes.c_void_p),
                ("vnormals", ctypes.c_void_p), ("tex_kind", ctypes.c_int32), ("vcolors", ctypes.c_void_p),
                ("verts_uvs", ctypes.c_void_p), ("faces_uvs", ctypes.c_void_p), ("tex_rgba", ctypes.c_void_p),
                ("tex_h", ctypes.c_int32), ("tex_w", ctypes.c_int32), ("vnormals_out", ctypes.c_void_p),
                ("vraw_out", ctypes.c_void_p), ("tex_u8", ctypes.c_void_p), ("tex_lut", ctypes.c_void_p),
                ("view_face_first", ctypes.c_void_p), ("view_face_count", ctypes.c_void_p),
                ("max_view_faces", ctypes.c_int64)]


# (name, restype, argtypes) — mirrors include/mi355r.h
_VP = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_SZ = ctypes.c_size_t
_SIGS = [
    ("mr_last_error", ctypes.c_char_p, []),
    ("mr_version", _I32, []),
    ("mr_struct_size", _I32, [_I32]),
    ("mr_rasterize_meshes_workspace", _SZ, [_I64, _I64, _I32, _I32, _I32]),
    ("mr_rasterize_meshes", _I32, [_VP, _VP, _VP, _I64, _I64, ctypes.POINTER(MrRasterSettings), _VP, _VP, _VP,
                                   _VP, _VP, _SZ, _VP]),
    ("mr_rasterize_meshes_backward", _I32, [_VP, _VP, _VP, _VP, _VP, _I64, _I64, ctypes.POINTER(MrRasterSettings),
                                            _VP, _VP]),
    ("mr_rasterize_meshes_world_workspace", _SZ, [_I64, _I64, _I32, _I32, _I32]),
    ("mr_rasterize_meshes_world", _I32, [_VP, _I64, _VP, _I64, ctypes.POINTER(MrPoses), _I64,
                                         ctypes.POINTER(MrRasterSettings), _VP, _VP, _VP, _VP, _VP, _VP, _VP, _SZ,
                                         _VP]),
    ("mr_binning_background_pixels", _I64, [_I64, _I64, _I32, _I32, _I32]),
    ("mr_soft_silhouette_workspace", _SZ, [_I64, _I64, _I32, _I32, _I32, _I32]),
    ("mr_soft_silhouette_forward", _I32, [_VP, _I64, _VP, _I64, ctypes.POINTER(MrPoses), _I64,
                                          ctypes.POINTER(MrRasterSettings), ctypes.c_float, _VP, _VP, _VP, _VP, _SZ,
                                          _VP]),
    ("mr_soft_silhouette_backward", _I32, [_VP, _I64, _I64, ctypes.POINTER(MrRasterSettings), ctypes.c_float, _VP,
                                           _VP, _VP, _VP]),
    ("mr_project_faces", _I32, [_VP, _I64, _VP, _I64, _VP, _I64, _VP, _VP]),
    ("mr_project_faces_meshes", _I32, [_VP, _I64, _VP, _I64, _VP, _I64, _VP, _I64, _VP, _VP]),
    ("mr_project_faces_meshes_backward", _I32, [_VP, _I64, _VP, _I64, _VP, _VP, _VP, _I64, _VP, _I64, _VP, _VP, _VP,
                                                _VP]),
    ("mr_views_from_opencv", _I32, [_VP, _I64, _VP, _I64, _VP, _I64, _I64, _VP, _VP]),
    ("mr_view_grads_to_opencv", _I32, [_VP, _I64, _VP, _VP, _VP]),
    ("mr_project_faces_backward", _I32, [_VP, _I64, _VP, _I64, _VP, _VP, _VP, _I64, _VP, _VP, _VP, _VP]),
    ("mr_vertex_normals", _I32, [_VP, _I64, _VP, _I64, _VP, _VP, _VP, _VP, _VP]),
    ("mr_render_workspace", _SZ, [_I64, _I64, _I32, _I32, _I32]),
    ("mr_render_workspace_meshes", _SZ, [_I64, _I64, _I32, _I32, _I32]),
    ("mr_render_forward", _I32, [ctypes.POINTER(MrMesh), _VP, _I64, _VP, _I64, ctypes.POINTER(MrRasterSettings),
                                 ctypes.POINTER(MrShadeParams), _VP, _VP, _VP, _VP, _VP, _SZ, _VP]),
    ("mr_render_forward_opencv", _I32, [ctypes.POINTER(MrMesh), ctypes.POINTER(MrOpencvPoses), _VP, _I64, _VP, _I64,
                                        ctypes.POINTER(MrRasterSettings), ctypes.POINTER(MrShadeParams), _VP, _VP,
                                        _VP, _VP, _VP, _SZ, _VP]),
    ("mr_render_forward_poses", _I32, [ctypes.POINTER(MrMesh), ctypes.POINTER(MrPoses), _VP, _I64, _VP, _I64,
                                       ctypes.POINTER(MrRasterSettings), ctypes.POINTER(MrShadeParams), _VP, _VP,
                                       _VP, _VP, _VP, _SZ, _VP]),
    ("mr_render_backward_workspace", _SZ, [_I64, _I64, _I64, _I32, _I32]),
    ("mr_render_backward", _I32, [ctypes.POINTER(MrMesh), _VP, _VP, _I64, _VP, _I64,
                                  ctypes.POINTER(MrRasterSettings), ctypes.POINTER(MrShadeParams), _VP, _VP, _VP,
                                  _VP, _VP, _SZ, _VP, _VP, _VP, _VP]),
    ("mr_render_backward_opencv", _I32, [ctypes.POINTER(MrMesh), _VP, _VP, _I64, _VP, _I64,
                                         ctypes.POINTER(MrRasterSettings), ctypes.POINTER(MrShadeParams), _VP, _VP,
                                         _VP, _VP, _VP, _SZ, _VP, _VP, _VP, _VP, _VP]),
    ("mr_shade_fragments_workspace", _SZ, [_I64]),
    ("mr_shade_fragments_forward", _I32, [ctypes.POINTER(MrMesh), _VP, _VP, _VP, _VP, _I64, _I32, _I32, _I32, _VP,
                                          _I64, ctypes.POINTER(MrShadeParams), _VP, _VP, _SZ, _VP]),
    ("mr_shade_fragments_backward_workspace", _SZ, [_I64, _I64]),
    ("mr_shade_fragments_backward", _I32, [ctypes.POINTER(MrMesh), _VP, _VP, _VP, _VP, _VP, _I64, _I32, _I32, _I32,
                                           _VP, _I64, ctypes.POINTER(MrShadeParams), _VP, _VP, _VP, _SZ, _VP, _VP,
                                           _VP, _VP, _VP, _VP, _VP, _I64, _VP]),
    ("mr_pose_loss_workspace", _SZ, [_I64]),
    ("mr_pose_loss_forward", _I32, [_VP, _VP, _I64, _VP, _I64, _VP, _VP, _VP, _I64, ctypes.c_float, ctypes.c_float,
                                    _VP, _VP, _SZ, _VP]),
    ("mr_pose_loss_backward", _I32, [_VP, _VP, _I64, _VP, _I64, _VP, _VP, _VP, _I64, ctypes.c_float, ctypes.c_float,
                                     _VP, _VP, _VP, _VP, _VP, _VP]),
    ("mr_pose_loss_forward_grad", _I32, [_VP, _VP, _I64, _VP, _I64, _VP, _VP, _VP, _I64, ctypes.c_float,
                                         ctypes.c_float, _VP, _VP, _VP, _SZ, _VP, _VP, _VP, _VP]),
    ("mr_pose_loss_scale", _I32, [_VP, _I64, _I64, _I64, _VP, _VP, _VP, _VP]),
    ("mr_quaternion_to_matrix", _I32, [_VP, _I64, _I64, _VP, _VP]),
    ("mr_quaternion_to_matrix_backward", _I32, [_VP, _I64, _VP, _I64, _VP, _VP]),
    ("mr_workspace_stats", _I32, [_VP, _I64, _I64, _I32, _I32, _I32, _VP, _VP]),
    ("mr_workspace_counters", _I32, [_VP, _I64, _I64, _I32, _I32, _I32, _VP, _VP]),
    ("mr_per_view_binning", _I32, [_I64, _I64, _I32, _I32]),
    ("mr_render_reshade", _I32, [ctypes.POINTER(MrMesh), _VP, _I64, _VP, _I64, ctypes.POINTER(MrRasterSettings),
                                 ctypes.POINTER(MrShadeParams), _VP, _VP, _VP, _VP, _VP, _SZ, _VP]),
    ("mr_timing_enable", _I32, [_I32]),
    ("mr_timing_read", _I32, [_VP, _VP, _I32]),
    ("mr_timing_kernel_name", ctypes.c_char_p, [_I32]),
    ("mr_timing_kernel_count", _I32, []),
]

EXPORTED_SYMBOLS = [s[0] for s in _SIGS]

_lib = None
_lock = threading.Lock()


def load(path: str | None = None) -> ctypes.CDLL:
    """Load (once) and return the library. Raises RuntimeError if it is missing."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or os.environ.get("MI355R_LIB") or LIB_PATH  # override: experiment builds
        if not os.path.exists(p):
            raise RuntimeError(
                f"mi355r: native library not found at {p}. Build it first "
                "(python -m torch_renderer_amd._build). There is no CPU fallback.")
        lib = ctypes.CDLL(p)
        for name, res, args in _SIGS:
            fn = getattr(lib, name, None)
            if fn is None and path is None and not os.environ.get("MI355R_LIB"):
                raise RuntimeError(f"mi355r: {p} does not export {name} (stale build?)")
            if fn is None:  # an experiment build older than the current ABI
                continue
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


_EXT = None
_EXT_FNS = ("mr_last_error", "mr_render_workspace", "mr_render_workspace_meshes", "mr_render_reshade",
            "mr_render_forward_opencv", "mr_render_forward_poses", "mr_render_backward_workspace",
            "mr_render_backward", "mr_render_backward_opencv", "mr_pose_loss_workspace", "mr_pose_loss_forward_grad",
            "mr_pose_loss_scale", "mr_pose_loss_backward", "mr_quaternion_to_matrix", "mr_quaternion_to_matrix_backward")


def torch_ext():
    """The fused render's autograd node in C++ (``_mr_torch.so``, csrc/mr_torch.cpp), bound to the C ABI
    functions of the library ``load()`` returned. Raises RuntimeError if it is missing (no fallback)."""
    global _EXT
    with _lock:
        if _EXT is not None:
            return _EXT
    path = os.path.join(_HERE, "_mr_torch.so")
    if not os.path.exists(path):
        raise RuntimeError(f"mi355r: {path} not found. Build it first (python -m torch_renderer_amd._build).")
    import importlib.util

    spec = importlib.util.spec_from_file_location("_mr_torch", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    import torch

    built = getattr(mod, "built_with_torch", "unknown")
    abi = getattr(mod, "built_with_cxx11_abi", None)
    if built != torch.__version__ or (abi is not None and bool(abi) != bool(torch._C._GLIBCXX_USE_CXX11_ABI)):
        raise RuntimeError(f"mi355r: {path} was built against torch {built} (cxx11 ABI {abi}), this process runs "
                           f"torch {torch.__version__} (cxx11 ABI {torch._C._GLIBCXX_USE_CXX11_ABI}): rebuild it "
                           "(python -m torch_renderer_amd._build)")
    lib = load()
    mod.init({name: ctypes.cast(getattr(lib, name), ctypes.c_void_p).value for name in _EXT_FNS})
    with _lock:
        _EXT = mod
    return mod


def check(rc: int) -> None:
    if rc != 0:
        msg = load().mr_last_error().decode(errors="replace")
        if rc == 3:
            raise NotImplementedError(f"mi355r: {msg}")
        raise RuntimeError(f"mi355r error {rc}: {msg}")


def ptr(t):
    """Device (or host) pointer of a contiguous tensor, or None."""
    if t is None:
        return None
    assert t.is_contiguous(), "mi355r: tensors passed across the C ABI must be contiguous"
    return ctypes.c_void_p(t.data_ptr())


def strided_ptr(t):
    """Pointer of a tensor whose layout the callee takes as explicit strides (e.g. a broadcast
    view with batch stride 0)."""
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    """The current HIP stream of `device` (torch.device, index or None: the current device) as a handle:
    the raw stream pointer, without building a torch Stream object per launch."""
    if isinstance(device, torch.device):
        idx = device.index if device.index is not None else torch.cuda.current_device()
    elif isinstance(device, int):
        idx = device
    else:
        idx = torch.cuda.current_device()
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(idx))


def timing_enable(on: bool = True) -> None:
    check(load().mr_timing_enable(1 if on else 0))


def timing_read() -> dict:
    """{kernel name: (launches, total_ms)} for launches recorded since timing_enable(True)."""
    L = load()
    n = L.mr_timing_kernel_count()
    launches = (ctypes.c_int32 * n)()
    total = (ctypes.c_double * n)()
    check(L.mr_timing_read(ctypes.cast(launches, ctypes.c_void_p), ctypes.cast(total, ctypes.c_void_p), n))
    return {L.mr_timing_kernel_name(k).decode(): (launches[k], total[k]) for k in range(n) if launches[k]}
