"""The C ABI library loads and exports every symbol include/mi355r.h declares; host-side
argument validation runs without a GPU (no compute calls here)."""
import ctypes
import os
import re

import pytest

from torch_renderer_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "mi355r.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mr_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        from torch_renderer_amd import _build

        _build.build()
    return _lib.load()


def test_all_header_symbols_exported(lib):
    syms = header_symbols()
    assert len(syms) >= 14
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(_lib.EXPORTED_SYMBOLS) == syms, "ctypes signature table out of sync with the header"


def test_version_and_workspace_queries(lib):
    assert lib.mr_version() == 5  # 2: mr_raster_settings_t gained clip_z / z_clip_value; 3: mr_mesh_t vnormals_out;
    # 4: mr_pose_loss_* take sil_stride (RGBA slices read in place), MR_OUT_ZBUF, quaternion kernels;
    # 5: MR_FRAG_SORTED moved to bit 10 (it shared 64 with MR_OUT_ZBUF)
    a = lib.mr_render_workspace(64, 5856, 512, 512, 0)
    b = lib.mr_render_workspace(8, 5856, 512, 512, 0)
    assert a > b > 0
    assert lib.mr_rasterize_meshes_workspace(2, 1000, 64, 64, 0) > 0
    assert lib.mr_render_backward_workspace(64, 2930, 5856, 512, 512) > 0


def test_invalid_arguments_fail_loudly_without_touching_the_gpu(lib):
    s = _lib.MrRasterSettings()
    s.H, s.W, s.faces_per_pixel, s.blur_radius = 64, 64, 129, 0.0  # K in [1, 128]
    rc = lib.mr_rasterize_meshes(None, None, None, 1, 10, ctypes.byref(s), None, None, None, None, None, 0, None)
    assert rc == 3 and b"faces_per_pixel" in lib.mr_last_error()
    with pytest.raises(NotImplementedError):
        _lib.check(rc)
    s.faces_per_pixel = 1
    s.H = 0
    rc = lib.mr_rasterize_meshes(None, None, None, 1, 10, ctypes.byref(s), None, None, None, None, None, 0, None)
    assert rc == 1 and b"image size" in lib.mr_last_error()
    s.H, s.blur_radius = 64, -1.0
    rc = lib.mr_rasterize_meshes(None, None, None, 1, 10, ctypes.byref(s), None, None, None, None, None, 0, None)
    assert rc == 1
    with pytest.raises(RuntimeError):
        _lib.check(rc)


def test_struct_layouts_match_header():
    """The ctypes mirrors have the sizes the library was compiled with (mr_struct_size)."""
    lib = _lib.load()
    assert ctypes.sizeof(_lib.MrView) == 64 == lib.mr_struct_size(0)
    assert ctypes.sizeof(_lib.MrRasterSettings) == 40 == lib.mr_struct_size(1)
    assert ctypes.sizeof(_lib.MrShadeParams) == lib.mr_struct_size(2) == 4 * (1 + 3 * 7 + 1 + 2 + 3 + 2 + 1 + 2)
    assert ctypes.sizeof(_lib.MrMesh) == lib.mr_struct_size(3)
    assert lib.mr_struct_size(9) == -1


def test_missing_library_raises(tmp_path):
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.load(str(tmp_path / "nope.so"))


def test_world_rasterizer_validation_and_workspace(lib):
    """mr_rasterize_meshes_world (MeshRasterizer.forward for an extended mesh): host-side checks
    fail with a status and a message before any device work; its workspace covers the modular
    rasterizer's plus the shared-mesh face ranges."""
    s = _lib.MrRasterSettings()
    s.H, s.W, s.faces_per_pixel, s.blur_radius = 64, 64, 1, 0.0
    ps = _lib.MrPoses(None, 0, None, 0, None, 0)
    rc = lib.mr_rasterize_meshes_world(None, 10, None, 10, ctypes.byref(ps), 2, ctypes.byref(s), None, None,
                                       None, None, None, None, None, 0, None)
    assert rc == 1 and b"NULL" in lib.mr_last_error()
    rc = lib.mr_rasterize_meshes_world(None, 10, None, 10, ctypes.byref(ps), 0, ctypes.byref(s), None, None,
                                       None, None, None, None, None, 0, None)
    assert rc == 1 and b"N must be" in lib.mr_last_error()
    s.faces_per_pixel = 0
    rc = lib.mr_rasterize_meshes_world(None, 10, None, 10, ctypes.byref(ps), 2, ctypes.byref(s), None, None,
                                       None, None, None, None, None, 0, None)
    assert rc == 3
    w = lib.mr_rasterize_meshes_world_workspace(64, 5856, 512, 512, 0)
    assert w >= lib.mr_rasterize_meshes_workspace(64, 64 * 5856, 512, 512, 0) + 16 * 64
    assert ctypes.sizeof(_lib.MrPoses) == ctypes.sizeof(_lib.MrOpencvPoses) == 48


def header_enum(names_prefix=("MR_OUT_", "MR_GRAD_", "MR_FRAG_", "MR_SREC_")):
    src = open(os.path.join(ROOT, "include", "mi355r.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return {k: int(v) for k, v in re.findall(r"\b(MR_[A-Z_0-9]+)\s*=\s*(\d+)", src) if k.startswith(names_prefix)}


def test_out_flags_are_distinct_bits():
    """Every out_flags value the header publishes is its own bit, none overlaps another or the ShadeRec
    slot field (bits MR_SREC_SLOT_SHIFT .. +1), and the Python binding uses the header's values."""
    vals = header_enum()
    shift = vals.pop("MR_SREC_SLOT_SHIFT")
    assert shift == _lib.MR_SREC_SLOT_SHIFT == 8
    slot_bits = 3 << shift
    seen = 0
    for name, v in vals.items():
        assert v > 0 and v & (v - 1) == 0, (name, v)
        assert not (v & seen), f"{name} = {v} overlaps another flag"
        assert not (v & slot_bits), f"{name} = {v} overlaps the ShadeRec slot bits"
        seen |= v
        assert getattr(_lib, name) == v, name
    assert {"MR_OUT_ZBUF", "MR_FRAG_SORTED", "MR_GRAD_ROWS_CLEARED"} <= set(vals)
