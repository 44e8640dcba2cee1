"""Round-4 host logic on CPU (no GPU calls): the host-path caches added for the eager caller loops must
never serve stale values.

* camera caches (cached_ndc_affine / cached_camera_center, keyed by _param_key): an in-place edit of a camera
  tensor, a replaced tensor attribute and a new tensor attribute each produce a new key;
* ShadeConfig's cached ctypes structs: every call returns an independent copy (callers OR flags into it), and a
  changed field gives a different struct;
* the workspace-size cache returns what the library computes for the same arguments.
"""
import ctypes

import torch

from torch_renderer_amd import _lib
from torch_renderer_amd import kernels as Kn
from torch_renderer_amd.cameras import FoVPerspectiveCameras, PerspectiveCameras, _param_key, cached_ndc_affine


def test_camera_key_tracks_edits_replacements_and_new_attributes():
    cams = PerspectiveCameras(focal_length=2.0, R=torch.eye(3)[None], T=torch.zeros(1, 3))
    k0 = _param_key(cams)
    assert _param_key(cams) == k0
    cams.T[0, 2] = 5.0  # in-place edit: version bump
    k1 = _param_key(cams)
    assert k1 != k0
    cams.fx = torch.tensor([3.0])  # replaced tensor attribute
    k2 = _param_key(cams)
    assert k2 != k1
    cams.extra = torch.zeros(2)  # new tensor attribute
    k3 = _param_key(cams)
    assert k3 != k2 and len(k3) == len(k2) + 2  # its (storage, version) joins the key
    cams.note = "x"  # any assignment bumps the generation
    assert _param_key(cams) != k3
    c0 = cams[0]  # a copy starts its own generation and key
    kc = _param_key(c0)
    assert _param_key(c0) == kc
    c0.T[0, 0] = 1.0
    assert _param_key(c0) != kc
    k4 = _param_key(cams)
    del cams.extra  # a removed attribute leaves the key (and is not looked up again)
    assert _param_key(cams) != k4 and len(_param_key(cams)) == len(k4) - 2


def test_cached_ndc_affine_follows_the_focal_length():
    cams = PerspectiveCameras(focal_length=2.0)
    a = cached_ndc_affine(cams, (64, 64), "cpu").clone()
    cams.fx.mul_(2.0)  # in place
    b = cached_ndc_affine(cams, (64, 64), "cpu")
    assert not torch.equal(a, b) and b[0, 0].item() == 2 * a[0, 0].item()
    fov = FoVPerspectiveCameras(fov=60.0)
    c = cached_ndc_affine(fov, (64, 64), "cpu").clone()
    fov.fov = 30.0  # a float field (upstream reads it on every call)
    d = cached_ndc_affine(fov, (64, 64), "cpu")
    assert torch.equal(d, fov.ndc_affine((64, 64))) and not torch.equal(c, d)


def test_shade_config_struct_cache_returns_independent_copies():
    cfg = Kn.ShadeConfig(H=32, W=32)
    a = cfg.shade_struct()
    a.out_flags |= 1 << _lib.MR_SREC_SLOT_SHIFT
    b = cfg.shade_struct()
    assert b.out_flags != a.out_flags  # the cached struct was not modified through the copy
    cfg2 = Kn.ShadeConfig(H=32, W=32, want_rgb=False)
    assert cfg2.shade_struct().out_flags != b.out_flags
    r1, r2 = cfg.raster_struct(), cfg.raster_struct()
    r1.H = 7
    assert r2.H == 32 and ctypes.addressof(r1) != ctypes.addressof(r2)


def test_workspace_size_cache_matches_the_library():
    L = _lib.load()
    args = (4, 100, 64, 48, 0)
    assert Kn._ws_size(L.mr_render_workspace, *args) == int(L.mr_render_workspace(*args))
    assert Kn._ws_size(L.mr_render_workspace, *args) == int(L.mr_render_workspace(*args))  # (cached)
    args2 = (8, 100, 64, 48, 0)
    assert Kn._ws_size(L.mr_render_workspace, *args2) == int(L.mr_render_workspace(*args2))
