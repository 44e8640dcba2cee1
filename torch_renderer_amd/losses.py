"""Fused pose-optimiser loss.

``pose_loss`` is camera_pose_optimizer.py:257-276 ``Model.calc_loss`` in three HIP launches forward
(mask count, one pass that sums the loss AND writes its gradients for dL/dtotal = 1, final reduction)
and one near-empty rescale in the backward (``mr_pose_loss_*``), instead of ~15 torch elementwise /
reduction kernels forward and as many backward:

* ``sil_loss   = torch.nn.L1Loss()(silhouette, mask.float())``
* ``hloss      = torch.nn.HuberLoss(delta=0.05)(depth[mask], depth_ref[mask])``
* ``color_loss = torch.nn.MSELoss()(color, rgb_ref)``
* ``total      = sil_loss + hloss + 0.01 * color_loss``

``color`` may be the RGBA view ``image[..., :3]`` and ``silhouette`` the view ``sil_image[..., 3]``
the reference passes (camera_pose_optimizer.py:248,250): both are read in place, and their gradients
are written by the loss's backward straight in the RGBA images' layout (zero in the channels the
views leave out) and handed to autograd for the images themselves — what the slices' backward
would produce, without its zero-filled (N,H,W,4) buffer and strided copy per image. The reductions
run in a fixed order (deterministic); the values agree with torch's to float32 rounding of a
different summation order. An empty mask gives NaN, like torch's mean of nothing.
"""
from __future__ import annotations

import torch

from . import _lib
from .kernels import _require_cuda


def _rgba_base(t: torch.Tensor, channels):
    """The dense float32 (..., 4) tensor `t` is the slice ``base[..., channels]`` of (a slice object
    or an int channel), or None."""
    b = t._base
    if b is None or b.dtype != torch.float32 or t.dtype != torch.float32 or b.dim() < 2 or b.shape[-1] != 4 \
            or not b.is_contiguous() or t.device != b.device:
        return None
    if isinstance(channels, int):
        ok = (tuple(t.shape) == tuple(b.shape[:-1]) and tuple(t.stride()) == tuple(b.stride()[:-1]) and
              t.storage_offset() == b.storage_offset() + channels)
    else:
        ok = (tuple(t.shape) == tuple(b.shape[:-1]) + (3,) and tuple(t.stride()) == tuple(b.stride()) and
              t.storage_offset() == b.storage_offset())
    return b if ok else None


def pose_loss(depth, silhouette, color, mask, depth_ref, rgb_ref, delta: float = 0.05, w_color: float = 0.01,
              return_terms: bool = False):
    """camera_pose_optimizer.py:257-276 calc_loss on the GPU. Returns the total loss (0-dim,
    differentiable w.r.t. depth, silhouette and color), or (total, (sil_loss, hloss, color_loss))
    with ``return_terms`` (the terms the reference logs; not differentiable)."""
    _require_cuda(depth, silhouette, color, mask, depth_ref, rgb_ref)
    sb = _rgba_base(silhouette, 3)
    cb = _rgba_base(color, slice(0, 3))
    # the autograd node is C++ (_mr_torch.pose_loss, csrc/mr_torch.cpp): forward and backward without Python
    total, terms = _lib.torch_ext().pose_loss(depth, silhouette if sb is None else sb, color if cb is None else cb,
                                              mask, depth_ref, rgb_ref, float(delta), float(w_color), sb is not None,
                                              cb is not None)
    if return_terms:
        return total, (terms[0], terms[1], terms[2])
    return total
