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

import ctypes

import torch

from . import _lib
from ._lib import check
from .kernels import _require_cuda


def _vp(t):
    return ctypes.c_void_p(t.data_ptr())


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


class PoseLoss(torch.autograd.Function):
    """sil_in / color_in: the silhouette (npix) and colour (npix, 3) tensors, or (sil_rgba / col_rgba
    set) the RGBA images they are the [..., 3] / [..., :3] slices of, whose gradients are returned."""

    @staticmethod
    def forward(ctx, depth, sil_in, color_in, mask, depth_ref, rgb_ref, delta, w_color, sil_rgba, col_rgba):
        _require_cuda(depth, sil_in, color_in, mask, depth_ref, rgb_ref)
        if rgb_ref.shape[-1] != 3 or color_in.shape[-1] != (4 if col_rgba else 3):
            raise ValueError("color and rgb_ref must end in 3 channels")
        npix = depth.numel()
        for name, t, k in (("silhouette", sil_in, 4 * npix if sil_rgba else npix), ("mask", mask, npix),
                           ("depth_ref", depth_ref, npix), ("color", color_in, (4 if col_rgba else 3) * npix),
                           ("rgb_ref", rgb_ref, 3 * npix)):
            if t.numel() != k:
                raise ValueError(f"pose_loss: {name} has {t.numel()} elements, expected {k} (no broadcasting)")
        L = _lib.load()
        dev = depth.device
        d = depth.detach().float().contiguous()
        if sil_rgba:  # channel 3 of the RGBA image, read in place
            s, s_stride, s_ptr = sil_in.detach(), 4, ctypes.c_void_p(sil_in.data_ptr() + 12)
        else:
            s = sil_in.detach().float().contiguous()
            s_stride, s_ptr = 1, _vp(s)
        if col_rgba:
            c, stride = color_in.detach(), 4
        else:  # (an RGBA slice pose_loss recognised comes as its image instead)
            c, stride = color_in.detach().float().contiguous(), 3
        m = mask.detach().to(torch.bool).contiguous().view(torch.uint8)
        dr = depth_ref.detach().float().contiguous()
        rr = rgb_ref.detach().float().contiguous()
        wsb = int(L.mr_pose_loss_workspace(npix))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        total = torch.empty((), device=dev)
        terms = torch.empty(3, device=dev)
        ctx.pre = None
        gd = gs = gc = None
        if any(ctx.needs_input_grad[:3]):
            # one pass: the gradients for dL/dtotal = 1 are written with the forward (the loss is linear
            # in dL/dtotal); the first backward rescales them in place unless dL/dtotal is 1
            gd = torch.empty_like(d)
            gs = torch.empty((npix, s_stride), device=dev)
            gc = torch.empty((npix, stride), device=dev)
            ctx.pre = (gd, gs, gc)
        check(L.mr_pose_loss_forward_grad(_vp(d), s_ptr, s_stride, _vp(c), stride, _vp(m), _vp(dr), _vp(rr), npix,
                                          float(delta), float(w_color), _vp(total), _vp(terms), _vp(ws), wsb,
                                          _lib.ptr(gd), _lib.ptr(gs), _lib.ptr(gc), _lib.stream_handle(dev)))
        ctx.save_for_backward(d, s, c, m, dr, rr, ws)
        ctx.stride, ctx.s_stride, ctx.npix, ctx.delta, ctx.w_color = stride, s_stride, npix, float(delta), float(w_color)
        ctx.shapes = (depth.shape, sil_in.shape, color_in.shape)
        ctx.mark_non_differentiable(terms)
        return total, terms

    @staticmethod
    def backward(ctx, g_total, g_terms):
        L = _lib.load()
        sd, ss, sc = ctx.shapes
        if ctx.pre is not None:  # the forward's gradients, scaled by dL/dtotal (first backward only)
            gd, gs, gc = ctx.pre
            ctx.pre = None
            dev = gd.device
            g = (g_total if g_total is not None else torch.zeros((), device=dev)).float().contiguous().reshape(1)
            check(L.mr_pose_loss_scale(_vp(g), ctx.npix, ctx.s_stride, ctx.stride, _vp(gd), _vp(gs), _vp(gc),
                                       _lib.stream_handle(dev)))
            return gd.reshape(sd), gs.reshape(ss), gc.reshape(sc), None, None, None, None, None, None, None
        d, s, c, m, dr, rr, ws = ctx.saved_tensors
        dev = d.device
        g = (g_total if g_total is not None else torch.zeros((), device=dev)).float().contiguous().reshape(1)
        gd = torch.empty_like(d)
        gs = torch.empty((ctx.npix, ctx.s_stride), device=dev)  # (npix, 4): the RGBA image's gradient
        gc = torch.empty((ctx.npix, ctx.stride), device=dev)
        s_ptr = ctypes.c_void_p(s.data_ptr() + 12) if ctx.s_stride == 4 else _vp(s)
        check(L.mr_pose_loss_backward(_vp(d), s_ptr, ctx.s_stride, _vp(c), ctx.stride, _vp(m), _vp(dr), _vp(rr),
                                      ctx.npix, ctx.delta, ctx.w_color, _vp(g), _vp(ws), _vp(gd), _vp(gs), _vp(gc),
                                      _lib.stream_handle(dev)))
        return gd.reshape(sd), gs.reshape(ss), gc.reshape(sc), None, None, None, None, None, None, None


def pose_loss(depth, silhouette, color, mask, depth_ref, rgb_ref, delta: float = 0.05, w_color: float = 0.01,
              return_terms: bool = False):
    """camera_pose_optimizer.py:257-276 calc_loss on the GPU. Returns the total loss (0-dim,
    differentiable w.r.t. depth, silhouette and color), or (total, (sil_loss, hloss, color_loss))
    with ``return_terms`` (the terms the reference logs; not differentiable)."""
    sb = _rgba_base(silhouette, 3)
    cb = _rgba_base(color, slice(0, 3))
    total, terms = PoseLoss.apply(depth, silhouette if sb is None else sb, color if cb is None else cb, mask,
                                  depth_ref, rgb_ref, delta, w_color, sb is not None, cb is not None)
    if return_terms:
        return total, (terms[0], terms[1], terms[2])
    return total
