"""Fused pose-optimiser loss.

``pose_loss`` is camera_pose_optimizer.py:257-276 ``Model.calc_loss`` in two HIP launches forward
and one backward (``mr_pose_loss_*``), instead of ~15 torch elementwise / reduction kernels:

* ``sil_loss   = torch.nn.L1Loss()(silhouette, mask.float())``
* ``hloss      = torch.nn.HuberLoss(delta=0.05)(depth[mask], depth_ref[mask])``
* ``color_loss = torch.nn.MSELoss()(color, rgb_ref)``
* ``total      = sil_loss + hloss + 0.01 * color_loss``

``color`` may be the RGBA view ``image[..., :3]`` the reference passes (read in place, no copy).
The reductions run in a fixed order (deterministic); the values agree with torch's to float32
rounding of a different summation order. An empty mask gives NaN, like torch's mean of nothing.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import check
from .kernels import _require_cuda


def _vp(t):
    return ctypes.c_void_p(t.data_ptr())


def _color_arg(color: torch.Tensor):
    """(tensor to read, floats between consecutive pixels): an RGBA view ``x[..., :3]`` of a dense
    (..., C) tensor is read in place with stride C; anything else is made contiguous (stride 3)."""
    c = color.detach()
    if c.dtype == torch.float32 and c.dim() >= 2 and c.stride(-1) == 1 and c.stride(-2) >= 3:
        st = c.stride(-2)
        expect = st
        ok = True
        for i in range(c.dim() - 2, -1, -1):
            if c.size(i) > 1 and c.stride(i) != expect:
                ok = False
                break
            expect *= c.size(i)
        if ok:
            return c, st
    return c.float().contiguous(), 3


class PoseLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, depth, silhouette, color, mask, depth_ref, rgb_ref, delta, w_color):
        _require_cuda(depth, silhouette, color, mask, depth_ref, rgb_ref)
        if color.shape[-1] != 3 or rgb_ref.shape[-1] != 3:
            raise ValueError("color and rgb_ref must end in 3 channels")
        npix = depth.numel()
        for name, t, k in (("silhouette", silhouette, npix), ("mask", mask, npix), ("depth_ref", depth_ref, npix),
                           ("color", color, 3 * npix), ("rgb_ref", rgb_ref, 3 * npix)):
            if t.numel() != k:
                raise ValueError(f"pose_loss: {name} has {t.numel()} elements, expected {k} (no broadcasting)")
        L = _lib.load()
        dev = depth.device
        d = depth.detach().float().contiguous()
        s = silhouette.detach().float().contiguous()
        c, stride = _color_arg(color)
        m = mask.detach().to(torch.bool).contiguous().view(torch.uint8)
        dr = depth_ref.detach().float().contiguous()
        rr = rgb_ref.detach().float().contiguous()
        wsb = int(L.mr_pose_loss_workspace(npix))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        out = torch.empty(4, device=dev)
        stream = _lib.stream_handle(dev)
        check(L.mr_pose_loss_forward(_vp(d), _vp(s), _vp(c), stride, _vp(m), _vp(dr), _vp(rr), npix,
                                     float(delta), float(w_color), _vp(out), _vp(ws), wsb, stream))
        ctx.save_for_backward(d, s, c, m, dr, rr, ws)
        ctx.stride, ctx.npix, ctx.delta, ctx.w_color = stride, npix, float(delta), float(w_color)
        ctx.shapes = (depth.shape, silhouette.shape, color.shape)
        terms = out[1:].clone()
        ctx.mark_non_differentiable(terms)
        return out[0].clone(), terms

    @staticmethod
    def backward(ctx, g_total, g_terms):
        d, s, c, m, dr, rr, ws = ctx.saved_tensors
        L = _lib.load()
        dev = d.device
        g = (g_total if g_total is not None else torch.zeros((), device=dev)).float().contiguous().reshape(1)
        gd = torch.empty_like(d)
        gs = torch.empty_like(s)
        gc = torch.empty((ctx.npix, 3), device=dev)
        check(L.mr_pose_loss_backward(_vp(d), _vp(s), _vp(c), ctx.stride, _vp(m), _vp(dr), _vp(rr), ctx.npix,
                                      ctx.delta, ctx.w_color, _vp(g), _vp(ws), _vp(gd), _vp(gs), _vp(gc),
                                      _lib.stream_handle(dev)))
        sd, ss, sc = ctx.shapes
        return gd.reshape(sd), gs.reshape(ss), gc.reshape(sc), None, None, None, None, None


def pose_loss(depth, silhouette, color, mask, depth_ref, rgb_ref, delta: float = 0.05, w_color: float = 0.01,
              return_terms: bool = False):
    """camera_pose_optimizer.py:257-276 calc_loss on the GPU. Returns the total loss (0-dim,
    differentiable w.r.t. depth, silhouette and color), or (total, (sil_loss, hloss, color_loss))
    with ``return_terms`` (the terms the reference logs; not differentiable)."""
    total, terms = PoseLoss.apply(depth, silhouette, color, mask, depth_ref, rgb_ref, delta, w_color)
    if return_terms:
        return total, (terms[0], terms[1], terms[2])
    return total
