"""Fused fit-loop losses on the HIP device (the caller's side of the render op).

``l1_loss(a, b, c=None, d=None, w2=0.0)`` = ``mean|a - b| + w2 * mean|c - d|``: the photometric L1
plus the weighted silhouette L1 of python/fit_multiview_stub.py:292-299, as one forward reduction
(k_l1_partial + k_l1_final) and one backward kernel (k_l1_grad) in libgr_hip.so instead of torch's
chain of sub / abs / mean / mul / add launches and their backward.  Same value and gradient as the
torch expression up to float32 summation order (tests/test_losses_gpu.py); deterministic.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

try:
    from . import _native
except ImportError:  # pragma: no cover
    import _native  # type: ignore


def _stream(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


class _L1Loss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, c, d, w2):
        L = _native.lib()
        n1 = a.numel()
        n2 = 0 if c is None else c.numel()
        loss = torch.empty((), dtype=torch.float32, device=a.device)
        ws = torch.empty((int(L.gr_l1_loss_ws_bytes()),), dtype=torch.uint8, device=a.device)
        _native.check(L.gr_l1_loss_fwd(_native.ptr(a), _native.ptr(b), n1, _native.ptr(c), _native.ptr(d), n2,
                                       ctypes.c_float(w2), _native.ptr(loss), _native.ptr(ws), ws.numel(), _stream(a)),
                      "gr_l1_loss_fwd")
        ctx.save_for_backward(a, b, c, d)
        ctx.w2 = w2
        return loss

    @staticmethod
    def backward(ctx, g):
        a, b, c, d = ctx.saved_tensors
        L = _native.lib()
        g = g.contiguous().float()
        ga = torch.empty_like(a)
        gc = None if c is None else torch.empty_like(c)
        _native.check(L.gr_l1_loss_bwd(_native.ptr(a), _native.ptr(b), a.numel(), _native.ptr(c), _native.ptr(d),
                                       0 if c is None else c.numel(), ctypes.c_float(ctx.w2), _native.ptr(g),
                                       _native.ptr(ga), _native.ptr(gc), _stream(a)), "gr_l1_loss_bwd")
        return ga, None, gc, None, None


def l1_loss(a: torch.Tensor, b: torch.Tensor, c: Optional[torch.Tensor] = None, d: Optional[torch.Tensor] = None,
            w2: float = 0.0) -> torch.Tensor:
    """mean|a - b| + w2 * mean|c - d| on the HIP device; gradients flow to a and c (the rendered
    image and alpha), not to the targets b and d."""
    if a.device.type != "cuda":
        raise RuntimeError("l1_loss runs on the HIP device; there is no CPU path")
    if a.shape != b.shape or (c is not None and (d is None or c.shape != d.shape)):
        raise ValueError("l1_loss: shape mismatch")
    f = lambda t: None if t is None else t.contiguous().float()  # noqa: E731
    return _L1Loss.apply(f(a), f(b).detach(), f(c), None if d is None else f(d).detach(), float(w2))


__all__ = ["l1_loss"]
