"""Spatial (Morton) order of Gaussians: a layout choice of the caller, not part of the math.

The rendered images and gradients do not depend on the order of the Gaussians beyond float summation order
(the reference's weighted average is order-independent, python/torch_renderer.py:164-203).  Neighbours in 3-D
Morton order are neighbours on screen in every view, so the tile sort writes runs instead of scattered pairs,
a block of 64 consecutive Gaussians finds its rows of one tile as one contiguous run, and a tile's records are
gathered from few cache lines.  Used by the fit driver (fit_multiview.ViewShardedFitter keeps its parameters in
this order) and by the drop-in op (torch_renderer renders a Morton-ordered copy of a caller's Gaussians).
"""
from __future__ import annotations

import torch


def _spread3(v: torch.Tensor) -> torch.Tensor:
    """Bits 0..9 of v moved to bits 0, 3, 6, .. 27 (Morton interleave of one axis)."""
    v = (v | (v << 16)) & 0x030000FF
    v = (v | (v << 8)) & 0x0300F00F
    v = (v | (v << 4)) & 0x030C30C3
    return (v | (v << 2)) & 0x09249249


def morton_order(means: torch.Tensor) -> torch.Tensor:
    """Permutation that puts the Gaussians in 3-D Morton (Z-curve) order of their centres, 10 bits per
    axis over the bounding box; stable, so every rank computes the same permutation from the same
    means.  Neighbours in this order are neighbours in space, hence on screen in every view: the
    pairs one wave emits land in few tiles (the tile sort writes runs instead of scattered 8-byte
    pairs) and a tile's records are gathered from few cache lines."""
    with torch.no_grad():
        m = means.detach()
        mt = m.t().contiguous()  # (3, N): row reductions (a dim-0 reduction of (N,3) is a slow strided kernel)
        lo = mt.amin(1)
        ext = (mt.amax(1) - lo).clamp_min(1e-20)
        q = ((m - lo) / ext * 1023.0).round().to(torch.int64).clamp_(0, 1023)
        key = _spread3(q[:, 0]) | (_spread3(q[:, 1]) << 1) | (_spread3(q[:, 2]) << 2)
        return torch.argsort(key, stable=True)
