"""TEST INFRASTRUCTURE ONLY: a tiny dense float32 torch restatement of the reference render op
(python/torch_renderer.py:57-203), used as a CPU stand-in renderer to test the data-parallel fit
plumbing with the gloo backend where no GPU exists.  Never used by the product."""
from __future__ import annotations

import torch


def render(means, scales, colors, opacities, cam, width, height, background):
    view = cam.view.to(torch.float32)
    proj = cam.proj.to(torch.float32)
    n = means.shape[0]
    p = torch.cat([means, torch.ones((n, 1))], 1)
    pc = (view @ p.t()).t()
    clip = (proj @ pc.t()).t()
    w = clip[:, 3:4]
    ws = torch.where(w.abs() < 1e-8, torch.ones_like(w), w)
    ndc = clip[:, :3] / ws
    px = (ndc[:, 0] * 0.5 + 0.5) * (width - 1)
    py = (1.0 - (ndc[:, 1] * 0.5 + 0.5)) * (height - 1)
    valid = ((ndc[:, 2] >= -1) & (ndc[:, 2] <= 1) & (w.squeeze(1) != 0)).float()
    za = pc[:, 2].abs().clamp_min(1e-6)
    col = colors.clamp(0, 1)
    sx = (scales[:, 0].abs() * 0.5 * width * proj[0, 0].abs() / za).clamp_min(1.0)
    sy = (scales[:, 1].abs() * 0.5 * height * proj[1, 1].abs() / za).clamp_min(1.0)
    ys = torch.arange(height, dtype=torch.float32) + 0.5
    xs = torch.arange(width, dtype=torch.float32) + 0.5
    gy, gx = torch.meshgrid(ys, xs, indexing="ij")
    dx = gx[None] - px[:, None, None]
    dy = gy[None] - py[:, None, None]
    e = -0.5 * (dx * dx / sx[:, None, None] ** 2 + dy * dy / sy[:, None, None] ** 2)
    wgt = (opacities.clamp_min(0) * valid)[:, None, None] * torch.exp(e)
    W = wgt.sum(0)
    C = torch.einsum("nhw,nc->hwc", wgt, col)
    D = torch.einsum("nhw,n->hw", wgt, za)
    out = ((background.view(1, 1, 3) + C) / (1 + W)[..., None]).clamp(0, 1)
    return out, (W / (1 + W)).clamp(0, 1), (D / (W + 1e-6)).clamp_min(0)
