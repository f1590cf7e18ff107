"""The render op for tensors on a CPU (or any non-HIP) device: config C1's "plumbing, no GPU" case.

The reference op is device-agnostic torch (python/torch_renderer.py:109-203) and the reference fit
loop runs it on ``cpu`` on Linux (device_utils.py:9-13, fit_multiview_stub.py:231).  The drop-in
``torch_renderer.render_gaussians_torch`` dispatches on the tensors' device: HIP tensors always go to
libgr_hip.so (and raise ImportError when it is missing: no fallback), CPU tensors come here.

Semantics are the reference's, without the tile cutoff of the HIP path: every Gaussian is evaluated at
every pixel.  The evaluation is organised differently from the reference's chunk loop (:164-190):

* the weight is separable, ``w_g(x, y) = o_g valid_g ex_g(x) ey_g(y)`` with
  ``ex_g(x) = exp(-(x+0.5-px)^2 / (2 sx^2))`` (same for y), so the forward accumulators are one GEMM
  per chunk of Gaussians, ``[W | C_r | C_g | C_b | D](y, x) = sum_g ey_g(y) (o_g v_g ex_g(x))``;
* the splat stage is a ``torch.autograd.Function`` whose backward is the closed form of SURVEY.md
  Appendix A evaluated through the same factorisation: per Gaussian, the moments
  ``sum_{x,y} ey(y) dy^b U_c(y, x) ex(x) dx^a`` of the five per-pixel upstream channels
  ``U = (dC_r, dC_g, dC_b, dW, dD)`` (two GEMMs per chunk), never an (N, H, W) autograd graph;
* projection, colour (RGB, SH degree 1 of :86-104, degree-3 extension) and sigma
  (:57-78, :141-150) are plain torch ops, differentiated by autograd as in the reference.

Memory stays O(chunk * (H + W) + H * W) per view instead of the reference's ~40 B per Gaussian-pixel.
"""
from __future__ import annotations

import torch

# Gaussians per GEMM chunk (bounds the (G, 5, W) operand)
_CHUNK_ELEMS = 1 << 22


def _project(means: torch.Tensor, view: torch.Tensor, proj: torch.Tensor, width: int, height: int):
    """torch_renderer.py:57-78: row-major V [m, 1], P p_cam, w_safe, ndc -> px, py, valid, z_abs."""
    n = means.shape[0]
    ones = torch.ones((n, 1), dtype=means.dtype, device=means.device)
    pc = torch.cat([means, ones], dim=1) @ view.t()
    clip = pc @ proj.t()
    w = clip[:, 3]
    w_safe = torch.where(w.abs() < 1e-8, torch.ones_like(w), w)
    ndc = clip[:, :3] / w_safe[:, None]
    px = (ndc[:, 0] * 0.5 + 0.5) * (width - 1)
    py = (1.0 - (ndc[:, 1] * 0.5 + 0.5)) * (height - 1)
    valid = (ndc[:, 2] >= -1.0) & (ndc[:, 2] <= 1.0) & (w != 0.0)
    za = pc[:, 2].abs().clamp_min(1e-6)
    return px, py, valid, za


def _sh3_tail(d: torch.Tensor) -> torch.Tensor:
    """Degree-2/3 terms of the build's unnormalised basis (extension; same polynomials as the HIP
    kernels and oracle/gr_oracle.c), (N, 12)."""
    x, y, z = d[:, 0], d[:, 1], d[:, 2]
    xx, yy, zz = x * x, y * y, z * z
    return torch.stack([x * y, y * z, 3.0 * zz - 1.0, x * z, xx - yy, y * (3.0 * xx - yy), x * y * z,
                        y * (5.0 * zz - 1.0), z * (5.0 * zz - 3.0), x * (5.0 * zz - 1.0), z * (xx - yy),
                        x * (xx - 3.0 * yy)], dim=1)


def _colors(colors: torch.Tensor, means: torch.Tensor, view: torch.Tensor) -> torch.Tensor:
    """torch_renderer.py:81-106 (+ the degree-3 extension), before the clamp."""
    if colors.ndim == 2:
        return colors
    cam = torch.linalg.inv(view)[:3, 3]
    d = cam.view(1, 3) - means
    d = d / (torch.linalg.norm(d, dim=1, keepdim=True) + 1e-8)
    out = colors[:, 0, :] + colors[:, 1, :] * d[:, 0:1] + colors[:, 2, :] * d[:, 1:2] + colors[:, 3, :] * d[:, 2:3]
    if colors.shape[1] == 16:
        out = out + torch.einsum("nb,nbc->nc", _sh3_tail(d), colors[:, 4:, :])
    return out


def _chunks(n: int, width: int, height: int):
    g = max(1, min(n, _CHUNK_ELEMS // (5 * max(width, height))))
    for a in range(0, n, g):
        yield a, min(n, a + g)


def _factors(px, py, sx, sy, width: int, height: int):
    xs = torch.arange(width, dtype=px.dtype, device=px.device) + 0.5
    ys = torch.arange(height, dtype=px.dtype, device=px.device) + 0.5
    dx = xs[None, :] - px[:, None]
    dy = ys[None, :] - py[:, None]
    ex = torch.exp(-0.5 * (dx * dx) / (sx * sx)[:, None])
    ey = torch.exp(-0.5 * (dy * dy) / (sy * sy)[:, None])
    return dx, dy, ex, ey


class _Splat(torch.autograd.Function):
    """(px, py, sx, sy, ov = max(o,0) valid, c = clamp(col), za, bg) -> (out, alpha, depth)."""

    @staticmethod
    def forward(ctx, px, py, sx, sy, ov, c, za, bg, width, height):
        n = px.shape[0]
        acc = torch.zeros((height, 5 * width), dtype=px.dtype, device=px.device)
        for a, b in _chunks(n, width, height):
            _, _, ex, ey = _factors(px[a:b], py[a:b], sx[a:b], sy[a:b], width, height)
            v = torch.cat([torch.ones_like(za[a:b, None]), c[a:b], za[a:b, None]], dim=1)  # (G, 5)
            op = (ov[a:b, None] * v)[:, :, None] * ex[:, None, :]  # (G, 5, W)
            acc += ey.t() @ op.reshape(b - a, 5 * width)
        acc = acc.view(height, 5, width).permute(1, 0, 2)  # (5, H, W)
        Wt, C, D = acc[0], acc[1:4].permute(1, 2, 0), acc[4]
        out_r = (bg.view(1, 1, 3) + C) / (1.0 + Wt)[..., None]
        alpha_r = Wt / (1.0 + Wt)
        depth_r = D / (Wt + 1e-6)
        ctx.save_for_backward(px, py, sx, sy, ov, c, za, Wt, D, out_r, alpha_r, depth_r)
        ctx.dims = (width, height)
        return out_r.clamp(0.0, 1.0), alpha_r.clamp(0.0, 1.0), depth_r.clamp_min(0.0)

    @staticmethod
    def backward(ctx, g_out, g_alpha, g_depth):
        px, py, sx, sy, ov, c, za, Wt, D, out_r, alpha_r, depth_r = ctx.saved_tensors
        width, height = ctx.dims
        z = torch.zeros_like(Wt)
        g_out = torch.zeros_like(out_r) if g_out is None else g_out
        g_alpha = z if g_alpha is None else g_alpha
        g_depth = z if g_depth is None else g_depth
        # clamp masks are inclusive (torch's clamp backward); Appendix A
        go = g_out * ((out_r >= 0.0) & (out_r <= 1.0))
        ga = g_alpha * ((alpha_r >= 0.0) & (alpha_r <= 1.0))
        gd = g_depth * (depth_r >= 0.0)
        den = 1.0 + Wt
        gC = go / den[..., None]
        gW = -(go * out_r).sum(-1) / den + ga / (den * den) - gd * D / ((Wt + 1e-6) * (Wt + 1e-6))
        gD = gd / (Wt + 1e-6)
        U = torch.stack([gC[..., 0], gC[..., 1], gC[..., 2], gW, gD], 0)  # (5, H, W)
        g_bg = gC.sum((0, 1))
        n = px.shape[0]
        d_px, d_py, d_sx, d_sy = (torch.empty_like(px) for _ in range(4))
        d_ov, d_za = torch.empty_like(ov), torch.empty_like(za)
        d_c = torch.empty_like(c)
        for a, b in _chunks(n, width, height):
            G = b - a
            dx, dy, ex, ey = _factors(px[a:b], py[a:b], sx[a:b], sy[a:b], width, height)
            xw = torch.stack([ex, ex * dx, ex * dx * dx], 1)  # (G, 3, W)
            yw = torch.stack([ey, ey * dy, ey * dy * dy], 1)  # (G, 3, H)
            R = (U.reshape(5 * height, width) @ xw.reshape(3 * G, width).t()).view(5, height, G, 3)
            # M[ch, g, a, b] = sum_y yw[g, b, y] R[ch, y, g, a]; the moments used are (a, b) in
            # {(0,0), (1,0), (0,1), (2,0), (0,2)}
            M0 = torch.einsum("gy,cyga->cga", ey, R)  # b = 0, a = 0..2
            R0 = R[..., 0]  # (5, H, G): a = 0
            M1 = torch.einsum("gy,cyg->cg", yw[:, 1], R0)  # (a, b) = (0, 1)
            M2 = torch.einsum("gy,cyg->cg", yw[:, 2], R0)  # (0, 2)
            cv = torch.cat([c[a:b], torch.ones_like(za[a:b, None]), za[a:b, None]], 1).t()  # (5, G)
            q = (cv[:, :, None] * M0).sum(0)  # (G, 3): gw moments over dx^0..2 (b = 0)
            q01, q02 = (cv * M1).sum(0), (cv * M2).sum(0)
            o = ov[a:b]
            s2x, s2y = sx[a:b] * sx[a:b], sy[a:b] * sy[a:b]
            d_ov[a:b] = q[:, 0]
            d_c[a:b] = (o[None, :] * M0[0:3, :, 0]).t()
            d_za[a:b] = o * M0[4, :, 0]
            d_px[a:b] = o * q[:, 1] / s2x
            d_py[a:b] = o * q01 / s2y
            d_sx[a:b] = o * q[:, 2] / (s2x * sx[a:b])
            d_sy[a:b] = o * q02 / (s2y * sy[a:b])
        return d_px, d_py, d_sx, d_sy, d_ov, d_c, d_za, g_bg, None, None


def render(means, scales, colors, opacities, view, proj, width: int, height: int, background):
    """Differentiable dense render on the tensors' (non-HIP) device: (out (H,W,3), alpha, depth)."""
    view = view.to(dtype=means.dtype, device=means.device)
    proj = proj.to(dtype=means.dtype, device=means.device)
    px, py, valid, za = _project(means, view, proj, width, height)
    col = _colors(colors, means, view).clamp(0.0, 1.0)
    fx, fy = proj[0, 0].abs(), proj[1, 1].abs()
    sx = (scales[:, 0].abs() * 0.5 * width * fx / za).clamp_min(1.0)
    sy = (scales[:, 1].abs() * 0.5 * height * fy / za).clamp_min(1.0)
    ov = opacities.clamp_min(0.0) * valid.to(opacities.dtype)
    return _Splat.apply(px, py, sx, sy, ov, col, za, background, width, height)
