"""GPU parity at the bench's own scale: one full view of config C4 (1M Gaussians, 800x800) and of C5
(3M Gaussians, 1920x1080), in the bench's precision mode (depth_grad=False: no upstream depth gradient,
two-piece splits) and in the default mode (depth_grad=True, upstream depth gradient), against

* the float64 binned oracle (the product's footprint: 7 sigma tail without a depth gradient, 8 sigma
  with one, 5.5 sigma core) on every pixel and every Gaussian:
  relL2 <= 2e-5 on out/alpha/depth, <= 1e-4 on all four gradients, PSNR >= 60 dB;
* the float64 DENSE reference semantics (torch_renderer.py:164-203: every Gaussian at every pixel, no
  cutoff) on a sample: out/alpha/depth at 1000 random pixels summed over all N Gaussians, and the exact
  gradients of 1000 random Gaussians each summed over the whole image (SURVEY.md §7 "oracle reach");
  relL2 <= 1e-4 over the sample.  This ties the tile footprint (7 sigma / 5.5 sigma core) to the dense
  math at the sizes the headline runs.

The "fit32" mode and the tile-32 fitted-state case run the kernels the headline times (k_fwd32_l1, k_bwd32: the
fused fit path at 32-pixel tiles) with the fit's L1 + silhouette loss; their upstream gradients are the L1 signs of
the HIP images, handed to the oracle and the dense reference alike.

Scenes: SURVEY.md §8(d)'s synthetic recipe (density-matched scale), Gaussians in the trainer's Morton
order (bench.py's layout), orbit view 0.  Upstream gradients: seeded standard normal."""
from __future__ import annotations

import importlib
import time

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

CONFIGS = {"C4": (1_000_000, 800, 800, 50), "C5": (3_000_000, 1920, 1080, 100)}
GRADS = ("d_means", "d_scales", "d_colors", "d_opac")


def _scene(n):
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    sc = orc.synthetic_scene(n, seed=0)
    perm = fm.morton_order(torch.from_numpy(sc.means)).numpy()
    return orc.Scene(sc.means[perm].copy(), sc.scales[perm].copy(), sc.colors[perm].copy(), sc.opacities[perm].copy())


def _fused32(tr, t, view, proj, W, H, target, mask, w_sil, g_scale, cuda):
    """The kernels the headline times, on one view: the fused fit path at the fit's tile size (fm.FIT_TILE = 32:
    k_fwd32_l1 with its L1 epilogue -> k_bwd32 -> k_gather_view -> k_reduce_sums), images written beside.
    Returns (loss, out, alpha, grads) as numpy and the L1 upstream (g_rgb, g_a) the references take: the HIP images'
    own signs sign(out - t), sign(alpha - m) (torch's abs' with sign(0) = 0), scaled as the kernel scales them, so a
    near-tie at the kink (which the last float bit decides) is the same pixel gradient on both sides."""
    from test_tile32_gpu import _fused_view

    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    t = [x.detach().contiguous() for x in t]
    loss, out, alpha, grads, _ = _fused_view(tr, t, view, proj, W, H, fm.FIT_TILE, target, mask, w_sil, g_scale, cuda)
    h_out, h_alpha = out.cpu().numpy(), alpha.cpu().numpy()
    tn, mn = target.cpu().numpy(), mask.cpu().numpy()
    HW = W * H
    g_rgb = (np.sign(h_out.astype(np.float64) - tn) * (g_scale / (3 * HW))).astype(np.float32)
    g_a = (np.sign(h_alpha.astype(np.float64) - mn) * (w_sil * g_scale / HW)).astype(np.float32)
    return loss, h_out, h_alpha, [g.cpu().numpy() for g in grads], g_rgb, g_a


def _l1_target(H, W, seed, cuda):
    g = torch.Generator(device=cuda).manual_seed(seed)
    target = torch.rand((H, W, 3), generator=g, device=cuda)
    return target, (target.mean(dim=2) > 0.5).float().contiguous()


def _fit_mode(tr, t, view, proj, W, H, g_rgb, g_a, cuda):
    """The fused fit path's render settings (fit_multiview._views_direct): one zone at FIT_CUTOFF, no
    depth channel, forward_native(want_depth=False) + gr_bwd (generic upstream gradients)."""
    gv = tr.make_view(view, proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF, depth_grad=False)
    m, s, c, o = (x.detach() for x in t)
    out, alpha, depth, st = tr.forward_native(m, s, c, o, gv, want_depth=False)
    assert depth is None
    grads = tr.backward_native(m, s, c, o, st, torch.from_numpy(g_rgb).to(cuda), torch.from_numpy(g_a).to(cuda), None)
    return out, alpha, grads


@pytest.mark.timeout(400)
@pytest.mark.parametrize("mode", ["no_depth_grad", "depth_grad", "fit", "fit32"])
@pytest.mark.parametrize("cfg", ["C4", "C5"])
def test_full_view_vs_oracle(pkg, cuda, cfg, mode):
    """mode: the bench's drop-in mode (depth_grad=False), the default mode (depth_grad=True, with an
    upstream depth gradient), the fit path's settings on the 16-pixel kernels (one FIT_CUTOFF zone, no depth,
    generic upstream), or "fit32": the headline's own kernels (the fused path at 32-pixel tiles, k_fwd32_l1 /
    k_bwd32, with the fit's L1 + silhouette loss on a random target; the references take the HIP images' signs)
    against the float64 binned oracle at tile 32 and the dense sample."""
    tr = pkg.torch_renderer
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    depth_grad = mode == "depth_grad"
    n, W, H, V = CONFIGS[cfg]
    sc = _scene(n)
    view, proj = orc.orbit_cameras(V, W, H)[0]
    rng = np.random.default_rng(7)
    g_rgb = rng.standard_normal((H, W, 3)).astype(np.float32)
    g_a = rng.standard_normal((H, W)).astype(np.float32)
    g_d = rng.standard_normal((H, W)).astype(np.float32) if depth_grad else None

    t = [torch.from_numpy(a).to(cuda).requires_grad_(True) for a in sc.arrays()]
    tile, h_loss = 0, None
    if mode == "fit32":
        tile = fm.FIT_TILE
        target, mask = _l1_target(H, W, 5, cuda)
        h_loss, h_out, h_a, h_grads, g_rgb, g_a = _fused32(tr, t, view, proj, W, H, target, mask, 0.2, 1.0 / V, cuda)
        hip = {"out": h_out, "alpha": h_a}
        hip.update(zip(GRADS, h_grads))
        hip["d_scales"] = hip["d_scales"][:, :2]  # (the fused path's scale gradient has no z column, the reference's either)
        depth = None
    elif mode == "fit":
        out, alpha, grads = _fit_mode(tr, t, view, proj, W, H, g_rgb, g_a, cuda)
        depth = None
    else:
        out, alpha, depth = tr.rasterize(*t, view, proj, W, H, depth_grad=depth_grad)
        loss = (out * torch.from_numpy(g_rgb).to(cuda)).sum() + (alpha * torch.from_numpy(g_a).to(cuda)).sum()
        if depth_grad:
            loss = loss + (depth * torch.from_numpy(g_d).to(cuda)).sum()
        loss.backward()
        grads = [x.grad for x in t]
    if mode != "fit32":
        torch.cuda.synchronize()
        hip = {"out": out.detach().cpu().numpy(), "alpha": alpha.detach().cpu().numpy()}
        if depth is not None:
            hip["depth"] = depth.detach().cpu().numpy()
        for k, x in zip(GRADS, grads):
            hip[k] = x.cpu().numpy()

    t0 = time.perf_counter()
    fit = mode in ("fit", "fit32")
    cut = tr.FIT_CUTOFF if fit else tr.default_cutoff(depth_grad)
    core = tr.FIT_CUTOFF if fit else tr.DEFAULT_CORE_CUTOFF
    v = orc.make_view(view, proj, W, H, None, cutoff=cut, core_cutoff=core, tile=tile)
    ora = dict(zip(("out", "alpha", "depth"), orc.forward(v, sc, binned=True)))
    if depth is None:
        del ora["depth"]
    ora.update(zip(GRADS, orc.backward(v, sc, g_rgb, g_a, g_d, binned=True)))
    if mode == "fit32":
        ora["d_scales"] = ora["d_scales"][:, :2]
        tn, mn = target.cpu().numpy().astype(np.float64), mask.cpu().numpy().astype(np.float64)
        # (the kernel's loss value is unscaled; g_scale scales its upstream gradients only)
        o_loss = np.abs(ora["out"].astype(np.float64) - tn).mean() + 0.2 * np.abs(ora["alpha"].astype(np.float64) - mn).mean()
    errs = {k: orc.rel_l2(hip[k], ora[k]) for k in ora}
    if h_loss is not None:
        errs["loss"] = abs(h_loss - o_loss) / o_loss
    t1 = time.perf_counter()

    pix = rng.choice(W * H, 1000, replace=False).astype(np.int32)
    d_out, d_a, d_d = orc.dense_pixels(v, sc, pix)
    sel = np.sort(rng.choice(n, 1000, replace=False)).astype(np.int32)
    dense_g = orc.dense_grads_sel(v, sc, sel, g_rgb, g_a, g_d)
    dense = {"out": orc.rel_l2(hip["out"].reshape(-1, 3)[pix], d_out),
             "alpha": orc.rel_l2(hip["alpha"].reshape(-1)[pix], d_a)}
    if depth is not None:
        dense["depth"] = orc.rel_l2(hip["depth"].reshape(-1)[pix], d_d)
    for k, gd in zip(GRADS, dense_g):
        dense[k] = orc.rel_l2(hip[k][sel], gd[:, :2] if (k == "d_scales" and mode == "fit32") else gd)
    print(f"{cfg} {mode}: vs binned oracle", {k: f"{e:.2e}" for k, e in errs.items()},
          f"({t1 - t0:.1f} s); vs dense sample", {k: f"{e:.2e}" for k, e in dense.items()},
          f"({time.perf_counter() - t1:.1f} s)")
    for k in ("out", "alpha", "depth"):
        if k in errs:
            assert errs[k] <= 2e-5, (k, errs[k])
    for k in GRADS:
        assert errs[k] <= 1e-4, (k, errs[k])
    if "loss" in errs:
        assert errs["loss"] <= 1e-5, errs["loss"]
    assert orc.psnr(hip["out"], ora["out"]) >= 60.0
    for k, e in dense.items():
        assert e <= 1e-4, (k, e)


@pytest.mark.timeout(400)
@pytest.mark.parametrize("tile", [16, 32])
def test_fit_path_on_fitted_state_vs_dense(pkg, cuda, tile):
    """The bench's own workload after several fit steps (Gaussians moved, scales and opacities changed by
    Adam): the fit footprint (one FIT_CUTOFF zone, no depth) against the dense float64 reference on a sample
    (1000 pixels, 1000 Gaussians), relL2 <= 1e-4.  tile 16: the 16-pixel kernels with generic upstream gradients;
    tile 32: the headline's own kernels (the fused path, k_fwd32_l1 / k_bwd32) with the fit's L1 + silhouette loss
    on that view's target, the dense reference taking the HIP images' signs."""
    import importlib

    tr = pkg.torch_renderer
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    n, W, H, V = CONFIGS["C4"]
    params = bench.synthetic_params(n, cuda)
    cams = fm.orbit_cameras(V, W, H, cuda)
    g = torch.Generator(device=cuda).manual_seed(1)
    targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    fit = fm.ViewShardedFitter(params, cams, targets, W, H, lr=0.02, masks=masks)
    for _ in range(8):
        fit.step()
    with torch.no_grad():
        acts = [a.detach().contiguous() for a in fm.activations(fit.params)]
    sc = orc.Scene(*(a.cpu().numpy() for a in acts))
    view, proj = orc.orbit_cameras(V, W, H)[3]
    rng = np.random.default_rng(9)
    g_rgb = rng.standard_normal((H, W, 3)).astype(np.float32)
    g_a = rng.standard_normal((H, W)).astype(np.float32)
    if tile == 32:
        _, out, alpha, grads, g_rgb, g_a = _fused32(tr, acts, view, proj, W, H, fit.targets[3], fit.masks[3], fit.w_sil,
                                                    1.0 / V, cuda)
        grads[1] = grads[1][:, :2]
    else:
        out, alpha, grads = _fit_mode(tr, acts, view, proj, W, H, g_rgb, g_a, cuda)
        out, alpha, grads = out.cpu().numpy(), alpha.cpu().numpy(), [x.cpu().numpy() for x in grads]
    v = orc.make_view(view, proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF)
    pix = rng.choice(W * H, 1000, replace=False).astype(np.int32)
    d_out, d_a, _ = orc.dense_pixels(v, sc, pix)
    sel = np.sort(rng.choice(n, 1000, replace=False)).astype(np.int32)
    dense_g = orc.dense_grads_sel(v, sc, sel, g_rgb, g_a, None)
    errs = {"out": orc.rel_l2(out.reshape(-1, 3)[pix], d_out),
            "alpha": orc.rel_l2(alpha.reshape(-1)[pix], d_a)}
    for k, x, gd in zip(GRADS, grads, dense_g):
        errs[k] = orc.rel_l2(x[sel], gd[:, : x.shape[1]] if x.ndim == 2 else gd)
    print(f"fitted C4 state, fit path at {tile}-pixel tiles vs dense sample:", {k: f"{e:.2e}" for k, e in errs.items()})
    for k, e in errs.items():
        assert e <= 1e-4, (k, e)


def _opacities(rng, opac_range, shape):
    """U(lo, hi); "mixed_negative": half from U(-1e5, -1) (clamped to 0 by the render, torch_renderer.py:177) and half
    from U(0, 2), interleaved, so large negative and live positive opacities meet on the same tiles."""
    if opac_range == "mixed_negative":
        o = rng.uniform(0.0, 2.0, shape)
        o[::2] = rng.uniform(-1e5, -1.0, o[::2].shape)
        return o.astype(np.float32)
    lo, hi = opac_range
    return rng.uniform(lo, hi, shape).astype(np.float32)


# "mixed_negative": large negative opacities beside live ones - the record keeps max(o, 0)
# and the colours clamp to [0, 1], so the A operands o c ex stay within max(o, 0) of the scale f16_sa_of sizes them by
@pytest.mark.parametrize("opac_range", [(1e-4, 1e-3), (0.0, 1.0), (100.0, 3000.0), (3000.0, 6000.0), (0.0, 1e5),
                                        "mixed_negative"])
def test_fit_mode_f16_operand_range(pkg, cuda, opac_range):
    """The fit-path forward (no depth channel) multiplies on f16 operand pieces pre-scaled by 2^sa (A) and
    2^12 (B), sa = 4 while the view's largest opacity is below 2^11 and lower above (f16_sa_of): opacities
    from 1e-4 (operands near the f16 subnormal range) up to 1e5 (past the fixed 2^4 scale's f16 range of
    4094) stay finite and within the parity bar vs the float64 binned oracle."""
    tr = pkg.torch_renderer
    rng = np.random.default_rng(7)
    sc = orc.synthetic_scene(3000, seed=3, scale=0.05)
    sc = orc.Scene(sc.means, sc.scales, sc.colors, _opacities(rng, opac_range, sc.opacities.shape))
    view, proj = orc.orbit_cameras(4, 160, 120)[2]
    W, H = 160, 120
    g_rgb = rng.standard_normal((H, W, 3)).astype(np.float32)
    g_a = rng.standard_normal((H, W)).astype(np.float32)
    t = [torch.from_numpy(a).to(cuda) for a in sc.arrays()]
    out, alpha, grads = _fit_mode(tr, t, view, proj, W, H, g_rgb, g_a, cuda)
    v = orc.make_view(view, proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF)
    o_out, o_a, _ = orc.forward(v, sc, binned=True)
    o_grads = orc.backward(v, sc, g_rgb, g_a, np.zeros((H, W), np.float32), binned=True)
    errs = {"out": orc.rel_l2(out.cpu().numpy(), o_out), "alpha": orc.rel_l2(alpha.cpu().numpy(), o_a)}
    for k, g, og in zip(GRADS, grads, o_grads):
        errs[k] = orc.rel_l2(g.cpu().numpy(), og)
    print(f"opacities {opac_range}: {int((sc.opacities > 0).sum())} live;", {k: f"{e:.2e}" for k, e in errs.items()})
    assert np.isfinite(out.cpu().numpy()).all()
    assert (sc.opacities > 0).sum() > 0 and float(out.abs().sum()) > 0.0  # a live scene, a non-empty image
    for k, e in errs.items():
        assert e <= 1e-4, (k, e)
