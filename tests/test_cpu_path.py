"""The drop-in on host tensors (config C1, "plumbing, no GPU"): render_gaussians_torch on CPU tensors runs
3dgaussian_amd/cpu_renderer.py, checked against the reference's own goldens (tests/golden/f1_*, f2_*:
forward and autograd gradients of python/torch_renderer.py:109-203) at relL2 <= 1e-4 / PSNR >= 60 dB
(the float64 oracle only as the checker of the one ill-conditioned tensor, as in test_parity_gpu.py)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import golden, golden_names

GRAD = (("d_means", "means"), ("d_scales", "scales"), ("d_colors", "colors"), ("d_opacities", "opacities"))


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("name", golden_names("f1_") + golden_names("f2_"))
@pytest.mark.parametrize("with_depth", [True, False])
def test_cpu_path_matches_reference_goldens(pkg, name, with_depth):
    tr = pkg.torch_renderer
    d = golden(name)
    W, H = int(d["width"]), int(d["height"])
    t = {k: torch.from_numpy(np.ascontiguousarray(d[k])).requires_grad_(True) for _, k in GRAD}
    cam = tr.Camera(view=torch.from_numpy(d["view"]), proj=torch.from_numpy(d["proj"]))
    res = tr.render_gaussians_torch(t["means"], t["scales"], t["colors"], t["opacities"], cam, W, H,
                                    background=torch.from_numpy(d["background"]),
                                    max_gaussians=max(10000, d["means"].shape[0]), return_aux=True)
    if d["means"].shape[0] == 0:
        np.testing.assert_array_equal(res.numpy(), d["out_rgb"])
        return
    out, alpha, depth = res
    loss = (out * torch.from_numpy(d["g_rgb"])).sum() + (alpha * torch.from_numpy(d["g_alpha"])).sum()
    if with_depth:
        loss = loss + (depth * torch.from_numpy(d["g_depth"])).sum()
    loss.backward()
    for k, v in (("out_rgb", out), ("out_alpha", alpha), ("out_depth", depth)):
        assert _rel(v.detach().numpy(), d[k]) <= 1e-4, (name, k)
    assert 10 * np.log10(1.0 / max(np.mean((out.detach().numpy() - d["out_rgb"]) ** 2), 1e-30)) >= 60.0
    if not with_depth:
        return  # the goldens' gradients include the depth term
    exact = None
    for gk, k in GRAD:
        err = _rel(t[k].grad.numpy(), d[gk])
        if err <= 1e-4:
            continue
        # ill-conditioned tensors (the one-Gaussian scene's opacity gradient: large cancelling terms)
        # where the reference's own float32 result is > 3e-5 from the exact value: the same rule as
        # tests/test_parity_gpu.py, distance to the float64 oracle <= max(1e-4, 3 x the reference's own)
        if exact is None:
            exact = _exact_grads(d)
        ref_err = _rel(d[gk], exact[gk])
        assert ref_err > 3e-5, f"{name} {gk}: relL2 vs reference {err:.2e}"
        err = _rel(t[k].grad.numpy(), exact[gk])
        assert err <= max(1e-4, 3 * ref_err), f"{name} {gk}: relL2 vs exact {err:.2e} (reference {ref_err:.1e})"


def _exact_grads(d):
    from oracle import oracle as orc  # the checker (float64), as in the GPU parity tests

    v = orc.make_view(d["view"], d["proj"], int(d["width"]), int(d["height"]), d["background"])
    sc = orc.Scene(d["means"], d["scales"], d["colors"], d["opacities"])
    g = orc.backward(v, sc, d["g_rgb"], d["g_alpha"], d["g_depth"], binned=False)
    return dict(zip((gk for gk, _ in GRAD), g))


def test_cpu_path_without_depth_matches_autograd(pkg):
    """Gradients with and without an upstream depth gradient against torch autograd of a dense
    float64 restatement (the goldens hold only the with-depth gradients)."""
    d = golden("f1_n300_64x48_sh")
    tr = pkg.torch_renderer
    W, H = int(d["width"]), int(d["height"])
    t = {k: torch.from_numpy(np.ascontiguousarray(d[k])).requires_grad_(True) for _, k in GRAD}
    cam = tr.Camera(view=torch.from_numpy(d["view"]), proj=torch.from_numpy(d["proj"]))
    out, alpha, depth = tr.render_gaussians_torch(t["means"], t["scales"], t["colors"], t["opacities"], cam, W, H,
                                                  return_aux=True)
    g = torch.from_numpy(d["g_rgb"])
    ((out * g).sum() + alpha.sum()).backward()
    t64 = {k: v.detach().double().requires_grad_(True) for k, v in t.items()}
    cr = pkg.cpu_renderer
    o2, a2, _ = cr.render(t64["means"], t64["scales"], t64["colors"], t64["opacities"], cam.view.double(),
                          cam.proj.double(), W, H, torch.zeros(3, dtype=torch.float64))
    ((o2 * g.double()).sum() + a2.sum()).backward()
    for _, k in GRAD:
        assert _rel(t[k].grad.numpy(), t64[k].grad.numpy()) <= 1e-4, k


def test_closed_form_backward_matches_autograd_of_forward(pkg):
    """The splat Function's closed-form backward against autograd through a float64 dense
    evaluation of the same forward (guards the moment bookkeeping, incl. the depth terms)."""
    cr = pkg.cpu_renderer
    gen = torch.Generator().manual_seed(3)
    n, W, H = 40, 23, 17
    px = (torch.rand(n, generator=gen, dtype=torch.float64) * W).requires_grad_(True)
    py = (torch.rand(n, generator=gen, dtype=torch.float64) * H).requires_grad_(True)
    sx = (1 + 3 * torch.rand(n, generator=gen, dtype=torch.float64)).requires_grad_(True)
    sy = (1 + 3 * torch.rand(n, generator=gen, dtype=torch.float64)).requires_grad_(True)
    ov = torch.rand(n, generator=gen, dtype=torch.float64).requires_grad_(True)
    c = torch.rand(n, 3, generator=gen, dtype=torch.float64).requires_grad_(True)
    za = (1 + torch.rand(n, generator=gen, dtype=torch.float64)).requires_grad_(True)
    bg = torch.rand(3, generator=gen, dtype=torch.float64).requires_grad_(True)
    ins = (px, py, sx, sy, ov, c, za, bg)
    go, ga, gd = (torch.randn(H, W, 3, generator=gen, dtype=torch.float64), torch.randn(H, W, generator=gen, dtype=torch.float64),
                  torch.randn(H, W, generator=gen, dtype=torch.float64))
    o, a, dd = cr._Splat.apply(*ins, W, H)
    g1 = torch.autograd.grad((o * go).sum() + (a * ga).sum() + (dd * gd).sum(), ins)
    xs, ys = torch.arange(W, dtype=torch.float64) + 0.5, torch.arange(H, dtype=torch.float64) + 0.5
    dx = xs[None, None, :] - px[:, None, None]
    dy = ys[None, :, None] - py[:, None, None]
    w = ov[:, None, None] * torch.exp(-0.5 * (dx * dx / sx[:, None, None] ** 2 + dy * dy / sy[:, None, None] ** 2))
    Wt, C, D = w.sum(0), torch.einsum("nhw,nc->hwc", w, c), torch.einsum("nhw,n->hw", w, za)
    o2 = ((bg + C) / (1 + Wt)[..., None]).clamp(0, 1)
    a2 = (Wt / (1 + Wt)).clamp(0, 1)
    d2 = (D / (Wt + 1e-6)).clamp_min(0)
    g2 = torch.autograd.grad((o2 * go).sum() + (a2 * ga).sum() + (d2 * gd).sum(), ins)
    for x, y in zip(g1, g2):
        assert _rel(x.detach().numpy(), y.detach().numpy()) <= 1e-10


def test_fit_driver_on_cpu_reproduces_reference_curve(pkg, tmp_path):
    """Config C1's plumbing: the fit driver (fit_multiview.main) on host tensors reproduces the loss
    curve of the reference's unchanged fit_multiview_stub.py (golden F4) at rtol 1e-4."""
    import importlib
    import os

    from conftest import GOLDEN

    d = golden("f4_fit_curve")  # the F4 run is square (make_golden.py: --width 48 --height 48; no height key stored)
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    fm.main(["--targets_dir", os.path.join(GOLDEN, "fit_targets"), "--out_dir", str(tmp_path), "--iters", str(int(d["iters"])),
             "--width", str(int(d["width"])), "--height", str(int(d["height"] if "height" in d else d["width"])), "--num_gaussians", str(int(d["num_gaussians"])),
             "--max_gaussians", str(int(d["max_gaussians"])), "--densify_interval", str(int(d["densify_interval"])),
             "--prune_interval", str(int(d["densify_interval"])), "--seed", str(int(d["seed"])), "--device", "cpu"])
    losses = np.array([float(x) for x in (tmp_path / "loss.txt").read_text().split()])
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-4)


def test_bench_cpu_baseline_small():
    """bench.cpu_baseline on a small scene (the leg the GPU bench runs at C4 on every usable core): the keys the bench
    line carries, the thread count equal to the usable cores."""
    import importlib

    bench = importlib.import_module("bench")
    cores, how = bench.usable_cores()
    out = bench.cpu_baseline(2000, 48, 2)
    assert out["value"] > 0 and out["kind"] == "port" and out["oracle"]["value"] > 0 and out["c1"]["value"] > 0
    assert out["usable_cores"] == cores and out["torch_threads"] == cores and out["cores"] == cores
    assert "sched_getaffinity" in how and "unscaled" in out["sample"]
