"""CPU: the trainer's Morton layout of the Gaussians (fit_multiview.spatial_order) is a permutation,
deterministic, spatially coherent, and leaves the fit's loss and (permuted) gradients unchanged."""
from __future__ import annotations

import importlib
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
fm = importlib.import_module("3dgaussian_amd.fit_multiview")


def test_morton_order_is_a_deterministic_permutation():
    torch.manual_seed(0)
    means = torch.rand(5000, 3) * 2 - 1
    p1, p2 = fm.morton_order(means), fm.morton_order(means.clone())
    assert torch.equal(p1, p2)
    assert torch.equal(torch.sort(p1).values, torch.arange(5000))


def test_morton_key_interleave():
    v = torch.tensor([0, 1, 2, 3, 1023], dtype=torch.int64)
    s = fm._spread3(v)
    ref = []
    for x in v.tolist():
        k = 0
        for b in range(10):
            k |= ((x >> b) & 1) << (3 * b)
        ref.append(k)
    assert s.tolist() == ref


def test_morton_order_is_spatially_coherent():
    torch.manual_seed(1)
    means = torch.rand(20000, 3)
    perm = fm.morton_order(means)
    step_sorted = (means[perm][1:] - means[perm][:-1]).norm(dim=1).mean()
    step_random = (means[1:] - means[:-1]).norm(dim=1).mean()
    assert step_sorted < 0.1 * step_random


def test_fit_loss_independent_of_order():
    torch.manual_seed(7)
    params = fm.build_params(30, torch.device("cpu"), use_sh=False)
    with torch.no_grad():
        params["scales_raw"].fill_(-1.0)
    W, H = 16, 12
    cams = fm.orbit_cameras(3, W, H, torch.device("cpu"))
    g = torch.Generator().manual_seed(3)
    targets = [torch.rand((H, W, 3), generator=g) for _ in range(3)]
    a = fm.ViewShardedFitter({k: torch.nn.Parameter(v.detach().clone()) for k, v in params.items()}, cams, targets, W,
                             H, reorder=False)
    b = fm.ViewShardedFitter({k: torch.nn.Parameter(v.detach().clone()) for k, v in params.items()}, cams, targets, W,
                             H, reorder=True)
    perm = fm.morton_order(params["means"])
    la, lb = float(a.step()), float(b.step())
    assert abs(la - lb) <= 1e-6 * max(1.0, abs(la))
    for k in params:
        torch.testing.assert_close(a.params[k].detach()[perm], b.params[k].detach(), rtol=1e-5, atol=1e-6)


def test_densify_sees_the_stub_order():
    """The trainer's permutation is invisible to densify/prune and to gaussians_fitted.npz: densify runs
    on canonical_params() (the stub's order, so top-k ties and jitter draws match the stub) and the
    result is re-permuted."""
    torch.manual_seed(11)
    params = fm.build_params(200, torch.device("cpu"), use_sh=False)
    with torch.no_grad():  # many exact ties in opacity, as after a few Adam steps
        params["opacities_raw"].copy_(-2.2 + 0.02 * torch.randint(-2, 3, (200,)).float())
    W, H = 16, 12
    cams = fm.orbit_cameras(2, W, H, torch.device("cpu"))
    targets = [torch.zeros((H, W, 3)) for _ in range(2)]
    f = fm.ViewShardedFitter({k: torch.nn.Parameter(v.detach().clone()) for k, v in params.items()}, cams, targets, W, H,
                             reorder=True)
    canon = f.canonical_params()
    for k in params:
        assert torch.equal(canon[k].detach(), params[k].detach())
    torch.manual_seed(5)
    ref = fm.densify_and_prune({k: torch.nn.Parameter(v.detach().clone()) for k, v in params.items()}, 400, 0.15, 0.05)
    torch.manual_seed(5)
    f.densify_and_prune(400, 0.15, 0.05, on_device=False)
    got = f.canonical_params()
    for k in ref:
        assert torch.equal(got[k].detach(), ref[k].detach()), k
    assert torch.equal(torch.sort(f.perm).values, torch.arange(ref["means"].shape[0]))


def test_respatialize_keeps_the_fit():
    """Re-establishing the Morton order mid-fit (ViewShardedFitter.respatialize, every RESORT_EVERY steps)
    permutes parameters and Adam moments together: the fit continues exactly as without it, and the
    canonical (stub-order) parameters are unchanged by the permutation."""
    torch.manual_seed(7)
    params = fm.build_params(60, torch.device("cpu"), use_sh=False)
    with torch.no_grad():
        params["scales_raw"].fill_(-1.0)
    W, H = 16, 12
    cams = fm.orbit_cameras(3, W, H, torch.device("cpu"))
    g = torch.Generator().manual_seed(3)
    targets = [torch.rand((H, W, 3), generator=g) for _ in range(3)]
    saved = fm.RESORT_EVERY
    try:
        fm.RESORT_EVERY = 0
        a = fm.ViewShardedFitter({k: torch.nn.Parameter(v.detach().clone()) for k, v in params.items()}, cams, targets, W, H)
        b = fm.ViewShardedFitter({k: torch.nn.Parameter(v.detach().clone()) for k, v in params.items()}, cams, targets, W, H)
        for _ in range(3):
            a.step()
            b.step()
        with torch.no_grad():  # move b's Gaussians out of order, as a long fit does
            for f in (a, b):
                f.params["means"].mul_(-1.0)
        before = {k: v.detach().clone() for k, v in b.canonical_params().items()}
        b.respatialize()
        after = b.canonical_params()
        for k in before:
            assert torch.equal(before[k], after[k].detach()), k
        assert torch.equal(b.perm.sort().values, torch.arange(60))
        for _ in range(2):
            la, lb = float(a.step()), float(b.step())
            assert abs(la - lb) <= 1e-6 * max(1.0, abs(la))
        ca, cb = a.canonical_params(), b.canonical_params()
        for k in ca:
            torch.testing.assert_close(ca[k].detach(), cb[k].detach(), rtol=1e-5, atol=1e-6)
    finally:
        fm.RESORT_EVERY = saved
