"""GPU: degree-3 colour (config C3's colour model) through the C ABI against the binned float64
oracle, at a small scene and at C3 size (50k Gaussians, 256x256), with depth and silhouette upstream
gradients."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as orc
from test_parity_gpu import CORE, DEPTH_CUTOFF, GRAD_KEYS

pytestmark = pytest.mark.gpu


def _sh3_scene(n, seed, scale):
    rng = np.random.default_rng(seed)
    sc = orc.synthetic_scene(n, seed=seed, scale=scale)
    sh = np.zeros((n, 16, 3), np.float32)
    sh[:, 0] = 0.3 + 0.4 * rng.random((n, 3))
    sh[:, 1:] = 0.1 * rng.standard_normal((n, 15, 3))
    return orc.Scene(sc.means, sc.scales, sh, sc.opacities)


@pytest.mark.parametrize("n,res,scale", [(300, 64, 0.1), (50_000, 256, 0.0306)])
def test_sh3_vs_binned_oracle(pkg, cuda, n, res, scale):
    tr = pkg.torch_renderer
    sc = _sh3_scene(n, 5, scale)
    view, proj = orc.orbit_cameras(8, res, res)[3]
    rng = np.random.default_rng(1)
    g_rgb = rng.standard_normal((res, res, 3)).astype(np.float32)
    g_a = rng.standard_normal((res, res)).astype(np.float32)
    g_d = rng.standard_normal((res, res)).astype(np.float32)
    t = [torch.from_numpy(a).to(cuda).requires_grad_(True) for a in sc.arrays()]
    out, alpha, depth = tr.rasterize(*t, view, proj, res, res)
    ((out * torch.from_numpy(g_rgb).to(cuda)).sum() + (alpha * torch.from_numpy(g_a).to(cuda)).sum()
     + (depth * torch.from_numpy(g_d).to(cuda)).sum()).backward()
    v = orc.make_view(view, proj, res, res, cutoff=DEPTH_CUTOFF, core_cutoff=CORE)
    o_out, o_a, o_d = orc.forward(v, sc, binned=True)
    grads = orc.backward(v, sc, g_rgb, g_a, g_d, binned=True)
    for got, ref in ((out, o_out), (alpha, o_a), (depth, o_d)):
        assert orc.rel_l2(got.detach().cpu().numpy(), ref) <= 2e-5
    for name, tt, g in zip(GRAD_KEYS, t, grads):
        assert orc.rel_l2(tt.grad.cpu().numpy(), g) <= 1e-4, name
    assert t[2].grad.shape == (n, 16, 3)
