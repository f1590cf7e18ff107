"""GPU: the fused fit-loop L1 loss (3dgaussian_amd/losses.py, gr_l1_loss_* in libgr_hip.so) against
the torch expression of python/fit_multiview_stub.py:292-299."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,w2", [((64, 48, 3), 0.2), ((800, 800, 3), 0.2), ((17, 13, 3), 0.0), ((1, 1, 3), 1.5)])
def test_l1_loss_matches_torch(pkg, cuda, shape, w2):
    g = torch.Generator(device=cuda).manual_seed(3)
    a = torch.rand(shape, generator=g, device=cuda).requires_grad_(True)
    b = torch.rand(shape, generator=g, device=cuda)
    b[0, 0] = a[0, 0].detach()  # exact ties: sign(0) = 0 in both
    c = torch.rand(shape[:2], generator=g, device=cuda).requires_grad_(True)
    d = (torch.rand(shape[:2], generator=g, device=cuda) > 0.5).float()
    if w2 > 0:
        got = pkg.losses.l1_loss(a, b, c, d, w2)
        ref = torch.mean(torch.abs(a - b)) + w2 * torch.mean(torch.abs(c - d))
    else:
        got = pkg.losses.l1_loss(a, b)
        ref = torch.mean(torch.abs(a - b))
    assert abs(float(got) - float(ref)) <= 2e-6 * max(1.0, abs(float(ref)))
    ga, gc = torch.autograd.grad(3.0 * got, [a, c], allow_unused=True)
    ra, rc = torch.autograd.grad(3.0 * ref, [a, c], allow_unused=True)
    torch.testing.assert_close(ga, ra, rtol=1e-6, atol=0)
    if w2 > 0:
        torch.testing.assert_close(gc, rc, rtol=1e-6, atol=0)
    # deterministic
    assert float(pkg.losses.l1_loss(a, b, c, d, w2)) == float(pkg.losses.l1_loss(a, b, c, d, w2))
