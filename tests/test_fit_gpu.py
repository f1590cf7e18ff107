"""GPU: the fit driver (3dgaussian_amd/fit_multiview.py, HIP render op) reproduces the loss curve
of the reference's unchanged fit_multiview_stub.py (golden F4: torch.manual_seed(1234), 300
Gaussians, 48x48, 3 synthetic targets, 6 iterations with densify/prune every 3)."""
from __future__ import annotations

import importlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden

pytestmark = pytest.mark.gpu


def test_fit_curve_matches_reference_stub(tmp_path, cuda):
    d = golden("f4_fit_curve")
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    fm.main(["--targets_dir", os.path.join(GOLDEN, "fit_targets"), "--out_dir", str(tmp_path), "--iters", str(int(d["iters"])),
             "--width", str(int(d["width"])), "--height", str(int(d["width"])), "--num_gaussians", str(int(d["num_gaussians"])),
             "--max_gaussians", str(int(d["max_gaussians"])), "--densify_interval", str(int(d["densify_interval"])),
             "--prune_interval", str(int(d["densify_interval"])), "--seed", str(int(d["seed"]))])
    losses = np.array([float(x) for x in (tmp_path / "loss.txt").read_text().split()])
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-4)
    npz = np.load(tmp_path / "gaussians_fitted.npz")
    assert set(npz.files) == {"means", "scales", "colors", "opacities"}
    assert (tmp_path / "preview_view0.png").exists()
