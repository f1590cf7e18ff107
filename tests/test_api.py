"""CPU: the drop-in Python surface keeps the reference's signatures, results and errors
(torch_renderer.py:10-138, bindings.cpp:15-70) without touching a GPU."""
from __future__ import annotations

import inspect

import numpy as np
import pytest
import torch

from conftest import golden


def test_signature_matches_reference(pkg):
    sig = inspect.signature(pkg.torch_renderer.render_gaussians_torch)
    names = list(sig.parameters)
    assert names[:11] == ["means", "scales", "colors", "opacities", "camera", "width", "height", "background",
                          "max_gaussians", "chunk_size", "return_aux"]
    assert sig.parameters["max_gaussians"].default == 10000
    assert sig.parameters["chunk_size"].default == 256
    assert sig.parameters["return_aux"].default is False


def test_perspective_and_look_at_match_reference_math(pkg):
    tr = pkg.torch_renderer
    d = golden("f2_c1_view2")
    P = tr.perspective(60.0, 1.0, 0.01, 100.0)
    np.testing.assert_allclose(P.numpy(), d["proj"], rtol=1e-6, atol=1e-7)
    import math

    yaw = 2.0 * math.pi * 2 / 4
    eye = torch.tensor([2.5 * math.cos(0.2) * math.sin(yaw), 2.5 * math.sin(0.2), 2.5 * math.cos(0.2) * math.cos(yaw)])
    V = tr.look_at(eye, torch.zeros(3), torch.tensor([0.0, 1.0, 0.0]))
    np.testing.assert_allclose(V.numpy(), d["view"], rtol=1e-6, atol=1e-6)


def _cam(pkg):
    return pkg.torch_renderer.Camera(view=torch.eye(4), proj=torch.eye(4))


def test_errors_match_reference(pkg):
    tr = pkg.torch_renderer
    with pytest.raises(ValueError, match=r"means must be \(N,3\)"):
        tr.render_gaussians_torch(torch.zeros(5, 2), torch.zeros(5, 3), torch.zeros(5, 3), torch.zeros(5), _cam(pkg), 8, 8)
    with pytest.raises(ValueError, match="too large for torch reference renderer"):
        tr.render_gaussians_torch(torch.zeros(11, 3), torch.zeros(11, 3), torch.zeros(11, 3), torch.zeros(11), _cam(pkg),
                                  8, 8, max_gaussians=10)
    with pytest.raises(ValueError, match=r"colors must be \(N,3\) or SH coeffs \(N,4,3\)"):
        tr.render_gaussians_torch(torch.zeros(4, 3), torch.zeros(4, 3), torch.zeros(4, 5), torch.zeros(4), _cam(pkg), 8, 8)


def test_zero_gaussians_returns_single_zero_image(pkg):
    out = pkg.torch_renderer.render_gaussians_torch(torch.zeros(0, 3), torch.zeros(0, 3), torch.zeros(0, 3), torch.zeros(0),
                                                    _cam(pkg), 7, 5, return_aux=True)
    assert isinstance(out, torch.Tensor) and out.shape == (5, 7, 3) and not out.any()


def test_hip_inputs_refuse_cpu_tensors(pkg):
    """The HIP entry points never take host tensors (no silent fallback); render_gaussians_torch
    dispatches host tensors to cpu_renderer instead (tests/test_cpu_path.py)."""
    with pytest.raises(RuntimeError, match="HIP device"):
        pkg.torch_renderer._device_inputs(torch.zeros(3, 3), torch.ones(3, 3), torch.zeros(3, 3), torch.ones(3))


def test_device_policy_prefers_hip(pkg):
    dev = pkg.device_utils.get_default_device()
    assert dev.type == ("cuda" if torch.cuda.is_available() else dev.type)


def test_legacy_binding_validation(pkg):
    gr = pkg.gaussian_renderer
    m = np.zeros((3, 3), np.float32)
    s = np.ones((3, 3), np.float32)
    o = np.ones((3,), np.float32)
    eye = np.eye(4, dtype=np.float32)
    with pytest.raises(RuntimeError, match="means must be float32"):
        gr.render_gaussians(m.astype(np.float64), s, m, o, 8, 8, eye, eye)
    with pytest.raises(RuntimeError, match="scales must be C-contiguous"):
        gr.render_gaussians(m, np.asfortranarray(np.ones((3, 4), np.float32))[:, :3], m, o, 8, 8, eye, eye)
    with pytest.raises(RuntimeError, match=r"colors must be \(N,3\)"):
        gr.render_gaussians(m, s, np.zeros((3, 4), np.float32), o, 8, 8, eye, eye)
    with pytest.raises(RuntimeError, match=r"opacities must be \(N,\)"):
        gr.render_gaussians(m, s, m, np.ones((3, 1), np.float32), 8, 8, eye, eye)
    with pytest.raises(RuntimeError, match=r"view must be \(4,4\)"):
        gr.render_gaussians(m, s, m, o, 8, 8, np.eye(3, dtype=np.float32), eye)
    with pytest.raises(RuntimeError, match=r"background must be \(3,\)"):
        gr.render_gaussians(m, s, m, o, 8, 8, eye, eye, np.zeros(4, np.float32))
    with pytest.raises(RuntimeError, match="matching N"):
        gr.render_gaussians(m, s, m, np.ones((2,), np.float32), 8, 8, eye, eye)
    with pytest.raises(RuntimeError, match="must be a numpy array"):
        gr.render_gaussians([[0, 0, 0]], s, m, o, 8, 8, eye, eye)
    with pytest.raises(TypeError):
        gr.render_gaussians(m, s, m, o, 8, 8)


def test_flat_import_like_the_reference(monkeypatch):
    """The package directory works as a drop-in for the reference's python/ on sys.path."""
    import importlib
    import os
    import sys

    from conftest import REPO

    monkeypatch.syspath_prepend(os.path.join(REPO, "3dgaussian_amd"))
    for mod in ("torch_renderer", "device_utils", "_native"):
        sys.modules.pop(mod, None)
    m = importlib.import_module("torch_renderer")
    assert hasattr(m, "render_gaussians_torch") and hasattr(m, "Camera")
    assert importlib.import_module("device_utils").get_default_device() is not None
    for mod in ("torch_renderer", "device_utils", "_native"):
        sys.modules.pop(mod, None)
