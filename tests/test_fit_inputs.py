"""CPU: the fused fit path's raw-pointer operands are checked (a permuted, float64 or
wrongly shaped target must raise or take the autograd path, never be read as the wrong bytes)."""
from __future__ import annotations

import importlib

import pytest
import torch


def test_check_operand_rejects_what_the_abi_would_misread(pkg):
    tr = pkg.torch_renderer
    dev = torch.device("cpu")
    ok = torch.zeros((4, 6, 3))
    tr._check_operand(ok, (4, 6, 3), "target", dev)
    tr._check_operand(None, (4, 6, 3), "mask", dev)
    for bad in (ok.double(), ok.permute(1, 0, 2).contiguous().permute(1, 0, 2), ok[:, :, :2], ok.reshape(4, 18)):
        with pytest.raises(ValueError):
            tr._check_operand(bad, (4, 6, 3), "target", dev)


def test_fit_images_normalise_or_fall_back():
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    t = torch.rand((3, 4, 5)).double().permute(1, 0, 2)  # (4,3,5) non-contiguous float64
    imgs, ok = fm._fit_images("targets", [t], (4, 3, 5), torch.device("cpu"))
    assert ok and imgs[0].dtype == torch.float32 and imgs[0].is_contiguous()
    assert torch.equal(imgs[0], t.float())
    imgs, ok = fm._fit_images("masks", [torch.zeros((4, 3, 1))], (4, 3), torch.device("cpu"))
    assert not ok  # (H,W,1) broadcasts in the stub's expression: the autograd path keeps that meaning
    assert fm._fit_images("depths", None, (4, 3), torch.device("cpu")) == (None, True)
