"""Host policy (no GPU): which fit steps take the native executor (fit_multiview.GR_NATIVE_EXEC)."""
from __future__ import annotations

import importlib

import pytest


@pytest.mark.parametrize("setting,size,expect", [
    ("auto", (512, 512), True),     # C2: host-bound small views -> gr_fit_views
    ("auto", (256, 256), True),     # C3
    ("auto", (800, 800), False),    # C4: GPU-bound, the Python schedule
    ("auto", (1920, 1080), False),  # C5
    ("0", (256, 256), False),
    ("1", (1920, 1080), True),
    (False, (256, 256), False),     # tests may set booleans
    (True, (800, 800), True),
])
def test_native_exec_policy(setting, size, expect):
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")

    class _F:
        width, height = size

    saved = fm.NATIVE_EXEC
    try:
        fm.NATIVE_EXEC = setting
        assert fm.ViewShardedFitter._native_exec(_F()) is expect
    finally:
        fm.NATIVE_EXEC = saved
