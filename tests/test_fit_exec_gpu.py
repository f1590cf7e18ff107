"""GPU: the native fit executor (gr_fit_views, 3dgaussian_amd/csrc/gr_fit_exec.cpp) runs the Python
driver's per-view schedule (fit_multiview._views_direct / _views_direct_depth: streams, preparation
groups, reduction batches) and gives bit-identical losses and parameters after a fit step."""
from __future__ import annotations

import importlib

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("streams", [1, 4])
@pytest.mark.parametrize("depth", [False, True])
def test_native_executor_matches_python_schedule(cuda, streams, depth):
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W, H, V = 256, 192, 11
    cams = fm.orbit_cameras(V, W, H, cuda)
    g = torch.Generator(device=cuda).manual_seed(21)
    targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    depths = [torch.rand((H, W), generator=g, device=cuda) for _ in range(V)] if depth else None
    res = {}
    saved = fm.NATIVE_EXEC, fm.NUM_STREAMS
    try:
        for native in (False, True):
            fm.NATIVE_EXEC, fm.NUM_STREAMS = ("1" if native else "0"), streams
            f = fm.ViewShardedFitter(bench.synthetic_params(50_000, cuda), cams, targets, W, H, masks=masks, depths=depths)
            losses = [float(f.step()) for _ in range(2)]
            res[native] = (losses, {k: v.detach().clone() for k, v in f.params.items()})
    finally:
        fm.NATIVE_EXEC, fm.NUM_STREAMS = saved
    assert res[True][0] == res[False][0]
    # the default ("auto") takes the native executor for views this small
    f = fm.ViewShardedFitter(bench.synthetic_params(1000, cuda), cams, targets, W, H)
    assert fm.NATIVE_EXEC != "auto" or f._native_exec()
    for k in res[False][1]:
        assert torch.equal(res[True][1][k], res[False][1][k]), k
