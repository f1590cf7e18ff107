"""GPU: the native fit executor (gr_fit_views, 3dgaussian_amd/csrc/gr_fit_exec.cpp) runs the Python
driver's per-view schedule (fit_multiview._views_direct / _views_direct_depth: streams, preparation
groups, reduction batches) and gives bit-identical losses and parameters after a fit step."""
from __future__ import annotations

import ctypes
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
    saved = fm.NATIVE_EXEC, fm.NUM_STREAMS, fm.GRAPH_MODE
    try:
        for native in (False, True):
            # the eager schedules every step (not the default's batched steps for views this small)
            fm.NATIVE_EXEC, fm.NUM_STREAMS, fm.GRAPH_MODE = ("1" if native else "0"), streams, "0"
            f = fm.ViewShardedFitter(bench.synthetic_params(50_000, cuda), cams, targets, W, H, masks=masks, depths=depths)
            losses = [float(f.step()) for _ in range(2)]
            res[native] = (losses, {k: v.detach().clone() for k, v in f.params.items()})
    finally:
        fm.NATIVE_EXEC, fm.NUM_STREAMS, fm.GRAPH_MODE = saved
    assert res[True][0] == res[False][0]
    # the default ("auto") takes the native executor for views this small
    f = fm.ViewShardedFitter(bench.synthetic_params(1000, cuda), cams, targets, W, H)
    assert fm.NATIVE_EXEC != "auto" or f._native_exec()
    for k in res[False][1]:
        assert torch.equal(res[True][1][k], res[False][1][k]), k


def test_native_executor_at_c4_size(cuda):
    """The size at which the executor's first design faulted (commit 3f15cae: cross-stream pool reuse at C4):
    1M Gaussians, 13 views of 800x800 (several views per stream and a second reduction batch), two steps, the
    second one reusing every workspace and geom slot; bit-identical to the Python schedule."""
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    R, V = 800, 13
    cams = fm.orbit_cameras(V, R, R, cuda)
    g = torch.Generator(device=cuda).manual_seed(4)
    targets = [torch.rand((R, R, 3), generator=g, device=cuda) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    res = {}
    saved = fm.NATIVE_EXEC, fm.REDUCE_BATCH
    try:
        for native in (False, True):
            fm.NATIVE_EXEC, fm.REDUCE_BATCH = ("1" if native else "0"), 2
            f = fm.ViewShardedFitter(bench.synthetic_params(1_000_000, cuda), cams, targets, R, R, masks=masks)
            losses = [float(f.step()) for _ in range(2)]
            torch.cuda.synchronize()
            res[native] = (losses, {k: v.detach().clone() for k, v in f.params.items()})
            del f
            torch.cuda.empty_cache()
    finally:
        fm.NATIVE_EXEC, fm.REDUCE_BATCH = saved
    assert res[True][0] == res[False][0]
    for k in res[False][1]:
        assert torch.equal(res[True][1][k], res[False][1][k]), k


def test_native_executor_rejects_out_of_range_config(pkg, cuda):
    """a configuration whose batches or preparation groups would not fit the fixed-size view arrays
    returns GR_ERR_INVALID_ARGUMENT (raised as ValueError) before anything is enqueued."""
    tr = pkg.torch_renderer
    nat = pkg._native
    L = nat.lib()
    n = 64
    p = [torch.zeros((n, 3), device=cuda), torch.ones((n, 3), device=cuda), torch.zeros((n, 3), device=cuda),
         torch.zeros((n,), device=cuda)]
    cam = importlib.import_module("3dgaussian_amd.fit_multiview").orbit_cameras(1, 32, 32, cuda)[0]
    tgt = torch.zeros((32, 32, 3), device=cuda)
    arr = (nat.GrFitTarget * 1)()
    arr[0].view = tr.make_view(cam.view, cam.proj, 32, 32, None, depth_grad=False)
    arr[0].target_rgb = tgt.data_ptr()
    acc = [torch.empty_like(t) for t in p]
    accp = (ctypes.c_void_p * 4)(*[t.data_ptr() for t in acc])
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    losses = torch.empty(1, device=cuda)
    bad = [dict(reduce_tail=17), dict(reduce_tail=5, reduce_batch=4), dict(prep_first=9), dict(prep_group=9),
           dict(reduce_batch=17)]
    for b in bad:
        c = dict(num_streams=1, prep_ahead=2, prep_group=2, prep_first=1, reduce_batch=4, reduce_tail=0)
        c.update(b)
        cfg = nat.GrFitConfig(c["num_streams"], c["prep_ahead"], c["prep_group"], c["prep_first"], c["reduce_batch"],
                              c["reduce_tail"])
        st = L.gr_fit_views(nat.executor(0), ctypes.byref(cfg), 1, arr, n, *[nat.ptr(t) for t in p[:3]], 3, nat.ptr(p[3]),
                            0.0, 0.0, 1.0, nat.ptr(losses), accp, stream)
        assert st == nat.GR_ERR_INVALID_ARGUMENT, (b, st)


def test_fit_step_is_deterministic_at_c4_size(cuda):
    """Round 6: the same fused fit step run twice from the same state (1M Gaussians, 13 views of 800x800, two steps,
    the Python schedule at 4 streams) leaves bit-identical parameters.  A reordering that left an inline-asm
    v_fma_mix without its wait state made the backward's operands timing-dependent: the losses still agreed, the updated
    means did not (profiles/r06_determinism.txt)."""
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    R, V = 800, 13
    cams = fm.orbit_cameras(V, R, R, cuda)
    g = torch.Generator(device=cuda).manual_seed(4)
    targets = [torch.rand((R, R, 3), generator=g, device=cuda) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    runs = []
    saved = fm.NATIVE_EXEC
    try:
        fm.NATIVE_EXEC = "0"
        for _ in range(2):
            f = fm.ViewShardedFitter(bench.synthetic_params(1_000_000, cuda), cams, targets, R, R, masks=masks)
            losses = [float(f.step()) for _ in range(2)]
            torch.cuda.synchronize()
            runs.append((losses, {k: v.detach().clone() for k, v in f.params.items()}))
            del f
            torch.cuda.empty_cache()
    finally:
        fm.NATIVE_EXEC = saved
    assert runs[0][0] == runs[1][0]
    for k in runs[0][1]:
        assert torch.equal(runs[0][1][k], runs[1][1][k]), k
