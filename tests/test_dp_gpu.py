"""GPU, world size 2 over gloo with both ranks on cuda:0: the view-sharded fit on the HIP fused path (the bench's
multi-GPU code: per-rank views with the leftover view in bands of tile rows, the gradient assembly into the flat
buffer, the bucketed all-reduce of HIP tensors, Adam per bucket) gives both ranks identical parameters, equal to
the single-process fit within float summation order.  (RCCL needs one GPU per rank; gloo carries the same
collective calls here.)"""
from __future__ import annotations

import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
V, W, H, N = 5, 256, 224, 40_000


def _fit(rank, world):
    sys.path.insert(0, REPO)
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    dev = torch.device("cuda:0")
    params = bench.synthetic_params(N, dev)
    cams = fm.orbit_cameras(V, W, H, dev)
    g = torch.Generator(device=dev).manual_seed(5)
    targets = [torch.rand((H, W, 3), generator=g, device=dev) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    fm.GRAPH_MODE = "0"  # (the graph modes run at world size 1 only: the same eager step on both sides)
    fm.BAND_OVERHEAD = 0.0  # bands whatever they cost: the band path is what this test runs on two ranks
    fit = fm.ViewShardedFitter(params, cams, targets, W, H, lr=0.02, masks=masks)
    views = list(fit.my_views)
    losses = [float(fit.step()) for _ in range(3)]
    torch.cuda.synchronize()
    return losses, {k: v.detach().cpu().numpy().copy() for k, v in fit.params.items()}, views


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out_q.put((rank,) + _fit(rank, world))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        out_q.put((rank, repr(e), None, None))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_two_ranks_on_one_gpu_match_single_process(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, losses, params, views = q.get(timeout=240)
        assert params is not None, losses
        res[r] = (losses, params, views)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_losses, ref_params, _ = _fit(0, 1)
    print("rank views:", res[0][2], res[1][2], "losses:", res[0][0], "single:", ref_losses)
    assert any(v >= V for v in res[0][2]) and any(v >= V for v in res[1][2])  # the fifth view in two bands
    assert res[0][0] == res[1][0]  # the all-reduced loss
    np.testing.assert_allclose(res[0][0], ref_losses, rtol=1e-6)
    for k in ref_params:
        assert np.array_equal(res[0][1][k], res[1][1][k]), k  # replicas identical
        err = float(np.linalg.norm(res[0][1][k] - ref_params[k]) / np.linalg.norm(ref_params[k]))
        assert err <= 1e-6, (k, err)
