"""CPU, world_size 2 over gloo: the view-sharded data-parallel fit (3dgaussian_amd/fit_multiview.py)
gives every rank the single-process gradient and keeps parameters identical across ranks, including
through densify/prune (decided on rank 0, broadcast).  On host tensors the drop-in render op runs
its CPU path (3dgaussian_amd/cpu_renderer.py) because this container has no GPU; the collective logic is
the same code the GPU bench runs with RCCL."""
from __future__ import annotations

import importlib
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _setup(n_views=4, n=40, W=16, H=12):
    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")

    torch.manual_seed(7)
    params = fm.build_params(n, torch.device("cpu"), use_sh=False)
    with torch.no_grad():
        params["scales_raw"].fill_(-1.0)
    cams = fm.orbit_cameras(n_views, W, H, torch.device("cpu"))
    g = torch.Generator().manual_seed(3)
    targets = [torch.rand((H, W, 3), generator=g) for _ in range(n_views)]
    masks = [(t.mean(2) > 0.5).float() for t in targets]
    return fm, params, cams, targets, masks, W, H


def _worker(rank, world, port, out_q, on_device=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fm, params, cams, targets, masks, W, H = _setup()
    fit = fm.ViewShardedFitter(params, cams, targets, W, H, masks=masks)
    losses = [float(fit.step()) for _ in range(2)]
    grads = {k: v.grad.clone() for k, v in fit.params.items()}
    before = {k: v.detach().numpy().copy() for k, v in fit.params.items()}
    torch.manual_seed(11)  # only rank 0's RNG decides the densify jitter
    fit.densify_and_prune(max_gaussians=60, densify_ratio=0.5, prune_opacity=0.05, on_device=on_device)
    losses.append(float(fit.step()))
    # numpy, not tensors: tensor shared-memory handles die with the worker process
    out_q.put((rank, losses, before, {k: v.detach().numpy().copy() for k, v in fit.params.items()},
               {k: v.numpy().copy() for k, v in grads.items()}))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("on_device", [False, True])
def test_two_rank_gloo_matches_single_process(on_device):
    """on_device: the device-side densify rule (the C5 path: generator on the parameters' device),
    decided on rank 0 and broadcast, as the host rule."""
    fm, params, cams, targets, masks, W, H = _setup()
    ref = fm.ViewShardedFitter(params, cams, targets, W, H, masks=masks)
    ref_losses = [float(ref.step()) for _ in range(2)]
    ref_grads = {k: v.grad.clone() for k, v in ref.params.items()}
    ref_params = {k: v.detach().clone() for k, v in ref.params.items()}

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, on_device)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (l, before, after, g)) for r, l, before, after, g in (q.get(timeout=240) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        losses, before, after, grads = res[r]
        # the full-loss value and gradient on every rank equal the single-process ones (up to the
        # summation order of the collective)
        for a, b in zip(losses[:2], ref_losses):
            assert abs(a - b) <= 1e-6 * max(1.0, abs(b))
        for k in ref_grads:
            torch.testing.assert_close(torch.from_numpy(grads[k]), ref_grads[k], rtol=1e-5, atol=1e-7)
        for k in ref_params:
            torch.testing.assert_close(torch.from_numpy(before[k]), ref_params[k], rtol=1e-5, atol=1e-6)
    # ranks hold bit-identical parameters after a broadcast densify/prune and one more step
    # (the densify top-k is not compared with the single-process run: near-tied opacities may
    # rank differently under a different summation order)
    assert res[0][0][2] == res[1][0][2]
    for k in res[0][2]:
        assert res[0][2][k].shape[0] > 40 and (res[0][2][k] == res[1][2][k]).all(), k


def _worker_edge(rank, world, port, out_q):
    """world > views (ranks with no views) and rank-dependent initial parameters."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fm, params, cams, targets, masks, W, H = _setup(n_views=2)
    with torch.no_grad():
        params["means"].add_(0.01 * rank)  # ranks disagree: rank 0's parameters must win
    fit = fm.ViewShardedFitter(params, cams, targets, W, H, masks=masks)
    losses = [float(fit.step()) for _ in range(2)]
    out_q.put((rank, len(fit.my_views), losses, {k: v.detach().numpy().copy() for k, v in fit.params.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_more_ranks_than_views_and_rank0_parameters_win():
    fm, params, cams, targets, masks, W, H = _setup(n_views=2)
    ref = fm.ViewShardedFitter(params, cams, targets, W, H, masks=masks)
    ref_losses = [float(ref.step()) for _ in range(2)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_edge, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = {r: (nv, l, prm) for r, nv, l, prm in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [res[r][0] for r in range(3)] == [1, 1, 0]
    for r in range(3):
        for a, b in zip(res[r][1], ref_losses):
            assert abs(a - b) <= 1e-6 * max(1.0, abs(b))
        for k in res[0][2]:
            assert (res[r][2][k] == res[0][2][k]).all(), (r, k)
        for k, v in ref.params.items():
            torch.testing.assert_close(torch.from_numpy(res[r][2][k]), v.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.timeout(300)
def test_bench_launcher_starts_ranks():
    """`python bench.py --gpus 2` with no torch.distributed environment starts 2 ranks itself (the
    driver's 1/2/4/8-GPU command); a host-tensor dry run over gloo checks the launch and the sharding."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--device", "cpu", "--gaussians", "200",
                        "--views", "5", "--res", "24", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["views_per_rank"] == [3, 2]
