"""GPU, world_size 2 on one card (gloo carries the collectives on device tensors): the fused parameter
step's multi-rank form (gradient assembly into the flat all-reduce buffer, the all-reduce, gr_adam_step)
gives the parameters the autograd + torch.optim.Adam path gives, and identical parameters on every rank.
The driver's 8-GPU bench runs the same code with RCCL."""
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

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, REPO)
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    cuda = torch.device("cuda:0")
    W, H = 128, 96
    cams = fm.orbit_cameras(4, W, H, cuda)
    g = torch.Generator(device=cuda).manual_seed(9)
    targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in cams]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    out = {}
    for fused in (False, True):
        fm.FUSED_STEP = fused
        f = fm.ViewShardedFitter(bench.synthetic_params(20_000, cuda), cams, targets, W, H, masks=masks)
        losses = [float(f.step()) for _ in range(3)]
        torch.cuda.synchronize()
        out[fused] = (losses, {k: v.detach().cpu().numpy().copy() for k, v in f.params.items()})
    out_q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_two_rank_fused_step_matches_torch_adam(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=200) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        (la, pa), (lf, pf) = res[r][False], res[r][True]
        np.testing.assert_allclose(lf, la, rtol=2e-6)
        for k in pa:
            err = float(np.linalg.norm(pf[k] - pa[k]) / np.linalg.norm(pa[k]))
            assert err <= 1e-6, (r, k, err)
    for k in res[0][True][1]:
        assert (res[0][True][1][k] == res[1][True][1][k]).all(), k
    assert res[0][True][0] == res[1][True][0]
