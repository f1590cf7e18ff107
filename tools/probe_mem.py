"""Allocator behaviour of the bench's fit step (device mallocs / retries per step, host time in Adam):
python tools/probe_mem.py  (GPU box)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

fm = bench.fm
device = torch.device("cuda", 0)
n, V, R = 1_000_000, 50, 800
params = bench.synthetic_params(n, device)
cams = fm.orbit_cameras(V, R, R, device)
g = torch.Generator(device=device).manual_seed(1)
targets = [torch.rand((R, R, 3), generator=g, device=device) for _ in range(V)]
masks = [(t.mean(dim=2) > 0.5).to(torch.float32) for t in targets]
fitter = fm.ViewShardedFitter(params, cams, targets, R, R, lr=0.02, masks=masks)
opt_step = fitter.opt.step
adam_host = []


def timed_step(*a, **k):
    t = time.perf_counter()
    r = opt_step(*a, **k)
    adam_host.append(time.perf_counter() - t)
    return r


fitter.opt.step = timed_step
for i in range(int(os.environ.get("PROBE_STEPS", "6"))):
    s0 = torch.cuda.memory_stats()
    t = time.perf_counter()
    fitter.step()
    torch.cuda.synchronize()
    s1 = torch.cuda.memory_stats()
    print(f"step {i}: {1e3 * (time.perf_counter() - t):.1f} ms  adam host {1e3 * adam_host[-1]:.2f} ms  "
          f"device mallocs +{s1.get('num_device_alloc', 0) - s0.get('num_device_alloc', 0)}  "
          f"frees +{s1.get('num_device_free', 0) - s0.get('num_device_free', 0)}  "
          f"retries +{s1.get('num_alloc_retries', 0) - s0.get('num_alloc_retries', 0)}  "
          f"reserved {s1.get('reserved_bytes.all.current', 0) / 2**30:.2f} GiB  "
          f"allocated {s1.get('allocated_bytes.all.current', 0) / 2**30:.2f} GiB  "
          f"peak {s1.get('allocated_bytes.all.peak', 0) / 2**30:.2f} GiB", flush=True)
    torch.cuda.reset_peak_memory_stats()
