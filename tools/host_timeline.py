"""Diagnostic: host-side timeline of the C4 fit step (bench.py's workload): when the host enters and
leaves each phase of ViewShardedFitter.step, how long it blocks in Prepared.plan() (waiting for a view's
pair count), and a device-side marker (a CUDA event per phase) to compare the two clocks.
    python tools/host_timeline.py [steps]"""
import functools
import importlib
import sys
import time

import torch

sys.path.insert(0, ".")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
tr = importlib.import_module("3dgaussian_amd.torch_renderer")
bench = importlib.import_module("bench")
dev = torch.device("cuda:0")
n, V, R = 1_000_000, 50, 800
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4

log = []


def wrap(obj, name, label):
    f = getattr(obj, name)

    @functools.wraps(f)
    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        log.append((label, t0, time.perf_counter()))
        return r

    setattr(obj, name, g)


wrap(tr.Prepared, "plan", "plan_wait")
wrap(tr, "forward_l1_native", "fwd_l1")
wrap(tr, "backward_splat_native", "bwd_splat")
wrap(tr, "reduce_views_native", "reduce")
wrap(tr, "prepare_native", "prepare")
wrap(fm.ViewShardedFitter, "_fused_param_step", "param_step")
wrap(fm.ViewShardedFitter, "_views_direct", "views_direct")
wrap(fm, "activations", "activations")

params = bench.synthetic_params(n, dev)
cams = fm.orbit_cameras(V, R, R, dev)
g = torch.Generator(device=dev).manual_seed(1)
targets = [torch.rand((R, R, 3), generator=g, device=dev) for _ in range(V)]
masks = [(t.mean(dim=2) > 0.5).to(torch.float32) for t in targets]
fit = fm.ViewShardedFitter(params, cams, targets, R, R, lr=0.02, masks=masks)
for _ in range(3):
    fit.step()
torch.cuda.synchronize()
log.clear()
marks = []
t_start = time.perf_counter()
for s in range(steps):
    t0 = time.perf_counter()
    fit.step()
    e = torch.cuda.Event()
    e.record()
    marks.append((t0, time.perf_counter(), e))
torch.cuda.synchronize()
t_end = time.perf_counter()
print(f"{steps} steps: {1e3 * (t_end - t_start) / steps:.2f} ms per step (host wall incl. final sync)")
for k, (a, b, e) in enumerate(marks):
    print(f"step {k}: host in step() {1e3 * (b - a):.2f} ms (enter at {1e3 * (a - t_start):.2f} ms)")
tot = {}
for lab, a, b in log:
    tot.setdefault(lab, [0.0, 0])
    tot[lab][0] += b - a
    tot[lab][1] += 1
for lab, (t, c) in sorted(tot.items(), key=lambda x: -x[1][0]):
    print(f"  {lab:14s} calls {c:4d}  total {1e3 * t / steps:8.2f} ms/step  avg {1e6 * t / c:8.1f} us")
# the last step's phases in order, relative to its entry
a0 = marks[-1][0]
print("last step, host phases (ms from step entry):")
for lab, a, b in log:
    if a >= a0 and lab in ("activations", "views_direct", "param_step") or (a >= a0 and lab == "plan_wait" and b - a > 2e-4):
        print(f"  {lab:14s} {1e3 * (a - a0):8.2f} -> {1e3 * (b - a0):8.2f}")
