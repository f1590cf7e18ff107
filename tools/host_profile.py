"""Host-side (Python) profile of the bench's fit step: cProfile over a few timed steps of the C4 workload,
top functions by own time and by cumulative time, plus the host time of one step's phases.
    python tools/host_profile.py [views] [steps]"""
import cProfile
import importlib
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

bench = importlib.import_module("bench")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")


def main():
    views = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    n, R = 1_000_000, 800
    params = bench.synthetic_params(n, dev)
    cams = fm.orbit_cameras(views, R, R, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    targets = [torch.rand((R, R, 3), generator=g, device=dev) for _ in range(views)]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    fit = fm.ViewShardedFitter(params, cams, targets, R, R, lr=0.02, masks=masks)
    for _ in range(3):
        fit.step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(steps):
        fit.step()
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{steps} steps: host {1e3 * (t1 - t0) / steps:.2f} ms/step enqueued, {1e3 * (t2 - t0) / steps:.2f} ms/step "
          f"with the device drained (profiled)")
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(30)
        print(s.getvalue())


if __name__ == "__main__":
    main()
