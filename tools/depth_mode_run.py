"""The bench's default-precision (depth-loss) fit step alone, for profiling: C4 with depth targets.
    python tools/depth_mode_run.py [steps] [views]     (GR_STREAMS=1 for single-stream kernel times)"""
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

bench = importlib.import_module("bench")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    views = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda", 0)
    R = 800
    params = bench.synthetic_params(1_000_000, dev)
    cams = fm.orbit_cameras(views, R, R, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    targets = [torch.rand((R, R, 3), generator=g, device=dev) for _ in range(views)]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    fit = fm.ViewShardedFitter(params, cams, targets, R, R, lr=0.02, masks=masks)
    gd = torch.Generator(device=dev).manual_seed(2)
    fit.depths = [torch.rand((R, R), generator=gd, device=dev) for _ in range(views)]
    fit.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fit.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"depth-loss step: {1e3 * dt:.2f} ms, {views * R * R / dt / 1e6:.1f} Mpx/s ({fm.NUM_STREAMS} streams)")


if __name__ == "__main__":
    main()
