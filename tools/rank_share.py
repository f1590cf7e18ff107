"""Ranks' shares of the multi-GPU C4 step on one GPU: the step time of rank r of R with whole views round-robin
(7 views for rank 0 of 8) and with the leftover views in bands of tile rows (6 views and one band of a quarter view,
round 6), no collective (the step's update runs as at world size 1).
    python tools/rank_share.py [R] [r|all] [steps] [both|whole|bands]"""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

fm = importlib.import_module("3dgaussian_amd.fit_multiview")
bench = importlib.import_module("bench")
Rk = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ranks = list(range(int(sys.argv[1]) if len(sys.argv) > 1 else 8)) if (len(sys.argv) > 2 and sys.argv[2] == "all") else \
    [int(sys.argv[2]) if len(sys.argv) > 2 else 0]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda:0")
R, V, N = 800, 50, 1_000_000


class Share(fm.ViewShardedFitter):
    fixed = None

    @property
    def my_views(self):
        return self.fixed if self.fixed is not None else super().my_views


def run(band, rk):
    params = bench.synthetic_params(N, dev)
    cams = fm.orbit_cameras(V, R, R, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    targets = [torch.rand((R, R, 3), generator=g, device=dev) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    f = Share(params, cams, targets, R, R, lr=0.02, masks=masks)
    fm.BAND_SPLIT = band
    f.rank, f.world = rk, Rk
    f._rr_views = list(range(rk, V, Rk))
    views = list(f.my_views)
    f.rank, f.world = 0, 1
    f.fixed = views
    for _ in range(3):
        f.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        f.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(f"rank {rk} of {Rk}, {'bands' if band else 'whole views'}: {len([v for v in views if v < V])} views + "
          f"{len([v for v in views if v >= V])} bands {[f._bands[v] for v in views if v >= V]}: {1e3 * dt:.3f} ms per step",
          flush=True)
    del f
    torch.cuda.empty_cache()


mode = sys.argv[4] if len(sys.argv) > 4 else "both"
if mode in ("both", "whole"):
    run(False, ranks[0])
if mode in ("both", "bands"):
    for rk in ranks:
        run(True, rk)
