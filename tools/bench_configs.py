"""Mpx/s fwd+bwd of the fit step (bench.py's metric) at BASELINE.json's other configs, on one GPU:

  C2  100k Gaussians, 8 orbit views, 512x512, L1 + silhouette
  C3  50k Gaussians, SH degree 3, 8 orbit views, 256x256, L1 + silhouette + depth losses
  C5  3M Gaussians, 100 orbit views, 1920x1080, L1 + silhouette (1-GPU share of the 8-GPU config)
  C4d the C4 workload with the depth term (bench.py's default_precision_mode)
  C5d the C5 densify/prune loop: starts at 2.7M Gaussians and densifies (ratio 0.15, prune opacity 0.05,
      device rule, Morton re-layout, Adam reset; fit_multiview_stub.py:318-325) every 2 steps to 3M, the
      densify steps inside the timed region

Synthetic, seeded data as in bench.py (density-matched scales).  One JSON line per config.
Usage: python tools/bench_configs.py [C2 C3 C5] [--steps K]
"""
import importlib, json, math, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

pkg = importlib.import_module("3dgaussian_amd")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
bench = importlib.import_module("bench")

CONFIGS = {
    "C2": dict(n=100_000, views=8, w=512, h=512, sh=0, depth=False),
    "C3": dict(n=50_000, views=8, w=256, h=256, sh=3, depth=True),
    "C5": dict(n=3_000_000, views=100, w=1920, h=1080, sh=0, depth=False),
    "C4d": dict(n=1_000_000, views=50, w=800, h=800, sh=0, depth=True),  # bench.py's default_precision_mode workload
    "C5d": dict(n=2_700_000, views=100, w=1920, h=1080, sh=0, depth=False,
                densify=dict(every=2, max_gaussians=3_000_000, ratio=0.15, prune=0.05)),
}


def params_for(n, sh, dev):
    p = bench.synthetic_params(n, dev)
    if sh:
        g = torch.Generator().manual_seed(2)
        shc = torch.zeros((n, 16, 3))
        shc[:, 0, :] = torch.sigmoid(0.1 * torch.rand((n, 3), generator=g))
        shc[:, 1:, :] = 0.02 * torch.randn((n, 15, 3), generator=g)
        del p["colors_raw"]
        p["sh_raw"] = torch.nn.Parameter(shc.to(dev))
    return p


def run(name, steps, warmup=2):
    c = CONFIGS[name]
    dev = torch.device("cuda:0")
    params = params_for(c["n"], c["sh"], dev)
    cams = fm.orbit_cameras(c["views"], c["w"], c["h"], dev)
    g = torch.Generator(device=dev).manual_seed(1)
    targets = [torch.rand((c["h"], c["w"], 3), generator=g, device=dev) for _ in range(c["views"])]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    depths = [torch.rand((c["h"], c["w"]), generator=g, device=dev) for _ in range(c["views"])] if c["depth"] else None
    fitter = fm.ViewShardedFitter(params, cams, targets, c["w"], c["h"], lr=0.02, masks=masks, depths=depths)
    for _ in range(warmup):  # as bench.py's default warmup (the first steps grow the allocator's pools)
        fitter.step()
    torch.cuda.synchronize()
    dens = c.get("densify")
    n_dens = 0
    t0 = time.perf_counter()
    for i in range(steps):
        loss = fitter.step()
        if dens and (i + 1) % dens["every"] == 0:
            fitter.densify_and_prune(dens["max_gaussians"], dens["ratio"], dens["prune"])
            n_dens += 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    px = c["views"] * c["w"] * c["h"] * steps
    print(json.dumps({"config": name, "gaussians": c["n"], "views": c["views"], "width": c["w"], "height": c["h"],
                      "sh_degree": c["sh"] or None, "depth_loss": c["depth"], "steps": steps, "warmup": warmup,
                      "ms_per_step": round(1e3 * dt / steps, 2), "mpx_per_s": round(px / dt / 1e6, 1),
                      "loss": float(loss), "streams": fm.NUM_STREAMS, "densify_calls": n_dens,
                      "gaussians_at_end": int(fitter.params["means"].shape[0])}), flush=True)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 3
    warmup = int(sys.argv[sys.argv.index("--warmup") + 1]) if "--warmup" in sys.argv else 2
    for name in (args or ["C2", "C3", "C5", "C5d"]):
        if name in CONFIGS:
            run(name, steps, warmup)
