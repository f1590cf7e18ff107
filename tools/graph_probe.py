"""Where the graph-replayed fit step's time goes (C2 / C3 of tools/bench_configs.py): captures, replay time with the
host waiting, the step's wall time back to back, against the eager step.
Usage: python tools/graph_probe.py [C2|C3] [steps]"""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

bc = importlib.import_module("tools.bench_configs") if False else None
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import bench_configs as bc  # noqa: E402

fm = bc.fm
name = sys.argv[1] if len(sys.argv) > 1 else "C3"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
c = bc.CONFIGS[name]
dev = torch.device("cuda:0")


def fitter():
    params = bc.params_for(c["n"], c["sh"], dev)
    cams = fm.orbit_cameras(c["views"], c["w"], c["h"], dev)
    g = torch.Generator(device=dev).manual_seed(1)
    targets = [torch.rand((c["h"], c["w"], 3), generator=g, device=dev) for _ in range(c["views"])]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    depths = [torch.rand((c["h"], c["w"]), generator=g, device=dev) for _ in range(c["views"])] if c["depth"] else None
    return fm.ViewShardedFitter(params, cams, targets, c["w"], c["h"], lr=0.02, masks=masks, depths=depths)


for graph in [m == "1" for m in os.environ.get("PROBE_MODES", "01")]:
    fm.GRAPH_MODE = os.environ.get("GR_GRAPH", "1") if graph else "0"
    f = fitter()
    f.step(); f.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        f.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    # host time of one step() call (no sync), then its GPU time
    per = []
    for _ in range(5):
        torch.cuda.synchronize()
        a = time.perf_counter()
        f.step()
        b = time.perf_counter()
        torch.cuda.synchronize()
        e = time.perf_counter()
        per.append((1e3 * (b - a), 1e3 * (e - a)))
    gs = getattr(f, "_gs", None)
    extra = ""
    if graph and gs is not None:
        torch.cuda.synchronize()
        a = time.perf_counter()
        for _ in range(10):
            gs.graph.replay()
        b = time.perf_counter()
        torch.cuda.synchronize()
        e = time.perf_counter()
        extra = (f" builds {gs.builds} overflows {gs.overflows}; 10 bare replays: host {1e3 * (b - a) / 10:.3f} ms each, "
                 f"wall {1e3 * (e - a) / 10:.3f} ms each; caps {[int(x.num_pairs) for x in gs.caps]} "
                 f"observed {[int(r[0]) for r in gs.observed.tolist()]}")
    print(f"{name} graph={graph}: {1e3 * dt:.3f} ms/step back to back; single step (host call, wall) ms: "
          f"{[(round(x, 3), round(y, 3)) for x, y in per]}{extra}", flush=True)
