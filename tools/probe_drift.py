"""Dev probe: how the bench workload drifts over a fit.  Runs bench.py's C4 fit for K steps and prints,
per step, the wall time, view 0's pair counts, the mean scale and the splat kernels' average launch times
(single stream).  Optionally re-establishes the Morton order at a given step (--resort S) to separate the
effect of the pair count from that of the Gaussians' layout drifting out of spatial order.

Usage: python tools/probe_drift.py [--steps 25] [--resort S] [--streams 1]
"""
import argparse, importlib, json, os, subprocess, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

pkg = importlib.import_module("3dgaussian_amd")
tr = pkg.torch_renderer
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
bench = importlib.import_module("bench")


def sclk():
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--json"], capture_output=True, text=True, timeout=20)
        d = json.loads(r.stdout)
        card = next(iter(d.values()))
        return {k: v for k, v in card.items() if "sclk" in k or "mclk" in k or "fclk" in k}
    except Exception as e:  # noqa: BLE001
        return {"err": str(e)[:80]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--resort", type=int, default=-1)
    ap.add_argument("--every", type=int, default=0, help="re-sort every k steps (probe of periodic re-layout)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, V, R = 1_000_000, 50, 800
    params = bench.synthetic_params(n, dev)
    cams = fm.orbit_cameras(V, R, R, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    targets = [torch.rand((R, R, 3), generator=g, device=dev) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).to(torch.float32) for t in targets]
    fit = fm.ViewShardedFitter(params, cams, targets, R, R, lr=0.02, masks=masks)
    print("clocks start", sclk(), flush=True)
    for s in range(args.steps):
        if s == args.resort or (args.every and s > 0 and s % args.every == 0):
            t0 = time.perf_counter()
            fit.respatialize() if hasattr(fit, "respatialize") else None
            torch.cuda.synchronize()
            print(f"  re-sorted at step {s} in {1e3*(time.perf_counter()-t0):.2f} ms", flush=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loss = fit.step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        line = f"step {s:3d} {1e3*dt:7.2f} ms  {V*R*R/dt/1e6:7.1f} Mpx/s  loss {float(loss):.5f}"
        if s % 4 == 0 or s == args.steps - 1:
            with torch.no_grad():
                means, scales, colors, opac = fm.activations(fit.params)
                gv = tr.make_view(cams[0].view, cams[0].proj, R, R, None, tr.DEFAULT_CUTOFF)
                _, _, _, st = tr.forward_native(means.contiguous(), scales.contiguous(), colors.contiguous(),
                                                opac.contiguous(), gv)
                line += f"  pairs {st.num_pairs} core {int(st.plan.num_core_pairs)} scale_mean {float(scales.mean()):.5f}"
            fm.NUM_STREAMS, ns = 1, fm.NUM_STREAMS
            torch.cuda.synchronize()
            pkg._native.profile_begin()
            fit.step()
            torch.cuda.synchronize()
            prof = pkg._native.profile_end()
            fm.NUM_STREAMS = ns
            f = prof["raster_fwd"]; b = prof["raster_bwd"]
            line += f"  [1-stream extra step: fwd {1e3*f[0]/max(f[1],1):.1f} us bwd {1e3*b[0]/max(b[1],1):.1f} us]"
        print(line, flush=True)
    print("clocks end", sclk(), flush=True)


if __name__ == "__main__":
    main()
