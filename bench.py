"""Benchmark of the MI355X render op on BASELINE.json's headline workload.

Metric: "Mpixels/sec fwd+bwd @1M Gaussians 800x800" (BASELINE.json).  Workload = config C4:
1M Gaussians, 50 orbit views of 800x800, views sharded across ranks (rank r renders views
r, r+R, ...), one RCCL all_reduce of the flat gradient buffer per step.

One step = one fit iteration of fit_multiview_stub.py:265-311 over the 50 views: activations, HIP
forward of this rank's views, L1 + silhouette losses, HIP backward, gradient all-reduce, Adam.
value = 50 * 800 * 800 * steps / max-over-ranks wall time (whole job, Mpx/s); total work is fixed
as N grows -> "scaling": "strong".

Synthetic data (no network): means ~ U(-0.6,0.6)^3, opacity sigmoid(-2.2), colours sigmoid(0.1 U),
density-matched scale 0.1061*(1200/N)^(1/3); targets are seeded random images.

Also reported on rank 0:
  roofline      the dominant kernel (the splat kernel with the longer launches, forward or backward; both
                under "splats"), timed live with HIP events
                on its launch stream (gr_profile_begin/end) over one single-stream step after the timed
                region (the timed steps overlap views on 3 streams): MFMA FLOP per launch (split-bf16
                formulation) / average launch time, against the bf16 dense peak, with the
                f32-equivalent rate beside it; plus its HBM traffic from rocprofv3 PMC counters when
                profiles/pmc_traffic.json exists (tools/pmc_traffic.py).
  hbm_model     the north_star's framing: SURVEY.md §8(d)'s byte model of the tile-binned path at the
                measured pairs per view, and the bench value as a fraction of its 8 TB/s roofline.
  cpu_baseline  the CPU oracle (oracle/gr_oracle.c, OpenMP) on one view of the same workload.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
     --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import importlib
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

pkg = importlib.import_module("3dgaussian_amd")
tr = pkg.torch_renderer
fm = importlib.import_module("3dgaussian_amd.fit_multiview")

F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 (f32-in MFMA) dense peak
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA dense peak
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E peak (spec)
MFMA_32x32x16 = 2 * 32 * 32 * 16  # FLOP of one v_mfma_f32_32x32x16_bf16
# Backward splat without an upstream depth gradient (the bench's loss: L1 + silhouette; the fit driver
# renders its views with depth_grad=False), per core pair: two K = 16 contractions (over
# x and over y) of 4 upstream channels,
#   f32-equivalent (algorithmic) FLOP = 2 sides x 4 channels x 16 x 16 x 2 = 4096,
#   executed on the bf16 pipe as two-piece splits: 2 sides x 2 channel pairs x 3 piece products of
#   v_mfma_f32_32x32x16_bf16 per 32 pairs = 12,288 FLOP per pair.
F32_FLOP_PER_CORE_PAIR_BWD = 2 * 4 * 16 * 16 * 2
BF16_FLOP_PER_CORE_PAIR_BWD = 2 * 2 * 3 * MFMA_32x32x16 / 32
# Forward splat, f32-equivalent: 5 channels (core) / 2 channels (tail) x 16 x 16 x 2 per pair; executed
# (depth_grad=False: two pieces, 3 products of v_mfma_f32_16x16x32_bf16 per channel per 32 pairs).
F32_FLOP_PER_CORE_PAIR_FWD = 5 * 16 * 16 * 2
F32_FLOP_PER_TAIL_PAIR_FWD = 2 * 16 * 16 * 2
MFMA_16x16x32 = 2 * 16 * 16 * 32
BF16_FLOP_PER_CORE_PAIR_FWD = 5 * 3 * MFMA_16x16x32 / 32
BF16_FLOP_PER_TAIL_PAIR_FWD = 2 * 3 * MFMA_16x16x32 / 32
FWD_KERNEL = "k_raster_fwd_mfma"
BWD_KERNEL = "k_raster_bwd_mfma" if os.environ.get("GR_BWD_F32") == "1" else "k_raster_bwd_bf16"
# SURVEY.md §8(d) HBM model of the tile-binned algorithm (the north_star's "fraction of the HBM
# roofline" framing): bytes per view = N (3 B_in + 2 x 36) + K (2 x 12 + 2 x 36 + 2 x 36) + 60 H W
# with B_in = 40 (RGB), K = pairs per view as binned here.
B_IN_RGB = 40


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--views", type=int, default=50)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-reorder", action="store_true",
                    help="keep the synthetic Gaussians in their random order (A/B of the trainer's Morton order)")
    return ap.parse_args()


def synthetic_params(n: int, device) -> dict:
    g = torch.Generator().manual_seed(0)
    means = (torch.rand((n, 3), generator=g) - 0.5) * 1.2
    scale = 0.1061 * (1200.0 / n) ** (1.0 / 3.0)
    scales_raw = torch.full((n, 3), math.log(math.expm1(scale - 1e-3)))  # softplus^-1(scale - 1e-3)
    op_raw = torch.full((n,), -2.2)
    colors_raw = 0.1 * torch.rand((n, 3), generator=g)
    p = {"means": means, "scales_raw": scales_raw, "opacities_raw": op_raw, "colors_raw": colors_raw}
    return {k: torch.nn.Parameter(v.to(device)) for k, v in p.items()}


def cpu_baseline(n: int, res: int, views: int) -> dict:
    """Oracle port (float64 accumulation, OpenMP over the host cores) on ONE view of the workload."""
    from oracle import oracle as orc

    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    scene = orc.synthetic_scene(n, seed=0)
    view, proj = orc.orbit_cameras(views, res, res)[0]
    v = orc.make_view(view, proj, res, res, cutoff=tr.DEFAULT_CUTOFF, core_cutoff=tr.DEFAULT_CORE_CUTOFF)
    g = np.random.default_rng(0).standard_normal((res, res, 3)).astype(np.float32)
    t0 = time.perf_counter()
    orc.forward(v, scene, binned=True)
    orc.backward(v, scene, g, None, None, binned=True)
    dt = time.perf_counter() - t0
    return {"value": round(res * res / dt / 1e6, 5), "unit": "Mpixels/sec fwd+bwd", "cores": cores, "kind": "port",
            "sample": f"1 view of the workload ({n} Gaussians, {res}x{res}), oracle/gr_oracle.c binned fwd+bwd, "
                      f"OpenMP {cores} threads, {dt:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    n, V, R = args.gaussians, args.views, args.res

    params = synthetic_params(n, device)
    cams = fm.orbit_cameras(V, R, R, device)
    g = torch.Generator(device=device).manual_seed(1)
    targets = [torch.rand((R, R, 3), generator=g, device=device) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).to(torch.float32) for t in targets]
    fitter = fm.ViewShardedFitter(params, cams, targets, R, R, lr=0.02, masks=masks, reorder=not args.no_reorder)

    for _ in range(args.warmup):
        fitter.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    pkg._native.profile_begin()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = fitter.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    prof_concurrent = pkg._native.profile_end()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=device)
    # Roofline pass: the timed steps rotate views over several HIP streams, so a launch's duration
    # there includes kernels of other views running beside it.  One more step on a single stream gives
    # each launch its own duration (with GR_STREAMS=1 the whole run is single-stream and both agree).
    streams_saved = fm.NUM_STREAMS
    fm.NUM_STREAMS = 1
    torch.cuda.synchronize()
    pkg._native.profile_begin()
    fitter.step()
    torch.cuda.synchronize()
    prof = pkg._native.profile_end()
    fm.NUM_STREAMS = streams_saved
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())

    # pairs per view for the algorithmic FLOP count (same binning as the kernels)
    pairs, core = [], []
    with torch.no_grad():
        means, scales, colors, opac = fm.activations(fitter.params)
        for i in fitter.my_views:
            gv = tr.make_view(cams[i].view, cams[i].proj, R, R, None, tr.DEFAULT_CUTOFF)
            _, _, _, st = tr.forward_native(means.contiguous(), scales.contiguous(), colors.contiguous(), opac.contiguous(), gv)
            pairs.append(st.num_pairs)
            core.append(int(st.plan.num_core_pairs))
    if rank == 0:
        bwd_ms, bwd_n = prof["raster_bwd"]
        fwd_ms, fwd_n = prof["raster_fwd"]
        bwd_conc_us = 1e3 * prof_concurrent["raster_bwd"][0] / max(prof_concurrent["raster_bwd"][1], 1)
        avg_pairs, avg_core = float(np.mean(pairs)), float(np.mean(core))
        bwd_avg_s = bwd_ms / max(bwd_n, 1) / 1e3
        fwd_avg_s = fwd_ms / max(fwd_n, 1) / 1e3
        fwd_conc_us = 1e3 * prof_concurrent["raster_fwd"][0] / max(prof_concurrent["raster_fwd"][1], 1)
        pmc_tab = {}
        pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                pmc_tab = json.load(f)
        avg_tail = avg_pairs - avg_core
        # the two splat kernels; the one with the longer launches is the bench's "roofline"
        kernels = {
            "bwd": dict(kernel=BWD_KERNEL, t=bwd_avg_s, n=bwd_n, conc_us=bwd_conc_us,
                        flop=BF16_FLOP_PER_CORE_PAIR_BWD * avg_core, f32=F32_FLOP_PER_CORE_PAIR_BWD * avg_core,
                        per_pair=f"{BF16_FLOP_PER_CORE_PAIR_BWD:.0f} per core pair (tail pairs skipped)"),
            "fwd": dict(kernel=FWD_KERNEL, t=fwd_avg_s, n=fwd_n, conc_us=fwd_conc_us,
                        flop=BF16_FLOP_PER_CORE_PAIR_FWD * avg_core + BF16_FLOP_PER_TAIL_PAIR_FWD * avg_tail,
                        f32=F32_FLOP_PER_CORE_PAIR_FWD * avg_core + F32_FLOP_PER_TAIL_PAIR_FWD * avg_tail,
                        per_pair=f"{BF16_FLOP_PER_CORE_PAIR_FWD:.0f} per core pair, {BF16_FLOP_PER_TAIL_PAIR_FWD:.0f} per tail pair"),
        }

        def roof(k):
            e = kernels[k]
            ach = e["flop"] / e["t"] / 1e12
            return {"bound": "mfma", "kernel": e["kernel"], "achieved": round(ach, 1), "peak": BF16_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(ach / BF16_MFMA_PEAK_TFLOPS, 4),
                    "traffic": pmc_tab.get(e["kernel"], {}).get("hbm_bytes_per_launch"),
                    "avg_launch_us": round(e["t"] * 1e6, 1), "launches": e["n"],
                    "timing": "HIP events on the launch stream, one single-stream step after the timed region",
                    "avg_launch_us_in_timed_region": round(e["conc_us"], 1), "streams_in_timed_region": streams_saved,
                    "flop_executed": e["per_pair"], "core_pairs_per_launch": int(avg_core),
                    "tail_pairs_per_launch": int(avg_tail),
                    "f32_equivalent_tflops": round(e["f32"] / e["t"] / 1e12, 1), "f32_peak": F32_MFMA_PEAK_TFLOPS}

        dominant = "fwd" if fwd_avg_s > bwd_avg_s else "bwd"
        hbm_bytes_view = n * (3 * B_IN_RGB + 2 * 36) + avg_pairs * (2 * 12 + 2 * 36 + 2 * 36) + 60 * R * R
        hbm_roof_mpx = HBM_PEAK_GBS * 1e9 / hbm_bytes_view * R * R / 1e6
        pixels = V * R * R * args.steps
        value = pixels / elapsed / 1e6
        out = {
            "metric": "Mpixels/sec fwd+bwd @1M Gaussians 800x800",
            "value": round(value, 2),
            "unit": "Mpixels/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded Gaussians per SURVEY.md 8(d), random targets)",
            "config": {"workload": f"C4: {n} Gaussians, {V} orbit views {R}x{R}, fwd+bwd+grad all-reduce+Adam per step",
                       "gaussians": n, "views": V, "width": R, "height": R, "cutoff_sigma": tr.DEFAULT_CUTOFF,
                       "core_cutoff_sigma": tr.DEFAULT_CORE_CUTOFF,
                       "scale": round(0.1061 * (1200.0 / n) ** (1.0 / 3.0), 5), "seed": 0,
                       "parallelism": f"view-sharded dp{world}", "pairs_per_view": int(avg_pairs),
                       "core_pairs_per_view": int(avg_core),
                       "gaussian_order": "random" if args.no_reorder else "morton (trainer layout, fit_multiview.spatial_order)"},
            # achieved = the splat kernel's MFMA FLOP/s as executed on the bf16 pipe (the split-precision
            # algorithm's own FLOP: 3 piece products per contraction) against the bf16 dense peak, for the
            # splat kernel with the longer launches; both splats in "splats", f32-equivalent rates beside
            "roofline": roof(dominant),
            "splats": {"fwd": roof("fwd"), "bwd": roof("bwd")},
            "hbm_model": {"bytes_per_view": int(hbm_bytes_view), "roofline_mpx_per_s": round(hbm_roof_mpx, 1),
                          "frac": round(value / (hbm_roof_mpx * world), 4),
                          "source": "SURVEY.md 8(d) tile-binned byte model at the measured pairs/view, 8 TB/s"},
            "loss": float(loss),
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(n, R, V)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
