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
  roofline      the dominant kernel (the backward splat; both splats under "splats"): at 32-pixel tiles its
                executed 16-bit MFMA FLOP/s against the dense bf16 peak (48 v_mfma_f32_32x32x16 per 32 pairs),
                with SURVEY.md 8(d)'s byte model beside it under "hbm" (48 B per pair forward, 84 B per pair
                backward, + 40 B per pixel, vs 8 TB/s); the launch time from splat_replay (HIP events around each
                launch in a single-stream schedule after the timed region, less an empty event pair's cost: the
                timed steps overlap views on 4 streams and run uninstrumented), which agrees with the GR_STREAMS=1
                rocprofv3 kernel-trace average in profiles/ (r05: 209.6 vs 206.0 us); PMC HBM traffic and
                VALU / MFMA busy fractions from profiles/pmc_traffic.json when its source stamp matches
  hbm_model     the north_star's framing: SURVEY.md 8(d)'s byte model of the tile-binned path per view at
                this run's pair count (the fit path bins the survey's 5-sigma footprint), the bench value
                as a fraction of that 8 TB/s roofline and of the survey table's C4 roof (2,830 Mpx/s)
  default_precision_mode
                a few more timed steps with a depth term in the loss (the f32-grade mode a depth-loss
                caller gets; the headline runs the fit's own loss, which has no depth term)
  f32_grade_fit the headline's fit step with every splat at f32 grade (three-piece splits,
                gr_view.no_depth_grad = 2): isolates what the two-piece operand splits buy
  dropin_op     the drop-in op exactly as the unchanged reference fit loop calls it
                (fit_multiview_stub.py:265-311): per view render_gaussians_torch(..., return_aux=True) with
                a fresh device background tensor, torch L1 + silhouette losses, loss.backward(),
                torch.optim.Adam, float(loss) per iteration; same C4 workload
  dropin_depth_loss
                the same loop with the stub's --depth_dir term (fit_multiview_stub.py:299-303): the depth
                output is differentiated, so the op renders at f32 grade with the depth footprint (after the
                first iteration up front: torch_renderer.LAZY_ADAPT); two warmup iterations
  psnr_vs_ref   the checker leg (outside every timed region): one view of the final fitted state, the
                bench's render path and the drop-in default path vs the exact float64 dense render
                (oracle/gr_oracle.c, every Gaussian at every pixel) at 2048 random pixels
  sclk_mhz      the shader clock before and after (rocm-smi)
  cpu_baseline  the build's CPU path (cpu_renderer.py: the reference's dense semantics, torch on the host
                cores) fwd+bwd on one view of the same workload; beside it config C1 (the reference stub's
                CPU plumbing case) through the same op and the float64 oracle on one view.
  pmc           per-launch HBM bytes and VALU / MFMA issue fractions of the kernels from
                profiles/pmc_traffic.json (tools/pmc_profile.sh), used only when its source stamp equals
                the sha256 of this tree's gr_hip.hip (else flagged stale and not used).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--device cpu]
N>1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
     --master-port P bench.py --gpus N --steps K --warmup W
     (or plain `python bench.py --gpus N`: it starts that launcher itself as a child process)
"""
from __future__ import annotations

import argparse
import ctypes
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
# renders its views without a depth gradient), per core pair: two K = 16 contractions (over
# x and over y) of 4 upstream channels,
#   f32-equivalent (algorithmic) FLOP = 2 sides x 4 channels x 16 x 16 x 2 = 4096,
#   executed on the bf16 pipe as two-piece splits: 2 sides x 2 channel pairs x 3 piece products of
#   v_mfma_f32_32x32x16_bf16 per 32 pairs = 12,288 FLOP per pair.
F32_FLOP_PER_CORE_PAIR_BWD = 2 * 4 * 16 * 16 * 2
BF16_FLOP_PER_CORE_PAIR_BWD = 2 * 2 * 3 * MFMA_32x32x16 / 32
# Forward splat of the fused fit path (no depth channel, one zone), f32-equivalent: 4 channels (W, R, G, B)
# x 16 x 16 x 2 per pair; executed as two pieces, 3 products of v_mfma_f32_16x16x32_bf16 per channel per
# 32 pairs.  (The fit path has no tail pairs.)
F32_FLOP_PER_CORE_PAIR_FWD = 4 * 16 * 16 * 2
F32_FLOP_PER_TAIL_PAIR_FWD = 1 * 16 * 16 * 2
MFMA_16x16x32 = 2 * 16 * 16 * 32
BF16_FLOP_PER_CORE_PAIR_FWD = 4 * 3 * MFMA_16x16x32 / 32
BF16_FLOP_PER_TAIL_PAIR_FWD = 1 * 3 * MFMA_16x16x32 / 32
FWD_KERNEL = "k_raster_fwd_mfma"
BWD_KERNEL = "k_raster_bwd_bf16"
# The same at 32-pixel tiles (gr_view.tile = 32, the fit path's default: k_fwd32_l1 / k_bwd32): per pair
#   backward f32-equivalent 2 sides x 4 channels x 32 rows x 32 (K) x 2 = 16,384; executed 48 v_mfma_f32_32x32x16_bf16
#   per 32 pairs (2 sides x 4 channels x 2 K-steps x 3 piece products) = 49,152 FLOP per pair;
#   forward f32-equivalent 4 channels x 32 x 32 x 2 = 8,192; executed 12 v_mfma_f32_32x32x16_f16 per 16 pairs
#   (4 channels x 3 products) = 24,576 FLOP per pair.
F32_FLOP_PER_PAIR_BWD32 = 2 * 4 * 32 * 32 * 2
MFMA_FLOP_PER_PAIR_BWD32 = 48 * MFMA_32x32x16 / 32
F32_FLOP_PER_PAIR_FWD32 = 4 * 32 * 32 * 2
MFMA_FLOP_PER_PAIR_FWD32 = 12 * MFMA_32x32x16 / 16
# SURVEY.md §8(d) HBM model of the tile-binned algorithm (the north_star's "fraction of the HBM
# roofline" framing): bytes per view = N (3 B_in + 2 x 36) + K (2 x 12 + 2 x 36 + 2 x 36) + 60 H W
# with B_in = 40 (RGB), K = pairs per view as binned here.
B_IN_RGB = 40
SURVEY_C4_ROOF_MPX = 2830.0  # the north_star target is >= 50% of it


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--views", type=int, default=50)
    ap.add_argument("--res", type=int, default=800)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra-modes", action="store_true",
                    help="skip the extra timed steps of the default (depth-loss) precision mode")
    ap.add_argument("--device", default="cuda", choices=("cuda", "cpu"),
                    help="cpu: a dry run of the launcher and sharding on host tensors (gloo; cpu_renderer), "
                         "not a measurement")
    ap.add_argument("--no-reorder", action="store_true",
                    help="keep the synthetic Gaussians in their random order (A/B of the trainer's Morton order)")
    ap.add_argument("--no-dropin", action="store_true", help="skip the dropin_op measurement")
    ap.add_argument("--no-psnr", action="store_true", help="skip the psnr_vs_ref checker leg")
    return ap.parse_args()


def launch(args) -> int:
    """``--gpus N`` without a torch.distributed environment: start N local ranks with
    torch.distributed.run (one process per GPU) as a child process, before this process touches the GPU,
    and return its exit status.  The driver's own command (torch.distributed.run ... bench.py --gpus N)
    sets WORLD_SIZE and never comes here."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def sclk_mhz():
    """Current shader clock of the visible GPU (rocm-smi), or None."""
    import subprocess

    # Under rocprofv3 its preloaded library is inherited by the child and initialises the GPU before
    # rocm-smi's `env python3` hop execs, which the GPU pool refuses: no clock reading there.
    if "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--json"], capture_output=True, text=True, timeout=20)
        card = next(iter(json.loads(r.stdout).values()))
        v = card.get("sclk clock speed:", "")
        return int(v.strip("()Mhz")) if v else None
    except Exception:  # noqa: BLE001 - diagnostics only
        return None


def synthetic_params(n: int, device) -> dict:
    g = torch.Generator().manual_seed(0)
    means = (torch.rand((n, 3), generator=g) - 0.5) * 1.2
    scale = 0.1061 * (1200.0 / n) ** (1.0 / 3.0)
    scales_raw = torch.full((n, 3), math.log(math.expm1(scale - 1e-3)))  # softplus^-1(scale - 1e-3)
    op_raw = torch.full((n,), -2.2)
    colors_raw = 0.1 * torch.rand((n, 3), generator=g)
    p = {"means": means, "scales_raw": scales_raw, "opacities_raw": op_raw, "colors_raw": colors_raw}
    return {k: torch.nn.Parameter(v.to(device)) for k, v in p.items()}


def _cpu_op_fwd_bwd(n: int, res: int, views: int, nviews: int, sample: int = 0) -> float:
    """Seconds for fwd + bwd of ``nviews`` views through the build's CPU op (render_gaussians_torch on host
    tensors -> cpu_renderer.py), L1 loss, on the synthetic scene of ``n`` Gaussians (its first ``sample``
    Gaussians when given: the dense op's cost is linear in the Gaussian count)."""
    p = synthetic_params(n, torch.device("cpu"))
    if sample:
        p = {k: torch.nn.Parameter(v.detach()[:sample].clone()) for k, v in p.items()}
    cams = fm.orbit_cameras(views, res, res, torch.device("cpu"))
    g = torch.Generator().manual_seed(3)
    tgt = torch.rand((res, res, 3), generator=g)
    t0 = time.perf_counter()
    means, scales, colors, opac = fm.activations(p)
    total = 0.0
    for i in range(nviews):
        out, alpha, _ = tr.render_gaussians_torch(means, scales, colors, opac, cams[i], res, res,
                                                  max_gaussians=max(10000, n), return_aux=True)
        total = total + torch.mean(torch.abs(out - tgt))
    total.backward()
    return time.perf_counter() - t0


def usable_cores() -> tuple:
    """(cores this process may run on, how that was found): the CPU affinity mask, capped by the cgroup's CPU quota
    when one is set (a GPU box's share of a many-core host shows there, not in os.cpu_count())."""
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    how = f"sched_getaffinity {cores}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, math.ceil(int(quota) / int(period)))
            how += f", cgroup cpu.max quota {q}"
            cores = min(cores, q)
    except (OSError, ValueError):
        pass
    return cores, how


def cpu_baseline(n: int, res: int, views: int) -> dict:
    """The build's CPU op (cpu_renderer.py, torch on the host cores: the reference's dense semantics) on ONE
    whole view of the workload (all n Gaussians, fwd + bwd, unscaled), torch and OpenMP on every usable core; plus
    config C1 through the same op and the float64 oracle port."""
    from oracle import oracle as orc

    cores, how = usable_cores()
    saved = torch.get_num_threads()
    torch.set_num_threads(cores)
    try:
        threads = torch.get_num_threads()
        dt = _cpu_op_fwd_bwd(n, res, views, 1)
        c1 = _cpu_op_fwd_bwd(1200, 128, 4, 4)
    finally:
        torch.set_num_threads(saved)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0")) or cores  # the oracle's OpenMP threads
    scene = orc.synthetic_scene(n, seed=0)
    view, proj = orc.orbit_cameras(views, res, res)[0]
    v = orc.make_view(view, proj, res, res, cutoff=tr.default_cutoff(False), core_cutoff=tr.DEFAULT_CORE_CUTOFF)
    gr = np.random.default_rng(0).standard_normal((res, res, 3)).astype(np.float32)
    t0 = time.perf_counter()
    orc.forward(v, scene, binned=True)
    orc.backward(v, scene, gr, None, None, binned=True)
    dto = time.perf_counter() - t0
    return {"value": round(res * res / dt / 1e6, 5), "unit": "Mpixels/sec fwd+bwd", "cores": threads, "kind": "port",
            "host_cpu_count": os.cpu_count(), "usable_cores": cores, "usable_cores_from": how, "torch_threads": threads,
            "sample": f"1 whole view of the workload ({n} Gaussians, {res}x{res}) fwd+bwd through render_gaussians_torch on "
                      f"host tensors (cpu_renderer.py, dense: every Gaussian at every pixel, as the reference), torch with "
                      f"{threads} threads, {dt:.1f} s, unscaled",
            "c1": {"value": round(4 * 128 * 128 / c1 / 1e6, 4), "unit": "Mpixels/sec fwd+bwd", "threads": threads,
                   "sample": f"config C1: 1200 Gaussians, 4 views 128x128, one fit step's fwd+bwd through the same op, "
                             f"{c1:.2f} s"},
            "oracle": {"value": round(res * res / dto / 1e6, 5), "unit": "Mpixels/sec fwd+bwd", "cores": omp,
                       "sample": f"1 view of the workload, oracle/gr_oracle.c binned float64 fwd+bwd, OpenMP {omp} "
                                 f"threads, {dto:.1f} s"}}


def source_sha256() -> str:
    import hashlib

    with open(os.path.join(REPO, "3dgaussian_amd", "csrc", "gr_hip.hip"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_table() -> dict:
    """profiles/pmc_traffic.json (tools/pmc_profile.sh + tools/pmc_summarize.py) when its stamp matches this
    tree's kernel source; else {"stale": True, ...} and no figures."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return {"stale": True, "reason": "no profiles/pmc_traffic.json"}
    with open(path) as f:
        tab = json.load(f)
    tree = source_sha256()
    if tab.get("source_sha256") != tree:
        return {"stale": True, "reason": "collected on another gr_hip.hip", "file_sha256": tab.get("source_sha256"),
                "tree_sha256": tree}
    return {"stale": False, "source_sha256": tree, "dir": tab.get("dir"), "kernels": tab.get("kernels", {})}


def pmc_of(pmc: dict, prefix: str) -> dict:
    if pmc.get("stale"):
        return {}
    for k, e in pmc["kernels"].items():
        if k.startswith(prefix):
            return e
    return {}


def dropin_op(n: int, V: int, R: int, steps: int, warmup: int, device, depth_loss: bool = False) -> dict:
    """fit_multiview_stub.py:265-311 as written, on the drop-in module: the unchanged reference loop's use of
    the op (render_gaussians_torch per view with a fresh device background, torch losses, autograd, Adam,
    float(loss) per iteration).  Mpx/s over ``steps`` iterations after ``warmup``.  depth_loss: the loop with its
    --depth_dir term, w_depth mean|depth / (depth.max() + 1e-6) - d_gt| (fit_multiview_stub.py:299-303)."""
    tr.reset_lazy_depth()  # a fresh loop: the op has not yet seen whether this loss differentiates the depth
    params = synthetic_params(n, device)
    cams = fm.orbit_cameras(V, R, R, device)
    g = torch.Generator(device=device).manual_seed(1)
    targets = [torch.rand((R, R, 3), generator=g, device=device) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).to(torch.float32) for t in targets]
    depths = [torch.rand((R, R), generator=g, device=device) for _ in range(V)] if depth_loss else None
    opt = torch.optim.Adam(list(params.values()), lr=0.02)

    def iteration():
        opt.zero_grad(set_to_none=True)
        means = params["means"]
        scales = torch.nn.functional.softplus(params["scales_raw"]) + 1e-3
        opacities = torch.sigmoid(params["opacities_raw"])
        colors_eval = torch.sigmoid(params["colors_raw"])
        total = torch.tensor(0.0, device=device)
        for i, tgt in enumerate(targets):
            pred, alpha, depth = tr.render_gaussians_torch(means, scales, colors_eval, opacities, cams[i], width=R,
                                                           height=R, background=torch.tensor([0.0, 0.0, 0.0], device=device),
                                                           max_gaussians=max(3000, means.shape[0]), return_aux=True)
            loss_i = torch.mean(torch.abs(pred - tgt)) + 0.2 * torch.mean(torch.abs(alpha - masks[i]))
            if depths is not None:
                d_pred = depth / (depth.max() + 1e-6)
                loss_i = loss_i + 0.05 * torch.mean(torch.abs(d_pred - depths[i]))
            total = total + loss_i
        reg = 1e-3 * opacities.mean() + 1e-3 * scales.mean()
        loss = total / len(targets) + reg
        loss.backward()
        opt.step()
        return float(loss.detach().cpu())

    for _ in range(warmup):
        iteration()
    spec0 = dict(tr._SPEC)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        lv = iteration()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"value": round(V * R * R * steps / dt / 1e6, 2), "unit": "Mpixels/sec", "steps": steps, "warmup": warmup,
            "ms_per_step": round(1e3 * dt / steps, 3), "loss": lv,
            "speculative_preparations": {"hits": tr._SPEC["hits"] - spec0["hits"],
                                         "misses": tr._SPEC["misses"] - spec0["misses"]},
            "path": "render_gaussians_torch (autograd op, default precision mode: depth_grad=True, 8/5.5-sigma "
                    "footprint) as fit_multiview_stub.py:277-311 calls it, unchanged loop"
                    + (", with the --depth_dir depth term (:299-303)" if depth_loss else "")}


def psnr_vs_ref(fitter, cams, R: int, device, npix: int = 2048) -> dict:
    """Checker leg: view 0 of the current fitted state, rendered by the bench's own forward (gr_fwd_render_l1 on the
    fitter's gr_view of view 0: the kernel the timed step runs, k_fwd32_l1 at the fit's 32-pixel tiles, with its L1
    epilogue against view 0's target, images written beside) and by the drop-in default path, against the exact
    float64 dense render (oracle/gr_oracle.c: every Gaussian at every pixel, no cutoff) at ``npix`` random pixels."""
    from oracle import oracle as orc

    with torch.no_grad():
        acts = [a.detach().float().contiguous() for a in fm.activations(fitter.params)]
    sc = orc.Scene(*(a.cpu().numpy() for a in acts))
    view, proj = orc.orbit_cameras(len(cams), R, R)[0]
    v = orc.make_view(view, proj, R, R, None)
    pix = np.random.default_rng(11).choice(R * R, npix, replace=False).astype(np.int32)
    t0 = time.perf_counter()
    d_out, d_a, _ = orc.dense_pixels(v, sc, pix)
    t_dense = time.perf_counter() - t0
    res = {}
    for name in ("bench_path", "dropin_default"):
        if name == "bench_path":
            gv = fitter._fit_view(0, device)
            out = torch.empty((R, R, 3), device=device)
            alpha = torch.empty((R, R), device=device)
            mask = fitter.masks[0] if fitter.masks is not None else None
            tr.forward_l1_native(*acts, gv, tr.prepare_native(*acts, gv), fitter.targets[0], mask,
                                 fitter.w_sil if mask is not None else 0.0, 1.0 / len(cams),
                                 torch.zeros(1, device=device), out=out, alpha=alpha)
            kernel = f"gr_fwd_render_l1 ({'k_fwd32_l1' if gv.tile == 32 else 'k_raster_fwd_mfma'}, tile {gv.tile or 16})"
        else:
            gv = tr.make_view(view, proj, R, R, None)
            out, alpha, _, _ = tr.forward_native(*acts, gv, want_depth=False)
            kernel = "gr_fwd_render (drop-in default footprint, 16-pixel tiles)"
        o = out.cpu().numpy().reshape(-1, 3)[pix]
        a = alpha.cpu().numpy().reshape(-1)[pix]
        res[name] = {"psnr_db": round(orc.psnr(o, d_out), 2), "rel_l2_rgb": float(f"{orc.rel_l2(o, d_out):.3e}"),
                     "rel_l2_alpha": float(f"{orc.rel_l2(a, d_a):.3e}"), "kernel": kernel}
    res.update(value=res["bench_path"]["psnr_db"], unit="dB", target=">= 60 dB (north_star)",
               sample=f"view 0 of the final fitted state, {npix} random pixels, exact float64 dense reference "
                      f"({t_dense:.1f} s on the host)")
    return res


def splat_replay(fitter, device) -> dict:
    """The fit path's two splat kernels timed on their own, in a single-stream schedule of this rank's views: per view
    its binning (untimed), then its forward splat (gr_fwd_render_l1 on the binned view) and backward splat
    (gr_bwd_splat), each between two HIP events on the stream.  Every preparation is enqueued first and the host never
    waits inside the loop, so the GPU runs the launches back to back (no host gap inside an event pair) with the
    caches as a single-stream step leaves them (binning -> forward -> backward of the same view): the averages compare
    with a rocprofv3 kernel-trace summary of the bench under GR_STREAMS=1 (profiles/)."""
    L = tr._native.lib()
    nat = tr._native
    with torch.no_grad():
        acts = [a.detach().float().contiguous() for a in fm.activations(fitter.params)]
    n = int(acts[0].shape[0])
    cur = torch.cuda.current_stream(device)
    sp = ctypes.c_void_p(cur.cuda_stream)
    V = max(len(fitter.targets), 1)
    w_sil = fitter.w_sil if fitter.masks is not None else 0.0
    preps = []
    whole = [i for i in fitter.my_views if i < V]  # (a band of a view, multi-GPU: the roofline times whole views)
    for i in whole or [0]:  # (a rank with bands only, V < R: one whole view stands in)
        gv = fitter._fit_view(i, device)
        preps.append((i, gv, tr.prepare_native(*acts, gv)))
    torch.cuda.synchronize()
    ev = []
    pairs = []
    for i, gv, prep in preps:
        plan = prep.plan()
        pairs.append(int(plan.num_pairs))
        bins, scratch, bgv, done = tr._bin_launch(L, gv, n, plan, prep, cur, device)
        ws = torch.empty((tr._ws_round(L.gr_bwd_bytes(ctypes.byref(gv), n, ctypes.byref(plan))),), dtype=torch.uint8,
                         device=device)
        loss = torch.zeros(1, device=device)
        mask = fitter.masks[fitter._vi(i)] if fitter.masks is not None else None
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record(cur)
        nat.check(L.gr_fwd_render_l1(ctypes.byref(bgv), n, ctypes.byref(plan), nat.ptr(prep.geom), nat.ptr(bins),
                                     bins.numel(), nat.ptr(scratch), scratch.numel(), nat.ptr(fitter.targets[fitter._vi(i)]),
                                     nat.ptr(mask), ctypes.c_float(w_sil), ctypes.c_float(1.0 / V), nat.ptr(loss), None,
                                     None, nat.ptr(ws), ws.numel(), sp), "gr_fwd_render_l1")
        e[1].record(cur)
        nat.check(L.gr_bwd_splat(ctypes.byref(gv), n, ctypes.byref(plan), nat.ptr(prep.geom), nat.ptr(bins), nat.ptr(ws),
                                 ws.numel(), sp), "gr_bwd_splat")
        e[2].record(cur)
        e[3].record(cur)  # an empty event pair: the markers' own cost, subtracted below
        ev.append(e)
    torch.cuda.synchronize()
    k = len(ev)
    mark = 1e3 * sum(e[2].elapsed_time(e[3]) for e in ev) / k
    fwd = 1e3 * sum(e[0].elapsed_time(e[1]) for e in ev) / k
    bwd = 1e3 * sum(e[1].elapsed_time(e[2]) for e in ev) / k
    out = {"fwd_us": fwd - mark, "bwd_us": bwd - mark, "fwd_us_events": fwd, "bwd_us_events": bwd, "marker_us": mark,
           "launches": k, "pairs": float(np.mean(pairs)), "tile": int(preps[0][1].tile) or 16}
    del preps, ev
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    on_gpu = args.device == "cuda"
    if on_gpu:
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
    if world > 1:
        if on_gpu:
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    n, V, R = args.gaussians, args.views, args.res
    clk0 = sclk_mhz() if (on_gpu and rank == 0) else None

    params = synthetic_params(n, device)
    cams = fm.orbit_cameras(V, R, R, device)
    g = torch.Generator(device=device).manual_seed(1)
    targets = [torch.rand((R, R, 3), generator=g, device=device) for _ in range(V)]
    masks = [(t.mean(dim=2) > 0.5).to(torch.float32) for t in targets]
    fitter = fm.ViewShardedFitter(params, cams, targets, R, R, lr=0.02, masks=masks, reorder=not args.no_reorder)
    views_per_rank = [len(range(r, V, world)) for r in range(world)]
    if fitter._bands_ok():  # the leftover views in bands of tile rows, one per rank
        views_per_rank = [round(V / world, 3)] * world

    def timed(steps):
        sync()
        if world > 1:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        loss = None
        for _ in range(steps):
            loss = fitter.step()
        sync()
        if world > 1:
            dist.barrier()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt.item()), loss

    for _ in range(args.warmup):
        fitter.step()
    # the timed region runs uninstrumented: HIP event marks around every splat launch cost ~1.5% of the
    # step (a marker packet per mark on each stream); the launch timings come from the profiled steps below
    elapsed, loss = timed(args.steps)
    pixels = V * R * R * args.steps
    value = pixels / elapsed / 1e6

    if not on_gpu:  # dry run of the launcher / sharding: no measurement keys
        if rank == 0:
            print(json.dumps({"metric": "Mpixels/sec fwd+bwd @1M Gaussians 800x800 (dry run on host tensors)",
                              "value": round(value, 4), "unit": "Mpixels/sec", "n_gpus": world, "steps": args.steps,
                              "warmup": args.warmup, "device": "cpu", "views_per_rank": views_per_rank,
                              "loss": float(loss)}), flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    # One profiled step as the timed ones (views rotating over several HIP streams): a launch's duration
    # there includes the kernels of other views running beside it.
    sync()
    pkg._native.profile_begin()
    fitter.step()
    sync()
    prof_concurrent = pkg._native.profile_end()
    # Roofline pass: one more step on a single stream gives each launch its own duration (with
    # GR_STREAMS=1 the whole run is single-stream and both agree).
    streams_saved = fm.NUM_STREAMS
    fm.NUM_STREAMS = 1
    sync()
    pkg._native.profile_begin()
    fitter.step()
    sync()
    prof = pkg._native.profile_end()
    fm.NUM_STREAMS = streams_saved
    # the splat kernels' launch durations for the roofline: replayed once per view back to back (splat_replay)
    replay = splat_replay(fitter, device) if rank == 0 else None
    # the fit step renders its views through the fused path: one zone at FIT_CUTOFF (fit_multiview._views_direct), at
    # the fit's tile size; the replay's plans are those views'
    avg_pairs = avg_core = replay["pairs"] if replay else 0.0

    # the default precision mode: what a caller with a depth loss gets (f32-grade W / D, three-piece
    # backward with the tail pairs): the same fit with a depth term in the loss (C3's losses)
    extra, f32g = {}, None
    if not args.no_extra_modes:
        gd = torch.Generator(device=device).manual_seed(2)
        fitter.depths = [torch.rand((R, R), generator=gd, device=device) for _ in range(V)]
        for _ in range(max(1, args.warmup)):  # the depth path's larger workspaces: warmed up as the headline's
            fitter.step()
        k = max(1, min(args.steps, 5))
        dt, _ = timed(k)
        fitter.depths = None
        extra = {"value": round(V * R * R * k / dt / 1e6, 2), "steps": k, "ms_per_step": round(1e3 * dt / k, 3),
                 "mode": "depth_grad=True: forward W/D f32-grade (3-piece bf16 split), backward 3-piece with tail "
                         "pairs; loss L1 + silhouette + 0.05 depth L1 (fit_multiview_stub.py:299-305)"}
        # the headline's own loss and footprint with every splat at f32 grade (no_depth_grad = 2)
        fm.F32_GRADE = True
        for _ in range(max(1, args.warmup)):
            fitter.step()
        dt, _ = timed(k)
        fm.F32_GRADE = False
        f32g = {"value": round(V * R * R * k / dt / 1e6, 2), "steps": k, "ms_per_step": round(1e3 * dt / k, 3),
                "mode": "the headline fit step (L1 + silhouette, 5-sigma fit footprint, fused path) with "
                        "gr_view.no_depth_grad = 2: forward W three bf16 pieces, colours two pieces x three-piece B, "
                        "backward three-piece splits (the default precision mode's splats, f32-grade)"}
    clk1 = sclk_mhz() if rank == 0 else None
    psnr = psnr_vs_ref(fitter, cams, R, device) if (rank == 0 and not args.no_psnr) else None
    my_views_n = max(len(fitter.my_views), 1)
    drop = drop_depth = None
    if rank == 0 and world == 1 and not args.no_dropin:
        del fitter
        torch.cuda.empty_cache()
        drop = dropin_op(n, V, R, steps=3, warmup=1, device=device)
        torch.cuda.empty_cache()
        # two warmup iterations: the first teaches the op that this loss differentiates the depth (adaptive
        # laziness), the second its camera order in that mode (speculation)
        drop_depth = dropin_op(n, V, R, steps=2, warmup=2, device=device, depth_loss=True)

    if rank == 0:
        bwd_conc_us = 1e3 * prof_concurrent["raster_bwd"][0] / max(prof_concurrent["raster_bwd"][1], 1)
        fwd_conc_us = 1e3 * prof_concurrent["raster_fwd"][0] / max(prof_concurrent["raster_fwd"][1], 1)
        bwd_avg_s = replay["bwd_us"] / 1e6
        fwd_avg_s = replay["fwd_us"] / 1e6
        pmc = pmc_table()
        px = R * R
        t32 = replay["tile"] == 32
        # SURVEY.md 8(d) per-unit bytes: a pair = 12 B key/value + 36 B projected record read once per
        # splat pass; the backward also writes its 36 B of gradient partials; per pixel 20 B of outputs
        # + 20 B of saved state written (forward) / 20 B of upstream grads + 20 B saved read (backward)
        kernels = {
            "fwd": dict(variant="k_fwd32_l1" if t32 else "k_raster_fwd_mfma<4>", t=fwd_avg_s, conc_us=fwd_conc_us,
                        units=avg_pairs, unit_bytes=12 + 36, px_bytes=40, units_desc="pairs per launch",
                        flop=(MFMA_FLOP_PER_PAIR_FWD32 if t32 else BF16_FLOP_PER_CORE_PAIR_FWD) * avg_pairs,
                        f32=(F32_FLOP_PER_PAIR_FWD32 if t32 else F32_FLOP_PER_CORE_PAIR_FWD) * avg_pairs),
            "bwd": dict(variant="k_bwd32" if t32 else "k_raster_bwd_bf16<false,2>", t=bwd_avg_s, conc_us=bwd_conc_us,
                        units=avg_pairs, unit_bytes=12 + 36 + 36, px_bytes=40, units_desc="pairs per launch",
                        flop=(MFMA_FLOP_PER_PAIR_BWD32 if t32 else BF16_FLOP_PER_CORE_PAIR_BWD) * avg_pairs,
                        f32=(F32_FLOP_PER_PAIR_BWD32 if t32 else F32_FLOP_PER_CORE_PAIR_BWD) * avg_pairs),
        }
        timing = (f"HIP events around each of {replay['launches']} launches (one per view, a single-stream schedule after "
                  f"the timed region: splat_replay), less the cost of an empty event pair measured beside them "
                  f"(avg_launch_us_events keeps it); compare the GR_STREAMS=1 rocprofv3 kernel-trace summary in profiles/")

        def roof(k):
            """The kernel against the bound that binds it: the MFMA pipe (executed 16-bit MFMA FLOP/s vs the dense
            bf16 peak; the split operands make it execute 3x the f32-equivalent contraction) - at 32-pixel tiles the
            splats do 4x the pixel work per pair on half the pairs, so their HBM traffic per pixel halves and the
            per-pair HBM model (under "hbm") no longer bounds them."""
            e = kernels[k]
            nbytes = e["unit_bytes"] * e["units"] + e["px_bytes"] * px
            t = e["t"] if e["t"] > 0 else float("inf")  # a launch left out (GR_DEBUG_SKIP variant builds)
            ach = nbytes / t / 1e9
            mf = e["flop"] / t / 1e12
            pk = pmc_of(pmc, e["variant"])
            hbm = {"achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                   "algorithmic_bytes_per_launch": int(nbytes),
                   "bytes_model": f"{e['unit_bytes']} B x {e['units_desc']} ({int(e['units'])}) + {e['px_bytes']} B x {px} px",
                   "traffic": pk.get("hbm_bytes_per_launch")}
            ev_us = replay[k + "_us_events"]
            if t32:
                return {"bound": "mfma", "kernel": e["variant"], "achieved": round(mf, 1), "peak": BF16_MFMA_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(mf / BF16_MFMA_PEAK_TFLOPS, 4), "traffic": pk.get("hbm_bytes_per_launch"),
                        "valu_frac": pk.get("valu_frac"), "mfma_frac": pk.get("mfma_frac"),
                        "executed_flop_per_launch": int(e["flop"]), "f32_equivalent_tflops": round(e["f32"] / t / 1e12, 1),
                        "f32_peak": F32_MFMA_PEAK_TFLOPS, "hbm": hbm,
                        "avg_launch_us": round(e["t"] * 1e6, 1), "avg_launch_us_events": round(ev_us, 1),
                        "event_marker_us": round(replay["marker_us"], 2), "launches": replay["launches"], "timing": timing,
                        "avg_launch_us_multi_stream": round(e["conc_us"], 1), "streams_in_timed_region": streams_saved}
            return {"bound": "hbm", "kernel": e["variant"], "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": pk.get("hbm_bytes_per_launch"),
                    "valu_frac": pk.get("valu_frac"), "mfma_frac": pk.get("mfma_frac"),
                    "algorithmic_bytes_per_launch": int(nbytes), "bytes_model": hbm["bytes_model"],
                    "avg_launch_us": round(e["t"] * 1e6, 1), "launches": replay["launches"], "timing": timing,
                    "avg_launch_us_multi_stream": round(e["conc_us"], 1), "streams_in_timed_region": streams_saved,
                    "mfma": {"executed_bf16_tflops": round(mf, 1), "peak": BF16_MFMA_PEAK_TFLOPS,
                             "frac": round(mf / BF16_MFMA_PEAK_TFLOPS, 4),
                             "f32_equivalent_tflops": round(e["f32"] / t / 1e12, 1), "f32_peak": F32_MFMA_PEAK_TFLOPS}}

        dominant = "fwd" if fwd_avg_s > bwd_avg_s else "bwd"

        def hbm_model(k):
            b = n * (3 * B_IN_RGB + 2 * 36) + k * (2 * 12 + 2 * 36 + 2 * 36) + 60 * px
            roof_mpx = HBM_PEAK_GBS * 1e9 / b * px / 1e6
            return {"pairs_per_view": int(k), "bytes_per_view": int(b), "roofline_mpx_per_s": round(roof_mpx, 1),
                    "frac": round(value / (roof_mpx * world), 4)}

        out = {
            "metric": "Mpixels/sec fwd+bwd @1M Gaussians 800\u00d7800; PSNR vs torch ref",
            "value": round(value, 2),
            "unit": "Mpixels/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32 (splat contractions on v_mfma_f32_32x32x16_f16 with f32 accumulation; every operand in two "
                     "round-to-nearest f16 pieces, pre-scaled into f16's normal range, three piece products: "
                     "<= 3*2^-22 per product, forward and backward; no-depth-gradient mode)",
            "data": "synthetic (seeded Gaussians per SURVEY.md 8(d), random targets)",
            "config": {"workload": f"C4: {n} Gaussians, {V} orbit views {R}x{R}, fwd+bwd+grad all-reduce+Adam per step",
                       "gaussians": n, "views": V, "width": R, "height": R, "cutoff_sigma": tr.FIT_CUTOFF, "core_cutoff_sigma": tr.FIT_CUTOFF,
                       "tile": replay["tile"],
                       "render_path": "fused fit path: per view gr_fwd_render_l1 (forward, loss and upstream gradients) "
                                      "+ gr_bwd_splat + gr_gather_view (per-Gaussian sums), then gr_reduce_sums (chain rule) "
                                      "per batch of a stream's views (fit_multiview._views_direct, 4 HIP streams)",
                       "scale": round(0.1061 * (1200.0 / n) ** (1.0 / 3.0), 5), "seed": 0,
                       "parallelism": f"view-sharded dp{world}", "views_per_rank": views_per_rank,
                       "pairs_per_view": int(avg_pairs), "core_pairs_per_view": int(avg_core),
                       "gaussian_order": "random" if args.no_reorder else
                       f"morton (trainer layout, re-established every {fm.RESORT_EVERY} steps)"},
            # the dominant splat kernel against the HBM roofline (SURVEY.md 8(d) bytes per pair); both
            # splats in "splats", with their MFMA rates beside
            "roofline": roof(dominant),
            "splats": {"fwd": roof("fwd"), "bwd": roof("bwd")},
            # the batched per-Gaussian reduction (gr_reduce_views), HIP events, per view of the single-stream step
            "reduce_us_per_view": round(1e3 * prof["reduce_bwd"][0] / my_views_n, 1),
            "binning_us_per_view": round(1e3 * prof["binning"][0] / my_views_n, 1),
            "hbm_model": dict(hbm_model(avg_pairs),
                              survey_table_roofline_mpx_per_s=SURVEY_C4_ROOF_MPX,
                              frac_of_survey_table=round(value / (SURVEY_C4_ROOF_MPX * world), 4),
                              source=f"SURVEY.md 8(d) tile-binned byte model at 8 TB/s with this run's pair count (the "
                                     f"fit path bins one {tr.FIT_CUTOFF:g}-sigma zone, the survey's footprint), and "
                                     f"the survey table's C4 roof (K = 9.41e6 pairs per view at view 0)"),
            "default_precision_mode": extra or None,
            "f32_grade_fit": f32g,
            "dropin_op": drop,
            "dropin_depth_loss": drop_depth,
            "psnr_vs_ref": psnr,
            "pmc": {k: v for k, v in pmc.items() if k != "kernels"},
            "sclk_mhz": {"before": clk0, "after": clk1},
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
