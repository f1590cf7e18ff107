"""View-sharded data-parallel multiview fitting on MI355X (one process per GPU, RCCL over xGMI).

The math of one iteration is the reference fit loop's (python/fit_multiview_stub.py:265-325):
activations (:268-275), per-view render + L1 / silhouette / depth losses (:277-305), loss =
sum / V + regularisers (:307-308), backward (:310), Adam (:311), densify/prune every interval with
an Adam reset (:318-325).  What changes is where it runs:

* rank r renders views i = r, r+R, r+2R, ... (R ranks) with the HIP render op and computes
  sum_{i in r} loss_i / V (the regulariser is added on rank 0 only);
* one all_reduce(SUM) of a flat fp32 buffer of every parameter gradient (10 floats per Gaussian
  RGB, 19 with SH degree 1) makes every rank hold the full-loss gradient, so the Adam steps are
  identical on all ranks (up to summation order of the collective);
* densify/prune is decided on rank 0 with the host RNG and broadcast, so parameters stay equal.

Random initialisation and densify jitter are drawn from torch's CPU generator in the same order as
the stub (torch.rand for means, then colours; torch.randn_like for jitter), so a seeded run
reproduces the stub's parameters exactly before the first step.

Run single-GPU:   python 3dgaussian_amd/fit_multiview.py --targets_dir DIR [stub flags]
Run on 8 GPUs:    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
                      3dgaussian_amd/fit_multiview.py --targets_dir DIR [stub flags]
"""
from __future__ import annotations

import argparse
import contextlib
import ctypes
import math
import os
import sys
from pathlib import Path
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import losses  # type: ignore
    import torch_renderer as tr  # type: ignore
    from spatial import _spread3, morton_order  # type: ignore  # noqa: F401
else:
    from . import losses
    from . import torch_renderer as tr
    from .spatial import _spread3, morton_order  # noqa: F401

RenderFn = Callable[..., tuple]


def ctypes_stream(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
DEVICE_DENSIFY_MIN = 100_000  # Gaussians from which densify/prune runs on the device (C5 scale)
FUSED_LOSS = os.environ.get("GR_FUSED_LOSS", "1") != "0"  # losses.l1_loss for the L1 terms (A/B switch)
# HIP streams the views rotate over (same-box A/B, 20 steps: 4 vs 3 +0.5% at 50 views, +0.8% at the 7 views
# one rank of 8 renders, +2% at 25; 6 or 8 streams lose)
NUM_STREAMS = max(1, int(os.environ.get("GR_STREAMS", "4")))
PREFETCH = max(1, int(os.environ.get("GR_PREFETCH", "3")))  # views prepared ahead of the one rendering
# steps between re-establishing the Morton order of the moving Gaussians (ViewShardedFitter.respatialize;
# 0 = only at construction and after densify/prune).  A re-sort costs ~1.2 ms at 1M Gaussians (codes,
# argsort, 12 permuted tensors); the means move little in 16 Adam steps, so the tile locality holds
# (same-box A/B at C4, 20 steps: 16 vs 4 +1%)
RESORT_EVERY = max(0, int(os.environ.get("GR_RESORT", "16")))
# the fit step without a depth loss renders through the fused path (ViewShardedFitter._views_direct:
# gr_bwd_l1 + per-stream gradient accumulators, no autograd per view); 0 = the autograd path
DIRECT_BACKWARD = os.environ.get("GR_DIRECT", "1") != "0"
# views of one stream whose gradient partials are reduced together (gr_reduce_views): the parameters are
# read and the stream's gradient accumulator read and written once per batch instead of once per view
# (at most REDUCE_BATCH views per batch, a stream's views split into equal batches)
REDUCE_BATCH = max(1, min(16, int(os.environ.get("GR_REDUCE_BATCH", "16"))))
# views in the last batch of each stream (0: near-equal batches only)
REDUCE_TAIL = max(0, min(REDUCE_BATCH, int(os.environ.get("GR_REDUCE_TAIL", "2"))))  # a batch holds <= REDUCE_BATCH
# fused path: gradient assembly through the activations and the Adam update in one HIP pass per parameter
# (gr_fit_param_step) instead of torch's autograd + foreach Adam (0 = torch)
FUSED_STEP = os.environ.get("GR_FUSED_STEP", "1") != "0"
# fused path: views prepared ahead of the one being rendered (on the preparation stream)
PREP_AHEAD = max(1, int(os.environ.get("GR_PREP_AHEAD", "6")))
L_MAX_ACC = 8  # GR_FIT_MAX_ACC: stream accumulators gr_fit_param_step sums
# views prepared together (gr_fwd_prepare_views_async: the parameters read once for the group)
PREP_GROUP = max(1, min(4, int(os.environ.get("GR_PREP_GROUP", "4"))))
PREP_FIRST = max(1, min(PREP_GROUP, int(os.environ.get("GR_PREP_FIRST", "1"))))
# groups prepared before the step's first render is enqueued: 2 (the first view's group and the next one), or 1
# (only the first view's: the next group is enqueued after the first render)
PREP_INITIAL = max(1, min(2, int(os.environ.get("GR_PREP_INITIAL", "2"))))
# the fused path's reduction in two stages: each view's pair partials gathered into per-Gaussian sums right
# after its backward splat (gr_gather_view: a lean kernel that runs beside the other streams' splats; the view's
# workspaces are released at once), the chain rules of a stream's batch of views from those sums
# (gr_reduce_sums).  0 = the one-pass gr_reduce_views over the batch's kept workspaces.
GATHER = os.environ.get("GR_GATHER", "1") != "0"
# the fused paths' per-view schedule as native host code (gr_fit_views, csrc/gr_fit_exec.cpp: the same streams,
# preparation groups and reduction batches, bit-identical results); 0 = the Python schedule below, 1 = always,
# auto (default) = for views of at most NATIVE_EXEC_MAX_PIXELS, where the per-view GPU work is short enough for the
# host's per-view enqueue time to show (C2, 8 views 512x512: 1.33 -> 1.10 ms per step; at 800x800 the step is
# GPU-bound and the Python schedule is level or 1-2% ahead: profiles/r03_ab_native_exec.txt)
NATIVE_EXEC = os.environ.get("GR_NATIVE_EXEC", "auto")
NATIVE_EXEC_MAX_PIXELS = 512 * 512
# the native executor on this driver's torch streams (1) or on streams of its own (0)
EXEC_STREAMS = os.environ.get("GR_EXEC_STREAMS", "1") != "0"
# priority of the preparation stream (torch's convention: 0 normal, -1 high).  HIP keeps one pool of hardware
# queues per priority, so a high-priority preparation stream also stops sharing a queue with a render stream.
PREP_PRIORITY = int(os.environ.get("GR_PREP_PRIORITY", "0"))
# the fused path's binning (gr_fwd_bin) on a stream of its own with this priority ("" = off: each view bins on
# its render stream inside gr_fwd_render_l1).  The binning kernels are latency-bound; behind the other streams'
# splats they take several times their standalone time while holding CU resources.
BIN_STREAM = os.environ.get("GR_BIN_STREAM", "")
# the fused path at f32 grade (gr_view.no_depth_grad = 2: three-piece splits in both splats, as the default
# precision mode) instead of its two-piece mode: the precision reference of the fit path (bench.py f32_grade_fit)
F32_GRADE = os.environ.get("GR_F32_GRADE", "0") != "0"
# screen tile edge of the fused path's views (gr_view.tile): 32-pixel tiles halve the (Gaussian, tile) pairs of the
# ~3-pixel-sigma C4 scene (7.8 -> 3.7 per Gaussian), so the binning and the per-pair gradient rows and their gather
# (DESIGN.md §5); 16 = the drop-in op's tiles.  The f32-grade reference mode (F32_GRADE) keeps 16.
FIT_TILE = int(os.environ.get("GR_FIT_TILE", "32"))
# How the fused step is enqueued (world size 1; ViewShardedFitter._graph_step): the views are prepared against per-view
# pair capacities (gr_fwd_prepare_views_sized: the counts stay on the device, nothing in the step waits for the host),
# the Adam scalars come from a device table indexed by a device step counter, and a step whose views exceed their
# capacities updates nothing and is redone with larger ones.  Modes (GR_GRAPH):
#   batch       every kernel launched once per batch of up to 8 views (gr_fit_views_batched), one stream: small views
#               fill the GPU (C3 580 -> 765, C2 2,020 -> 2,720 Mpx/s, profiles/r05_batched.txt)
#   batchgraph  that step captured once as a HIP graph and replayed
#   1           the multi-stream step captured and replayed (ROCm runs a captured graph's branches at most two at a
#               time here: slower than eager, profiles/r05_graph_ab.txt)
#   sized/exec  the device-sized multi-stream step enqueued eagerly, Python / native executor (diagnostics)
#   0           the eager multi-stream step, host-sized
#   auto        (default) batch for views of at most GRAPH_AUTO_PIXELS, else 0: at 800x800 the per-view launches already
#               fill the GPU and the eager step's stream overlap wins (C4 1,557 eager vs 1,446 batched)
GRAPH_MODE = os.environ.get("GR_GRAPH", "auto")
GRAPH_AUTO_PIXELS = 512 * 512
# multi-GPU: the r = V mod R views left over by the even split are cut into bands of tile rows (gr_view.row0 / rows),
# the ranks split into r groups, one per leftover view, each group cutting its view into as many bands as it has ranks:
# every rank renders V // R views and ONE band (50 views on 8 ranks: 6 views and a quarter view each instead of 7 on
# two ranks; round 5 gave every rank a band of every leftover view, two eighths, each paying a band's fixed cost); the
# fused path without a depth term only (a depth term needs the whole image's depth maximum).  0 = whole views round-robin.
BAND_SPLIT = os.environ.get("GR_BAND_SPLIT", "1") != "0"
# a band costs about this fraction of a whole view beyond its share of the view's pairs (its preparation, binning
# launches, gather and chain rule run over every Gaussian: ~90 of ~560 us single-stream at C4, tools/band_probe.py;
# more in the overlapped step): the split is used when the most loaded rank's band (this plus its largest share of the
# pairs) is below a whole view.  Measured per rank (profiles/r06_rank_share.txt): C4 at 8 ranks, quarter-view bands
# (29% of the pairs): 3.25 -> 3.02-3.10 ms for every rank; at 4 ranks, half-view bands: 5.82 -> 6.13-6.19, so 0.5 keeps
# whole views there
BAND_OVERHEAD = float(os.environ.get("GR_BAND_OVERHEAD", "0.5"))
GRAPH_MARGIN = float(os.environ.get("GR_GRAPH_MARGIN", "1.25"))  # capacity over the counts seen (+ 4096 pairs)


# ------------------------------------------------------------------------------------------------
# Parameters (fit_multiview_stub.py:114-137) — CPU RNG, then moved to the device.
# ------------------------------------------------------------------------------------------------
def build_params(n: int, device: torch.device, use_sh: bool, sh_degree: int = 1) -> dict:
    """sh_degree 3 (extension, config C3): (N,16,3) coefficients, the degree-1 init of the stub plus
    zero degree-2/3 terms."""
    means = (torch.rand((n, 3)) - 0.5) * 1.2
    scales_raw = torch.full((n, 3), -2.2)
    opacities_raw = torch.full((n,), -2.2)
    params = {"means": means, "scales_raw": scales_raw, "opacities_raw": opacities_raw}
    if use_sh:
        sh = torch.zeros((n, 16 if sh_degree == 3 else 4, 3))
        sh[:, 0, :] = 0.1 * torch.rand((n, 3))
        params["sh_raw"] = sh
    else:
        params["colors_raw"] = 0.1 * torch.rand((n, 3))
    return {k: torch.nn.Parameter(v.to(device)) for k, v in params.items()}


def activations(params: dict):
    """fit_multiview_stub.py:268-275.  Leaf parameters used as they are (means, SH coefficients) pass
    through a view, so the per-view gradients that arrive from the render streams meet in a node made on
    this (the main) stream rather than in the leaf's accumulator."""
    means = params["means"].view(params["means"].shape)
    scales = torch.nn.functional.softplus(params["scales_raw"]) + 1e-3
    opacities = torch.sigmoid(params["opacities_raw"])
    colors = params["sh_raw"].view(params["sh_raw"].shape) if "sh_raw" in params else torch.sigmoid(params["colors_raw"])
    return means, scales, colors, opacities


def activations_native(params: dict, reg=None, ws=None):
    """activations() in one HIP launch (gr_fit_activations: the same float formulas as torch's softplus and
    sigmoid), for the fused step, which needs no autograd graph; with reg = (reg_opacity, reg_scale) also the
    regulariser reg_opacity * mean(opacities) + reg_scale * mean(scales) (fit_multiview_stub.py:307-308) as a 0-d
    device tensor, summed in the same launch (ws: a zeroed uint8 tensor of gr_fit_activations_ws_bytes).
    Returns (means, scales, colors, opacities, reg or None)."""
    nat = tr._native
    L = nat.lib()
    means = params["means"].detach()
    sr, orw = params["scales_raw"].detach().contiguous(), params["opacities_raw"].detach().contiguous()
    cr = params["colors_raw"].detach().contiguous() if "colors_raw" in params else None
    n = int(means.shape[0])
    scales, opacities = torch.empty_like(sr), torch.empty_like(orw)
    colors = torch.empty_like(cr) if cr is not None else params["sh_raw"].detach()
    out = torch.empty((), dtype=torch.float32, device=means.device) if reg is not None and n > 0 else None
    nat.check(L.gr_fit_activations(n, nat.ptr(sr), nat.ptr(orw), nat.ptr(cr) if cr is not None else None,
                                   int(cr.numel()) if cr is not None else 0, nat.ptr(scales), nat.ptr(opacities),
                                   nat.ptr(colors) if cr is not None else None,
                                   ctypes.c_float(reg[1] if reg else 0.0), ctypes.c_float(reg[0] if reg else 0.0),
                                   nat.ptr(out) if out is not None else None,
                                   ws.data_ptr() if ws is not None else None, ws.numel() if ws is not None else 0,
                                   ctypes_stream(means.device)), "gr_fit_activations")
    return means, scales, colors, opacities, out


def densify_and_prune(params: dict, max_gaussians: int, densify_ratio: float, prune_opacity: float) -> dict:
    """fit_multiview_stub.py:140-197, evaluated on the host (CPU RNG for the jitter) so that every
    rank that calls it with the same RNG state gets identical parameters."""
    with torch.no_grad():
        cpu = {k: v.detach().cpu() for k, v in params.items()}
        means, scales_raw, op_raw = cpu["means"], cpu["scales_raw"], cpu["opacities_raw"]
        op = torch.sigmoid(op_raw)
        scales = torch.nn.functional.softplus(scales_raw) + 1e-3
        keep = op > prune_opacity
        if int(keep.sum()) < 64:
            top_keep = torch.topk(op, k=min(64, op.shape[0]), largest=True).indices
            keep = torch.zeros_like(keep, dtype=torch.bool)
            keep[top_keep] = True
        means, scales_raw, op_raw, scales = means[keep], scales_raw[keep], op_raw[keep], scales[keep]
        op = torch.sigmoid(op_raw)
        n = means.shape[0]
        room = max(0, max_gaussians - n)
        add_n = min(room, max(0, int(n * densify_ratio)))
        if add_n > 0 and n > 0:
            idx = torch.topk(op, k=min(n, add_n), largest=True).indices
            jitter = 0.25 * scales[idx] * torch.randn_like(means[idx])
            means = torch.cat([means, means[idx] + jitter], dim=0)
            scales_raw = torch.cat([scales_raw, scales_raw[idx]], dim=0)
            op_raw = torch.cat([op_raw, op_raw[idx] - 0.1], dim=0)
        out = {"means": means, "scales_raw": scales_raw, "opacities_raw": op_raw}
        key = "sh_raw" if "sh_raw" in cpu else "colors_raw"
        col = cpu[key][keep]
        if add_n > 0 and col.shape[0] > 0:
            base_n = col.shape[0]
            idx = torch.topk(torch.sigmoid(op_raw[:base_n]), k=min(base_n, add_n), largest=True).indices
            col = torch.cat([col, col[idx]], dim=0)
        out[key] = col
    device = params["means"].device
    return {k: torch.nn.Parameter(v.to(device)) for k, v in out.items()}


def densify_and_prune_device(params: dict, max_gaussians: int, densify_ratio: float, prune_opacity: float,
                             generator: Optional[torch.Generator] = None, noise: Optional[torch.Tensor] = None) -> dict:
    """The same rule as densify_and_prune (fit_multiview_stub.py:140-197) evaluated on the device, for
    fits at scale (config C5: millions of Gaussians), with the jitter drawn from a device generator:
    no host round trip of the parameters.  Same keep / top-k / jitter / -0.1 opacity / colour
    duplication; only the random stream differs from the stub's CPU one.  ``noise`` (>= added rows x 3,
    standard normal) replaces the generator's draw: with the stub's own draw the result is the host
    rule's (tests/test_densify.py)."""
    with torch.no_grad():
        means, scales_raw, op_raw = params["means"].detach(), params["scales_raw"].detach(), params["opacities_raw"].detach()
        key = "sh_raw" if "sh_raw" in params else "colors_raw"
        col = params[key].detach()
        op = torch.sigmoid(op_raw)
        keep = op > prune_opacity
        if int(keep.sum()) < 64:
            top_keep = torch.topk(op, k=min(64, op.shape[0]), largest=True).indices
            keep = torch.zeros_like(keep, dtype=torch.bool)
            keep[top_keep] = True
        means, scales_raw, op_raw, col = means[keep], scales_raw[keep], op_raw[keep], col[keep]
        n = means.shape[0]
        room = max(0, max_gaussians - n)
        add_n = min(room, max(0, int(n * densify_ratio)))
        if add_n > 0 and n > 0:
            idx = torch.topk(torch.sigmoid(op_raw), k=min(n, add_n), largest=True).indices
            scales = torch.nn.functional.softplus(scales_raw[idx]) + 1e-3
            if noise is not None:
                z = noise[:idx.shape[0]].to(device=means.device, dtype=means.dtype)
            else:
                z = torch.randn(means[idx].shape, generator=generator, device=means.device, dtype=means.dtype)
            jitter = 0.25 * scales * z
            means = torch.cat([means, means[idx] + jitter], dim=0)
            scales_raw = torch.cat([scales_raw, scales_raw[idx]], dim=0)
            col = torch.cat([col, col[idx]], dim=0)
            op_raw = torch.cat([op_raw, op_raw[idx] - 0.1], dim=0)
        out = {"means": means, "scales_raw": scales_raw, "opacities_raw": op_raw, key: col}
    return {k: torch.nn.Parameter(v.contiguous()) for k, v in out.items()}


def spatial_order(params: dict) -> dict:
    """The same Gaussians, permuted into morton_order (a layout choice of the trainer: the rendered
    images and the loss do not depend on the order of the Gaussians beyond float summation order)."""
    if params["means"].shape[0] < 2:
        return params
    perm = morton_order(params["means"])
    return {k: torch.nn.Parameter(v.detach()[perm].contiguous()) for k, v in params.items()}


def _fit_images(name: str, imgs: Optional[list], shape: tuple, device) -> tuple:
    """The fused fit path reads the targets / masks / depths through raw device pointers (gr_fwd_render_l1,
    gr_bwd_fit): each must be exactly ``shape``, float32, contiguous, on the parameters' device.  Returns
    (images, ok): images normalised to that (a copy only where the dtype, layout or device differ), ok =
    False when a shape differs (the fit then takes the autograd path, which broadcasts or raises as torch
    does for the stub's expressions)."""
    if imgs is None:
        return None, True
    if any(tuple(t.shape) != shape for t in imgs):
        return list(imgs), False
    return [torch.as_tensor(t).to(device=device, dtype=torch.float32).contiguous() for t in imgs], True


def _batch_sizes(ns: int, nviews: int, tail: Optional[int] = None) -> list:
    """Per stream (views j = k, k + ns, ...): its views' reduction batches, near-equal and at most REDUCE_BATCH, in
    the order they fill; a short last batch of REDUCE_TAIL views (the reductions left when the renders end run alone).
    The native executor's schedule() is the same rule."""
    sizes = []
    for k in range(ns):
        p = len(range(k, nviews, ns))
        rt = REDUCE_TAIL if tail is None else tail
        t = min(rt, REDUCE_BATCH) if 0 < rt < p else 0  # (gr_fit_views: tail <= batch)
        nb = max(1, -(-(p - t) // REDUCE_BATCH))
        sizes.append([(p - t) // nb + (1 if b < (p - t) % nb else 0) for b in range(nb)] + ([t] if t else []))
    return sizes


def _int_hist(idx: torch.Tensor, wts: torch.Tensor, nb: int) -> torch.Tensor:
    """Sum of the int64 weights per bin 0..nb-1 (indices in range): sorted indices, prefix sums, bin ends."""
    srt, order = torch.sort(idx)
    cw = torch.cumsum(wts[order], 0)
    ends = torch.searchsorted(srt, torch.arange(nb, device=idx.device, dtype=srt.dtype), right=True)
    upto = torch.where(ends > 0, cw[(ends - 1).clamp_min(0)], torch.zeros_like(ends))
    return torch.diff(upto, prepend=torch.zeros(1, dtype=upto.dtype, device=upto.device))


def _min_max_cuts(w, g: int) -> list:
    """Boundaries 0 = c_0 < c_1 < ... < c_g = len(w) of g non-empty contiguous runs of `w` whose largest sum is
    the smallest possible (dynamic programming over the cut positions; ties to the earliest cut)."""
    n = len(w)
    c = np.concatenate([[0.0], np.cumsum(np.asarray(w, np.float64))])
    best = np.full((g + 1, n + 1), np.inf)
    arg = np.zeros((g + 1, n + 1), np.int64)
    best[0, 0] = 0.0
    for k in range(1, g + 1):
        for j in range(k, n - (g - k) + 1):
            for i in range(k - 1, j):
                v = max(best[k - 1, i], c[j] - c[i])
                if v < best[k, j]:
                    best[k, j], arg[k, j] = v, i
    cuts = [n]
    for k in range(g, 0, -1):
        cuts.append(int(arg[k, cuts[-1]]))
    return cuts[::-1]


def bucketed_all_reduce(buckets: list, assemble: Callable[[int], None], finish: Callable[[int], None], group=None) -> None:
    """The step's one real exchange (SUM over ranks) in buckets, one per parameter tensor (plus the loss in
    the last): bucket b is assembled (``assemble(b)``, on the current stream) and its all-reduce issued
    asynchronously at once, so RCCL moves bucket b over xGMI while bucket b + 1 is assembled; then each
    bucket's update (``finish(b)``) waits for its own all-reduce only.  Summation order per element is the
    collective's, as for one flat buffer."""
    works = []
    for b in range(len(buckets)):
        assemble(b)
        works.append(dist.all_reduce(buckets[b], op=dist.ReduceOp.SUM, group=group, async_op=True))
    for b, w in enumerate(works):
        w.wait()
        finish(b)


def hip_render(means, scales, colors, opacities, cam, width, height, background, prepared=None, depth_grad=True):
    return tr.render_gaussians_torch(means, scales, colors, opacities, cam, width=width, height=height,
                                     background=background, max_gaussians=max(10000, int(means.shape[0])), return_aux=True,
                                     prepared=prepared, depth_grad=depth_grad)


class _EagerReplay:
    """GR_GRAPH=sized: replay() enqueues the device-sized step again instead of launching a captured graph."""

    def __init__(self, body, gs):
        self.body, self.gs = body, gs

    def replay(self):
        self.gs.loss = self.body()


class _GraphState:
    """The captured fused step (ViewShardedFitter._graph_build) and its device-side sizing state."""

    def __init__(self):
        self.graph = None
        self.key = None
        self.sched = None
        self.sched_len = 0
        self.sched_key = None
        self.overflows = 0  # steps redone with larger capacities (tests, bench)
        self.builds = 0  # captures
        self.inflight = []


class ViewShardedFitter:
    """One fit iteration = render own views, backward, one gradient all-reduce, Adam.

    On the fused path every parameter's ``.grad`` after ``step()`` is a tensor the fitter keeps and overwrites in
    place on the next step (no allocation per step): copy it to keep a step's gradient."""

    def __init__(self, params: dict, cams: list, targets: list, width: int, height: int, lr: float = 0.02,
                 masks: Optional[list] = None, depths: Optional[list] = None, silhouette_weight: float = 0.2,
                 depth_weight: float = 0.05, reg_opacity: float = 1e-3, reg_scale: float = 1e-3,
                 render_fn: RenderFn = hip_render, group=None, reorder: bool = True):
        # reorder: keep the Gaussians in spatial (Morton) order, re-established after every
        # densify/prune (spatial_order); off only to compare with an unpermuted run
        # perm: self.params[k][i] = canonical[k][perm[i]], the canonical order being the stub's (the
        # order densify_and_prune and gaussians_fitted.npz see: top-k ties and jitter draws follow it)
        self.reorder = reorder
        self.perm = None
        self.group = group
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            # data parallelism needs identical replicas: rank 0's initial parameters win (the Morton
            # permutation below is then computed from identical means on every rank)
            src = dist.get_global_rank(group, 0) if group is not None else 0
            for k in sorted(params):
                dist.broadcast(params[k].data, src, group=group)
        if reorder and params["means"].shape[0] >= 2:
            self.perm = morton_order(params["means"])
            params = {k: torch.nn.Parameter(v.detach()[self.perm].contiguous()) for k, v in params.items()}
        self.params = params
        dev = params["means"].device
        targets, ok_t = _fit_images("targets", targets, (height, width, 3), dev)
        masks, ok_m = _fit_images("masks", masks, (height, width), dev)
        depths, ok_d = _fit_images("depths", depths, (height, width), dev)
        self._images_ok = ok_t and ok_m and ok_d  # the fused path's exact-shape precondition
        self.cams, self.targets, self.masks, self.depths = cams, targets, masks, depths
        self.width, self.height, self.lr = width, height, lr
        self.w_sil, self.w_depth = silhouette_weight, depth_weight
        self.reg_opacity, self.reg_scale = reg_opacity, reg_scale
        self.render_fn = render_fn
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.world = dist.get_world_size(group) if self.distributed else 1
        self._rr_views = list(range(self.rank, len(targets), self.world))
        self._bands = {}  # virtual view id (>= V) -> (view, first tile row, tile rows) of this rank's bands
        self.opt = torch.optim.Adam(list(self.params.values()), lr=lr)
        self.densify_seed = 1234
        self.steps_done = 0

    def canonical_params(self) -> dict:
        """The parameters in the stub's order (undoes the trainer's Morton permutation)."""
        self.graph_sync()
        if self.perm is None:
            return self.params
        out = {}
        for k, v in self.params.items():
            c = torch.empty_like(v.detach())
            c[self.perm] = v.detach()
            out[k] = torch.nn.Parameter(c)
        return out

    def respatialize(self) -> None:
        """Re-establish the Morton order of the Gaussians as they move during the fit: parameters and
        Adam moments are permuted in place (the optimizer keeps its state), self.perm follows."""
        if not self.reorder or self.params["means"].shape[0] < 2:
            return
        with torch.no_grad():
            p2 = morton_order(self.params["means"])
            for p in self.params.values():
                p.data.copy_(p.data[p2])
                st = self.opt.state.get(p)
                if st:
                    for k in ("exp_avg", "exp_avg_sq"):
                        if k in st:
                            st[k].copy_(st[k][p2])
            self.perm = p2 if self.perm is None else self.perm[p2]

    def reset_optimizer(self) -> None:
        self.opt = torch.optim.Adam(list(self.params.values()), lr=self.lr)

    def _background(self, device) -> torch.Tensor:
        # one persistent tensor: the renderer reads its value on the host once, not per view
        if getattr(self, "_bg", None) is None or self._bg.device != device:
            self._bg = torch.zeros(3, device=device)
        return self._bg

    @property
    def my_views(self) -> list:
        """This rank's views: i = r, r + R, ... (whole views), or with band splitting the first R * (V // R) views
        round-robin and this rank's band of its group's leftover view (a virtual id V + i, _vi / _bands)."""
        if not self._bands_ok():
            return self._rr_views
        V, W = len(self.targets), self.world
        q = V // W
        whole = list(range(self.rank, q * W, W))
        band = self._band_of(self.rank)
        if band is None:  # (more ranks in the group than the view has tile rows: this rank renders no band)
            return whole
        i, lo, rows = band
        self._bands[V + i] = band
        return whole + [V + i]

    def _band_groups(self) -> list:
        """[(leftover view, first rank, ranks)]: the R ranks in r = V mod R contiguous groups, one per leftover view."""
        V, W = len(self.targets), self.world
        r = V % W
        return [(V - r + j, j * W // r, (j + 1) * W // r - j * W // r) for j in range(r)]

    def _band_of(self, rank: int):
        """(view, first tile row, tile rows) of `rank`'s band, or None (its group's view has fewer tile rows than ranks)."""
        for i, r0, g in self._band_groups():
            if r0 <= rank < r0 + g:
                cuts = self._band_cuts(i, g)
                k = rank - r0
                return (i, cuts[k], cuts[k + 1] - cuts[k]) if cuts[k + 1] > cuts[k] else None
        return None

    def _band_cuts(self, i: int, g: int) -> list:
        """Tile-row boundaries cutting view i into g bands of about equal work: a band's time is a fixed part plus its
        (Gaussian, tile) pairs (tools/band_probe.py: ~90 us + ~130 us per million pairs at C4, single stream), and a
        scene's pairs crowd the middle rows (view 48 of C4: rows 6-18 of 25 hold 97% of them), so equal rows left the
        middle bands twice the edge ones' work.  The pairs per row are estimated from the Gaussians' projected 5-sigma
        boxes (rows x tile columns touched), recomputed with the Morton re-sort and after densify; every rank computes
        the same cuts from its identical replica."""
        tile = self.views_tile()
        ty = -(-self.height // tile)
        key = (i, g, tile, int(self.params["means"].shape[0]), self.steps_done // max(1, RESORT_EVERY))
        cache = self.__dict__.setdefault("_cuts_cache", {})
        if key in cache:
            return cache[key]
        if len(cache) > 64:
            cache.clear()
        w = self._row_pairs_cached(i, tile, ty)
        cuts = _min_max_cuts(w, g) if ty >= g else [ty * k // g for k in range(g + 1)]
        cache[key] = cuts
        return cuts

    def _row_pairs_cached(self, i: int, tile: int, ty: int) -> np.ndarray:
        key = (i, tile, int(self.params["means"].shape[0]), self.steps_done // max(1, RESORT_EVERY))
        cache = self.__dict__.setdefault("_rows_cache", {})
        if key not in cache:
            if len(cache) > 64:
                cache.clear()
            cache[key] = self._row_pairs(i, tile, ty)
        return cache[key]

    def _row_pairs(self, i: int, tile: int, ty: int) -> np.ndarray:
        """Estimated (Gaussian, tile) pairs per tile row of view i: per Gaussian the tile rows and columns of its
        FIT_CUTOFF-sigma box (torch_renderer.py:57-78, 146-150's projection and sigma rule; rectangle, not the
        elliptical test), summed over the rows it spans (a difference array)."""
        with torch.no_grad():
            m, sc, _, _ = activations(self.params)
            cam = self.cams[i]
            V, P = cam.view.float(), cam.proj.float()
            pc = m.float() @ V[:3, :3].T + V[:3, 3]
            clip = pc @ P[:3, :3].T + P[:3, 3]
            w4 = pc @ P[3, :3] + P[3, 3]
            ws = torch.where(w4.abs() < 1e-8, torch.ones_like(w4), w4)
            ndc = clip / ws[:, None]
            ok = (ndc[:, 2] >= -1) & (ndc[:, 2] <= 1) & (w4 != 0)
            px = (ndc[:, 0] * 0.5 + 0.5) * (self.width - 1)
            py = (1 - (ndc[:, 1] * 0.5 + 0.5)) * (self.height - 1)
            za = pc[:, 2].abs().clamp_min(1e-6)
            sx = (sc[:, 0].abs() * 0.5 * self.width * P[0, 0].abs() / za).clamp_min(1.0) * tr.FIT_CUTOFF
            sy = (sc[:, 1].abs() * 0.5 * self.height * P[1, 1].abs() / za).clamp_min(1.0) * tr.FIT_CUTOFF
            tx = -(-self.width // tile)
            c0 = ((px - sx) / tile).floor().clamp(0, tx - 1)
            c1 = ((px + sx) / tile).floor().clamp(0, tx - 1)
            r0 = ((py - sy) / tile).floor().clamp(0, ty - 1)
            r1 = ((py + sy) / tile).floor().clamp(0, ty - 1)
            ok = ok & (px + sx >= 0) & (px - sx <= self.width - 1) & (py + sy >= 0) & (py - sy <= self.height - 1)
            cols = torch.where(ok, c1 - c0 + 1, torch.zeros_like(c0)).long()
            # a difference array of integer counts, summed without atomics (a sort, a prefix sum and a search): exact
            # and the same on every rank (an index_add_ of float64 took 28 ms per view at C4)
            d = _int_hist(r0.long(), cols, ty + 1) - _int_hist((r1 + 1).long(), cols, ty + 1)
            return torch.cumsum(d, 0)[:ty].double().cpu().numpy()

    def views_tile(self) -> int:
        """The tile size the fused path renders this fit's views at: FIT_TILE, or 16 in the f32-grade mode (its
        three-piece splits have 16-pixel kernels only)."""
        return (16 if F32_GRADE else FIT_TILE) or 16

    def _bands_ok(self) -> bool:
        V, W = len(self.targets), self.world
        r = V % W if W > 1 else 0
        if not (BAND_SPLIT and r and not self._depth_grad()):
            return False
        if self.params["means"].shape[0] == 0:  # (the generic loop renders whole views only)
            return False
        dev = self.params["means"].device
        if not (dev.type == "cuda" and self._direct(dev)):
            return False
        # the most loaded rank: V // R views and one band, its largest share of its view's pairs plus the band's fixed
        # cost (a group of one renders its whole view, no band cost): bands only where that beats a whole view
        load = max((1.0 if g == 1 else BAND_OVERHEAD + self._band_share(i, g)) for i, _, g in self._band_groups())
        return load < 1.0

    def _band_share(self, i: int, g: int) -> float:
        """The largest band's share of view i's estimated pairs when cut into g bands (_band_cuts)."""
        tile = self.views_tile()
        w = self._row_pairs_cached(i, tile, -(-self.height // tile))
        cuts = self._band_cuts(i, g)
        tot = float(w.sum())
        return max(float(w[cuts[k]:cuts[k + 1]].sum()) for k in range(g)) / tot if tot > 0 else 1.0 / g

    def _vi(self, v: int) -> int:
        """The view index of a (possibly virtual, band) view id."""
        return v - len(self.targets) if v >= len(self.targets) else v

    def _depth_grad(self) -> bool:
        """The loss differentiates the depth output (a depth term): the views render in the default
        precision mode with the depth-gradient cutoff; otherwise depth_grad=False (gr_view.no_depth_grad)."""
        return self.depths is not None and self.w_depth > 0.0

    def _prepare(self, i: int, means, scales, colors, opacities, fit_view: bool = False, plan_host=None):
        """fit_view: a view of the fused path (_views_direct): one zone at tr.FIT_CUTOFF."""
        cam = self.cams[i]
        cut = tr.FIT_CUTOFF if fit_view else None
        return tr.prepare_view(means, scales, colors, opacities, cam.view, cam.proj, self.width, self.height,
                               self._background(means.device), cutoff=cut,
                               core_cutoff=tr.FIT_CUTOFF if fit_view else tr.DEFAULT_CORE_CUTOFF,
                               depth_grad="eager" if self._depth_grad() else False, plan_host=plan_host)

    @staticmethod
    def _prep_groups(views, ahead: dict, prepare_views: Callable, prep) -> Callable[[int], None]:
        """prepare_upto(j): the views up to j prepared on stream `prep` (whole groups, in order: the first
        PREP_FIRST views, then PREP_GROUP at a time; their states go to `ahead`).  Called with the first two
        groups at once, then after each render (its j + PREP_AHEAD): the step's first render is launched
        before the host spends time on later groups (a 7-view step waited ~180 us for them)."""
        nxt = [0]

        def prepare_upto(j):
            while nxt[0] <= j and nxt[0] < len(views):
                j0 = nxt[0]
                js = range(j0, min(len(views), j0 + (PREP_FIRST if j0 == 0 else PREP_GROUP)))
                with torch.cuda.stream(prep):
                    ahead.update(zip(js, prepare_views(js)))
                nxt[0] = js.stop

        prepare_upto(min(PREP_FIRST, PREP_AHEAD - 1) if PREP_INITIAL > 1 else 0)
        return prepare_upto

    def _fit_view(self, i: int, device) -> "tr._native.GrView":
        """The gr_view of view i for the fused path (one FIT_CUTOFF zone, no depth gradient), built once:
        cameras and background do not change during a fit (saves the host's matrix inverse and copies
        twice per view and step).  A band id (>= V): that view with its band of tile rows."""
        if i >= len(self.targets):
            b = getattr(self, "_band_gv", None)
            if b is None:
                self._band_gv = b = {}
            key = (i, F32_GRADE, FIT_TILE) + self._bands[i]
            gv = b.get(key)
            if gv is None:
                base, row0, rows = self._bands[i]
                gv = b[key] = tr._native.GrView.from_buffer_copy(self._fit_view(base, device))
                gv.row0, gv.rows = row0, rows
            return gv
        cache = getattr(self, "_gv_cache", None)
        if cache is None:
            self._gv_cache = cache = {}
        gv = cache.get((i, F32_GRADE, FIT_TILE))
        if gv is None:
            cam = self.cams[i]
            gv = cache[(i, F32_GRADE, FIT_TILE)] = tr.make_view(cam.view, cam.proj, self.width, self.height,
                                                      self._background(device), cutoff=tr.FIT_CUTOFF,
                                                      core_cutoff=tr.FIT_CUTOFF, depth_grad=False,
                                                      tile=0 if F32_GRADE else FIT_TILE)
            if F32_GRADE:
                gv.no_depth_grad = 2
        return gv

    def _plan_pins(self, count: int) -> torch.Tensor:
        """One pinned (count, 3) int64 buffer for the views' plans, kept across steps (a pinned allocation
        per view and step costs host time on the render path)."""
        pins = getattr(self, "_pins", None)
        if pins is None or pins.shape[0] < count:
            self._pins = pins = torch.zeros((max(count, 1), 3), dtype=torch.int64, pin_memory=True)
        return pins

    def view_loss(self, i: int, means, scales, colors, opacities, prepared=None) -> torch.Tensor:
        device = means.device
        kw = {} if prepared is None else {"prepared": prepared}
        if self.render_fn is hip_render:
            # without a depth loss the depth output gets no gradient: the forward may accumulate W and D
            # at the colours' precision (gr_view.no_depth_grad)
            kw["depth_grad"] = "eager" if self._depth_grad() else False  # a depth loss differentiates depth
        pred, alpha, depth = self.render_fn(means, scales, colors, opacities, self.cams[i], self.width, self.height,
                                            self._background(device), **kw)
        use_sil = self.masks is not None and self.w_sil > 0.0
        if self.render_fn is hip_render and pred.device.type == "cuda" and FUSED_LOSS:
            # photometric + silhouette L1 fused on the device (losses.l1_loss); same value and gradient
            loss = losses.l1_loss(pred, self.targets[i], alpha if use_sil else None,
                                  self.masks[i] if use_sil else None, self.w_sil if use_sil else 0.0)
        else:
            loss = torch.mean(torch.abs(pred - self.targets[i]))
            if use_sil:
                loss = loss + self.w_sil * torch.mean(torch.abs(alpha - self.masks[i]))
        if self.depths is not None and self.w_depth > 0.0:
            d_pred = depth / (depth.max() + 1e-6)
            loss = loss + self.w_depth * torch.mean(torch.abs(d_pred - self.depths[i]))
        return loss

    def _direct(self, device) -> bool:
        """The fused path (_views_direct, or _views_direct_depth with a depth term): HIP render op, the
        view loss and its gradients in the C ABI, no autograd per view.  Needs float32 parameters and
        targets / masks / depths of exactly the image's shape (checked at construction)."""
        return (self.render_fn is hip_render and device.type == "cuda" and FUSED_LOSS and DIRECT_BACKWARD
                and self._images_ok and all(p.dtype == torch.float32 for p in self.params.values()))

    def step(self) -> torch.Tensor:
        """One iteration; returns the full (all-rank) loss as a 0-d tensor on the device."""
        if RESORT_EVERY and self.steps_done and self.steps_done % RESORT_EVERY == 0:
            self.respatialize()
        self.steps_done += 1
        device = self.params["means"].device
        if self._graph_ok(device):
            return self._graph_step(device)
        self._graph_leave()
        self.opt.zero_grad(set_to_none=True)
        if self._direct(device) and self.params["means"].shape[0] > 0 and self._fused_step_ok():
            with torch.no_grad():
                means, scales, colors, opacities, reg_t = self._activations_fused(device)
                reg_fn = (lambda: reg_t) if reg_t is not None else None
                reg = None
                if self._native_exec() and GATHER:
                    total = self._views_native(means, scales, colors, opacities, self._depth_grad())
                    # the regulariser's small kernels after the executor's call (the host starts the views'
                    # preparations first), on the preparation stream behind the last preparation when the executor
                    # runs on this driver's streams (as the Python schedule does; no extra hardware queue)
                    rs = getattr(self, "_prep", None) if EXEC_STREAMS else None
                    if reg_fn and rs is not None:
                        main = torch.cuda.current_stream(device)
                        with torch.cuda.stream(rs):
                            reg = reg_fn()
                        reg.record_stream(main)  # allocated on rs, read on main: not reused by rs early
                        main.wait_stream(rs)
                    elif reg_fn:
                        reg = reg_fn()
                elif self._depth_grad():
                    reg = reg_fn() if reg_fn else None
                    total = self._views_direct_depth(means, scales, colors, opacities)
                else:
                    # the regulariser's small kernels run on the preparation stream once the last
                    # preparation is enqueued: neither before the first view nor between the last
                    # reduction and the parameter update
                    total, reg = self._views_direct(means, scales, colors, opacities, reg_fn)
                loss = total / len(self.targets)
                if reg is not None:
                    loss = loss + reg
            return self._fused_param_step(scales, opacities, loss)
        means, scales, colors, opacities = activations(self.params)
        if self._direct(device) and means.shape[0] > 0:
            if self._depth_grad():
                total = self._views_direct_depth(means, scales, colors, opacities)
            else:
                total, _ = self._views_direct(means, scales, colors, opacities)
            parts = self._acc_parts
            acc = []
            for q in range(4):  # in stream order
                t = parts[0][q]
                for pp in parts[1:]:
                    t = t + pp[q]
                acc.append(t)
            self._acc = tuple(acc)
            loss = total / len(self.targets)
            if self.rank == 0:
                reg = self.reg_opacity * opacities.mean() + self.reg_scale * scales.mean()
                loss = loss + reg.detach()
                torch.autograd.backward([means, scales, colors, opacities, reg], list(self._acc) + [None])
            else:
                torch.autograd.backward([means, scales, colors, opacities], list(self._acc))
            self._acc = None
            return self._finish_step(loss)
        # HIP renderer: the next view's preparation is enqueued before this view renders, so the
        # host reads each view's pair count while the device is still busy (no idle gap per view);
        # views rotate over NUM_STREAMS HIP streams, so one view's latency-bound binning kernels run
        # beside another's splat kernels (autograd runs each view's backward on its forward stream)
        prefetch = self.render_fn is hip_render and means.device.type == "cuda" and means.shape[0] > 0
        streams = [None]
        ns = min(NUM_STREAMS, len(self.my_views))
        if prefetch and ns > 1:
            main = torch.cuda.current_stream(device)
            side = getattr(self, "_side", None)
            if side is None or len(side) != ns - 1 or side[0].device != device:
                self._side = side = [torch.cuda.Stream(device) for _ in range(ns - 1)]
            for st in side:
                st.wait_stream(main)  # the activations are produced on the main stream
            streams = [main] + side
        # per-stream accumulators start empty and are created by their stream's first view (a zeros
        # tensor made here on the main stream would be read by a side stream with no ordering)
        totals: list = [None for _ in streams]
        views = self.my_views

        def on(j):
            s = streams[j % len(streams)]
            return torch.cuda.stream(s) if s is not None else contextlib.nullcontext()

        # preparations run PREFETCH views ahead (each on its view's stream), so the host's wait for a
        # view's pair count is for work enqueued well before
        ahead = {}

        def prepare(j):
            if prefetch and j < len(views) and j not in ahead:
                with on(j):
                    ahead[j] = self._prepare(views[j], means, scales, colors, opacities)

        for j in range(PREFETCH):
            prepare(j)
        for j, i in enumerate(views):
            prepare(j + PREFETCH)
            with on(j):
                k = j % len(streams)
                lv = self.view_loss(i, means, scales, colors, opacities, prepared=ahead.pop(j, None))
                totals[k] = lv if totals[k] is None else totals[k] + lv
        for st in streams[1:]:
            streams[0].wait_stream(st)
        total = None
        for t in totals:
            if t is not None:
                total = t if total is None else total + t
        if total is None:
            # a rank with no views (world size > number of views): a zero loss that still reaches every
            # parameter, so backward() runs and the rank joins the all-reduce with zero gradients
            total = sum(p.sum() for p in self.params.values()) * 0.0
        loss = total / len(self.targets)
        if self.rank == 0:
            loss = loss + self.reg_opacity * opacities.mean() + self.reg_scale * scales.mean()
        loss.backward()
        return self._finish_step(loss)

    def _native_exec(self) -> bool:
        """Whether this step's views go through the native executor (GR_NATIVE_EXEC)."""
        if NATIVE_EXEC == "auto":
            return self.width * self.height <= NATIVE_EXEC_MAX_PIXELS
        return str(NATIVE_EXEC) not in ("0", "False", "")

    def _views_native(self, means, scales, colors, opacities, depth: bool, sized=None) -> torch.Tensor:
        """_views_direct / _views_direct_depth through the native executor (gr_fit_views): one C call per
        step; returns the sum of the view losses and leaves the stream accumulators in self._acc_parts."""
        device = means.device
        m, s, c, o = (t.detach().float().contiguous() for t in (means, scales, colors, opacities))
        views = self.my_views
        if not views:
            self._acc_parts = [tuple(torch.zeros_like(t) for t in (m, s, c, o))]
            return torch.zeros((), device=device)
        ns = max(1, min(NUM_STREAMS, len(views)))
        w_sil = self.w_sil if (self.masks is not None and self.w_sil > 0.0) else 0.0
        key = (tuple(views), depth, F32_GRADE, w_sil > 0.0, str(device), sized is not None)
        cache = getattr(self, "_native_targets", None)
        if cache is None or cache[0] != key:
            arr = (tr._native.GrFitTarget * len(views))()
            for j, i in enumerate(views):
                if depth:
                    cam = self.cams[i]
                    gvd = getattr(self, "_gvd_cache", None)
                    if gvd is None:
                        self._gvd_cache = gvd = {}
                    if i not in gvd:
                        gvd[i] = tr.make_view(cam.view, cam.proj, self.width, self.height, self._background(device),
                                              depth_grad=True)
                    arr[j].view = gvd[i] if sized is None else tr.sized_view(gvd[i])
                    arr[j].target_depth = self.depths[i].data_ptr()
                else:
                    arr[j].view = self._fit_view(i, device) if sized is None else tr.sized_view(self._fit_view(i, device))
                    arr[j].target_depth = None
                arr[j].target_rgb = self.targets[self._vi(i)].data_ptr()
                arr[j].target_mask = self.masks[self._vi(i)].data_ptr() if w_sil > 0.0 else None
            self._native_targets = cache = (key, arr)
        cfg = tr._native.GrFitConfig(NUM_STREAMS, PREP_AHEAD, PREP_GROUP, PREP_FIRST, REDUCE_BATCH, min(REDUCE_TAIL, REDUCE_BATCH))
        if sized is not None:  # device-side sizing: the capacities, the observed counts, the overflow word
            cfg.caps = sized.caps_arr
            cfg.observed = sized.observed.data_ptr()
            cfg.overflow = sized.ovf.data_ptr()
        if EXEC_STREAMS:
            # the Python schedule's own torch streams: the same hardware-queue placement (stream creation
            # order decides it), so the two schedules differ only in their host code
            side = getattr(self, "_side", None)
            if ns > 1 and (side is None or len(side) != ns - 1 or side[0].device != device):
                self._side = side = [torch.cuda.Stream(device) for _ in range(ns - 1)]
            prep = getattr(self, "_prep", None)
            if prep is None or prep.device != device:
                self._prep = prep = torch.cuda.Stream(device, priority=PREP_PRIORITY)
            self._exec_streams = rs = (ctypes.c_void_p * max(1, ns - 1))(
                *[st.cuda_stream for st in (side[:ns - 1] if ns > 1 else [])])
            cfg.render_streams = rs
            cfg.prep_stream = prep.cuda_stream
        losses_v = torch.empty(len(views), dtype=torch.float32, device=device)
        # the streams' accumulators (and their pointer array) are kept across steps while the shapes hold: the
        # executor writes them (accumulate = 0 first) only after the caller's stream, so after the previous step's
        # parameter update read them; 4 x streams allocations per step were host time before the first launch
        shapes = (ns,) + tuple(tuple(t.shape) for t in (m, s, c, o))
        cached = getattr(self, "_native_acc", None)
        if cached is None or cached[0] != shapes or cached[1][0][0].device != device:
            acc = [tuple(torch.empty_like(t) for t in (m, s, c, o)) for _ in range(ns)]
            self._native_acc = cached = (shapes, acc, (ctypes.c_void_p * (4 * ns))(*[t.data_ptr() for a in acc for t in a]))
        acc, ptrs = cached[1], cached[2]
        L = tr._native.lib()
        tr._native.check(L.gr_fit_views(tr._native.executor(device.index or 0), ctypes.byref(cfg), len(views), cache[1],
                                        int(m.shape[0]), tr._native.ptr(m), tr._native.ptr(s), tr._native.ptr(c),
                                        tr._color_dim(c), tr._native.ptr(o), ctypes.c_float(w_sil),
                                        ctypes.c_float(self.w_depth), ctypes.c_float(1.0 / len(self.targets)),
                                        tr._native.ptr(losses_v), ptrs, ctypes_stream(device)), "gr_fit_views")
        self._acc_parts = acc
        self._native_keep = (m, s, c, o)  # read by the executor's streams until the caller's stream passes them
        return losses_v.sum()

    def _views_direct(self, means, scales, colors, opacities, tail_fn=None, sized=None):
        """This rank's views without autograd: per view, gr_fwd_render_l1 (the HIP forward whose epilogue
        evaluates the view's L1 + silhouette loss and its upstream gradients, fit_multiview_stub.py:292-299)
        and gr_bwd_splat (the backward splat, :310); every REDUCE_BATCH views of a HIP stream,
        gr_reduce_views adds their gradient w.r.t. the
        activated parameters into that stream's accumulator set (in view order: deterministic).  The
        accumulators are summed in stream order and leave in self._acc for one autograd pass through the
        activations; returns (the sum of the view losses (device, 0-d), tail_fn() evaluated on the
        preparation stream after the last preparation, or None)."""
        device = means.device
        m, s, c, o = (t.detach().float().contiguous() for t in (means, scales, colors, opacities))
        views = self.my_views
        main = torch.cuda.current_stream(device)
        ns = max(1, min(NUM_STREAMS, len(views)))
        side = getattr(self, "_side", None)
        if ns > 1 and (side is None or len(side) != ns - 1 or side[0].device != device):
            self._side = side = [torch.cuda.Stream(device) for _ in range(ns - 1)]
        streams = [main] + (side[:ns - 1] if ns > 1 else [])
        # made on the main stream before the side streams wait for it: every stream's use is ordered
        # after its allocation, and main waits for every stream before they are read or freed
        losses_v = torch.empty(max(1, len(views)), dtype=torch.float32, device=device)
        # the streams' accumulators are kept across steps while the shapes hold (written only after the side
        # streams wait for main below, i.e. after the previous step's parameter update read them): 4 x streams
        # allocations per step were host time before the first preparation
        shapes = (len(streams),) + tuple(tuple(t.shape) for t in (m, s, c, o))
        cached = getattr(self, "_direct_acc", None)
        if cached is None or cached[0] != shapes or cached[1][0][0].device != device:
            self._direct_acc = cached = (shapes, [tuple(torch.empty_like(t) for t in (m, s, c, o)) for _ in streams])
        acc = cached[1]
        for st in streams[1:]:
            st.wait_stream(main)
        w_sil = self.w_sil if (self.masks is not None and self.w_sil > 0.0) else 0.0
        g_scale = 1.0 / len(self.targets)
        # the views' preparations (projection, culling, pair counts) run on a stream of their own,
        # PREP_AHEAD views ahead of the view being rendered: the host's read of a view's pair count never
        # waits behind other views' renders, the preparations run beside the splat kernels, and the host
        # starts the first render after enqueueing a few preparations (not all of them)
        prep = getattr(self, "_prep", None)
        if prep is None or prep.device != device:
            self._prep = prep = torch.cuda.Stream(device, priority=PREP_PRIORITY)
        prep.wait_stream(main)
        bin_stream = None
        if BIN_STREAM != "":
            bin_stream = getattr(self, "_bin", None)
            if bin_stream is None or bin_stream.device != device:
                self._bin = bin_stream = torch.cuda.Stream(device, priority=int(BIN_STREAM))
            bin_stream.wait_stream(main)
        pins = self._plan_pins(len(views))
        ahead: dict = {}
        if sized is None:
            prepare_upto = self._prep_groups(views, ahead, lambda js: tr.prepare_views_native(
                m, s, c, o, [self._fit_view(views[q], device) for q in js], [pins[q] for q in js]), prep)
        else:  # device-side sizing (_graph_step): capacities in, true counts to the pinned `observed` rows
            prepare_upto = self._prep_groups(views, ahead, lambda js: tr.prepare_views_sized(
                m, s, c, o, [tr.sized_view(self._fit_view(views[q], device)) for q in js], [sized.caps[q] for q in js],
                [sized.observed[q] for q in js], sized.ovf), prep)
        pending: list = [[] for _ in streams]  # per stream: (render state, partials) awaiting their reduction
        started = [False] * ns
        sizes = _batch_sizes(ns, len(views))

        def reduce_pending(k):
            if pending[k]:
                with torch.cuda.stream(streams[k]):
                    if GATHER:
                        tr.reduce_sums_native(m, s, c, o, pending[k], acc[k], accumulate=started[k])
                    else:
                        tr.reduce_views_native(m, s, c, o, pending[k], acc[k], accumulate=started[k])
                started[k] = True
                pending[k] = []

        for j, i in enumerate(views):
            k = j % ns
            prepare_upto(j)
            pv = ahead.pop(j)
            streams[k].wait_event(pv.event)
            pv.geom.record_stream(streams[k])
            with torch.cuda.stream(streams[k]):
                # one zone at the core cutoff and no depth channel: the loss reads neither depth nor the
                # tail-only part of W's footprint (torch_renderer.FIT_CUTOFF)
                rs, ws = tr.forward_l1_native(m, s, c, o, pv.gv, pv, self.targets[self._vi(i)],
                                              self.masks[self._vi(i)] if w_sil > 0.0 else None, w_sil, g_scale, losses_v[j:j + 1],
                                              bin_stream=bin_stream)
                pv = None
                tr.backward_splat_native(rs, ws)
                if GATHER:  # the view's sums; its bins, geom and workspace go back to the allocator here
                    pending[k].append((rs.gv, tr.gather_view_native(rs, ws)))
                    rs = ws = None
            if rs is not None:
                pending[k].append((rs, ws))
            prepare_upto(j + PREP_AHEAD)
            if len(pending[k]) >= sizes[k][0]:
                reduce_pending(k)
                if len(sizes[k]) > 1:
                    sizes[k].pop(0)
        for k in range(ns):
            reduce_pending(k)
        tail = None
        if tail_fn is not None:
            with torch.cuda.stream(prep):
                tail = tail_fn()
                if isinstance(tail, torch.Tensor):
                    tail.record_stream(main)  # allocated on the preparation stream, read on main
        for st in streams[1:]:
            main.wait_stream(st)
        main.wait_stream(prep)
        if bin_stream is not None:
            main.wait_stream(bin_stream)
        used = min(ns, len(views))
        # the streams' accumulators (summed in stream order by the caller: gr_fit_param_step or torch adds)
        self._acc_parts = acc[:used] if used > 0 else [tuple(torch.zeros_like(t) for t in (m, s, c, o))]
        return (losses_v[:len(views)].sum() if views else torch.zeros((), device=device)), tail

    def _views_direct_depth(self, means, scales, colors, opacities, sized=None) -> torch.Tensor:
        """The fused path with the depth term (fit_multiview_stub.py:301-305): per view the HIP forward in the
        default precision mode (depth output, f32-grade W and D, the depth-gradient footprint), then
        gr_bwd_fit (L1 + silhouette + depth loss gradients and the render backward) adding the gradient into
        the stream's accumulator set (in view order: deterministic).  Returns the sum of the view losses."""
        device = means.device
        m, s, c, o = (t.detach().float().contiguous() for t in (means, scales, colors, opacities))
        views = self.my_views
        main = torch.cuda.current_stream(device)
        ns = max(1, min(NUM_STREAMS, len(views)))
        side = getattr(self, "_side", None)
        if ns > 1 and (side is None or len(side) != ns - 1 or side[0].device != device):
            self._side = side = [torch.cuda.Stream(device) for _ in range(ns - 1)]
        streams = [main] + (side[:ns - 1] if ns > 1 else [])
        losses_v = torch.empty(max(1, len(views)), dtype=torch.float32, device=device)
        shapes = (len(streams),) + tuple(tuple(t.shape) for t in (m, s, c, o))  # kept across steps (_views_direct)
        cached = getattr(self, "_direct_acc", None)
        if cached is None or cached[0] != shapes or cached[1][0][0].device != device:
            self._direct_acc = cached = (shapes, [tuple(torch.empty_like(t) for t in (m, s, c, o)) for _ in streams])
        acc = cached[1]
        for st in streams[1:]:
            st.wait_stream(main)
        w_sil = self.w_sil if (self.masks is not None and self.w_sil > 0.0) else 0.0
        g_scale = 1.0 / len(self.targets)
        prep = getattr(self, "_prep", None)
        if prep is None or prep.device != device:
            self._prep = prep = torch.cuda.Stream(device, priority=PREP_PRIORITY)
        prep.wait_stream(main)
        pins = self._plan_pins(len(views))
        cache = getattr(self, "_gvd_cache", None)
        if cache is None:
            self._gvd_cache = cache = {}
        ahead: dict = {}

        def gv_of(i):
            if i not in cache:
                cam = self.cams[i]
                cache[i] = tr.make_view(cam.view, cam.proj, self.width, self.height, self._background(device),
                                        depth_grad=True)
            return cache[i]

        if sized is None:
            prepare_upto = self._prep_groups(views, ahead, lambda js: tr.prepare_views_native(
                m, s, c, o, [gv_of(views[q]) for q in js], [pins[q] for q in js]), prep)
        else:  # device-side sizing (_graph_step)
            prepare_upto = self._prep_groups(views, ahead, lambda js: tr.prepare_views_sized(
                m, s, c, o, [tr.sized_view(gv_of(views[q])) for q in js], [sized.caps[q] for q in js],
                [sized.observed[q] for q in js], sized.ovf), prep)
        # per view its render and the depth-loss backward up to the per-Gaussian sums (gr_bwd_fit_gather); per batch
        # of a stream's views one chain-rule pass (gr_reduce_sums with the depth sums), as _views_direct
        pending: list = [[] for _ in streams]
        started = [False] * ns
        sizes = _batch_sizes(ns, len(views))

        def reduce_pending(k):
            if pending[k]:
                with torch.cuda.stream(streams[k]):
                    tr.reduce_sums_native(m, s, c, o, pending[k], acc[k], accumulate=started[k])
                started[k] = True
                pending[k] = []

        for j, i in enumerate(views):
            k = j % ns
            prepare_upto(j)
            pv = ahead.pop(j)
            streams[k].wait_event(pv.event)
            pv.geom.record_stream(streams[k])
            with torch.cuda.stream(streams[k]):
                _, _, _, rs = tr.forward_native(m, s, c, o, pv.gv, pv, images=False)  # the backward reads the sums
                pv = None
                sums, sums3 = tr.backward_fit_gather_native(rs, self.targets[i], self.masks[i] if w_sil > 0.0 else None,
                                                            w_sil, self.depths[i], self.w_depth, g_scale,
                                                            losses_v[j:j + 1])
                pending[k].append((rs.gv, sums, sums3))
                rs = None
            prepare_upto(j + PREP_AHEAD)
            if len(pending[k]) >= sizes[k][0]:
                reduce_pending(k)
                if len(sizes[k]) > 1:
                    sizes[k].pop(0)
        for k in range(ns):
            reduce_pending(k)
        for st in streams[1:]:
            main.wait_stream(st)
        main.wait_stream(prep)
        used = min(ns, len(views))
        # the streams' accumulators (summed in stream order by the caller: gr_fit_param_step or torch adds)
        self._acc_parts = acc[:used] if used > 0 else [tuple(torch.zeros_like(t) for t in (m, s, c, o))]
        return losses_v[:len(views)].sum() if views else torch.zeros((), device=device)

    def _fused_step_ok(self) -> bool:
        """The fused parameter update applies: plain Adam (torch.optim.Adam defaults: no weight decay, no
        amsgrad, not maximize), one parameter group, the stub's parameter names, float32 contiguous tensors on
        the HIP device (gr_fit_param_step reads them through raw pointers)."""
        if not FUSED_STEP or type(self.opt) is not torch.optim.Adam or len(self.opt.param_groups) != 1:
            return False
        if not all(p.dtype == torch.float32 and p.is_cuda and p.is_contiguous() for p in self.params.values()):
            return False
        g = self.opt.param_groups[0]
        if g["weight_decay"] != 0 or g["amsgrad"] or g.get("maximize", False) or isinstance(g["lr"], torch.Tensor):
            return False
        return set(self.params) in ({"means", "scales_raw", "opacities_raw", "colors_raw"},
                                    {"means", "scales_raw", "opacities_raw", "sh_raw"})

    def _fused_param_step(self, scales, opacities, loss, sized=None) -> torch.Tensor:
        """fit_multiview_stub.py:307-311 after the views: d loss / d raw parameters through the activations
        (softplus + 1e-3, sigmoid, identity) and the regulariser (rank 0), then torch.optim.Adam's update with
        its own state tensors, one gr_fit_param_step pass per parameter (world size 1), or gradient assembly
        into the flat all-reduce buffer, the all-reduce, then gr_adam_step per parameter."""
        L = tr._native.lib()
        g = self.opt.param_groups[0]
        lr, (b1, b2), eps = float(g["lr"]), g["betas"], float(g["eps"])
        parts = self._acc_parts
        self._acc_parts = None
        slot = {"means": 0, "scales_raw": 1, "colors_raw": 2, "sh_raw": 2, "opacities_raw": 3}
        act = {"means": 0, "scales_raw": 1, "colors_raw": 2, "sh_raw": 0, "opacities_raw": 2}
        # mean()'s backward: the float32 weight divided by the float32 element count, as autograd computes it
        reg = {"scales_raw": float(np.float32(self.reg_scale) / np.float32(max(1, scales.numel()))),
               "opacities_raw": float(np.float32(self.reg_opacity) / np.float32(max(1, opacities.numel())))}
        names = list(self.params)
        plist = [self.params[k] for k in names]
        stream = ctypes_stream(plist[0].device)
        flat = None
        if self.world > 1:
            flat = torch.empty(sum(p.numel() for p in plist) + 1, dtype=torch.float32, device=plist[0].device)
        off = 0
        steps = []
        assembly = []
        for k, p in zip(names, plist):
            st = self.opt.state[p]
            if not st:  # torch.optim.Adam's lazy state, same tensors and layout
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if sized is None:  # (a captured step: the graph driver advances the host counts per replay)
                st["step"] += 1
            t = float(st["step"])
            neg_step = -(lr / (1.0 - b1 ** t))
            bc2s = (1.0 - b2 ** t) ** 0.5
            steps.append((neg_step, bc2s))
            a = [pp[slot[k]] for pp in parts]
            if len(a) > L_MAX_ACC:  # more streams than the kernel sums: fold the rest in stream order first
                t = a[L_MAX_ACC - 1]
                for x in a[L_MAX_ACC:]:
                    t = t + x
                a = a[:L_MAX_ACC - 1] + [t]
            accs = (ctypes.c_void_p * max(1, len(a)))(*[x.data_ptr() for x in a])
            if flat is not None:
                grad = flat[off:off + p.numel()].view_as(p)
                off += p.numel()
            else:
                # the gradient tensor is kept across steps (zero_grad(set_to_none) drops p.grad each step; the
                # kernel overwrites every element, in stream order after the previous step's readers)
                kept = self._grad_keep.get(k) if hasattr(self, "_grad_keep") else None
                if kept is None or kept.shape != p.shape or kept.device != p.device:
                    if not hasattr(self, "_grad_keep"):
                        self._grad_keep = {}
                    self._grad_keep[k] = kept = torch.empty_like(p)
                grad = kept
            # p.grad is this kept tensor, overwritten in place every step (an alias, not a fresh tensor): a caller that
            # keeps a reference to p.grad across steps (logging, clipping history, EMA) must copy it
            p.grad = grad
            r = reg.get(k, 0.0) if self.rank == 0 else 0.0

            def step_call(p=p, grad=grad, accs=accs, a=a, r=r, k=k, st=st, neg_step=neg_step, bc2s=bc2s):
                tr._native.check(L.gr_fit_param_step(p.numel(), act[k], tr._native.ptr(p.data), tr._native.ptr(grad),
                                                     accs, len(a), ctypes.c_float(r), 0 if flat is not None else 1,
                                                     tr._native.ptr(st["exp_avg"]), tr._native.ptr(st["exp_avg_sq"]),
                                                     ctypes.c_float(neg_step), ctypes.c_float(bc2s), ctypes.c_double(b1),
                                                     ctypes.c_double(b2), ctypes.c_float(eps), stream), "gr_fit_param_step")
            assembly.append(step_call)
        if flat is None:
            if len(plist) <= tr._native.FIT_MAX_PARAMS and all(len(pp) <= tr._native.FIT_MAX_ACC for pp in parts):
                # world size 1: every parameter's gradient and Adam update in one launch (gr_fit_param_steps)
                arr = (tr._native.GrParamStep * len(plist))()
                for q, (k, p) in enumerate(zip(names, plist)):
                    st, (neg_step, bc2s) = self.opt.state[p], steps[q]
                    a = [pp[slot[k]] for pp in parts]
                    e = arr[q]
                    e.count, e.act, e.num_accs = p.numel(), act[k], len(a)
                    e.param, e.grad = p.data.data_ptr(), p.grad.data_ptr()
                    for j, x in enumerate(a):
                        e.accs[j] = x.data_ptr()
                    e.exp_avg, e.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                    e.reg = reg.get(k, 0.0) if self.rank == 0 else 0.0
                    e.neg_step_size, e.bias_correction2_sqrt = neg_step, bc2s
                if sized is None:
                    tr._native.check(L.gr_fit_param_steps(len(plist), arr, ctypes.c_double(b1), ctypes.c_double(b2),
                                                          ctypes.c_float(eps), stream), "gr_fit_param_steps")
                else:  # the step's scalars from the device table, skipped on overflow (gr_fit_param_steps_sched)
                    tr._native.check(L.gr_fit_param_steps_sched(
                        len(plist), arr, ctypes.c_double(b1), ctypes.c_double(b2), ctypes.c_float(eps),
                        tr._native.ptr(sized.sched), tr._native.ptr(sized.step_dev), tr._native.ptr(sized.ovf),
                        ctypes.c_void_p(sized.flags.data_ptr()), stream), "gr_fit_param_steps_sched")
            elif sized is not None:
                raise RuntimeError("graph step: more parameters or stream accumulators than one gr_fit_param_steps launch")
            else:
                for call in assembly:
                    call()
            return loss.detach()
        bounds, o0 = [], 0
        for p in plist:
            bounds.append((o0, o0 + p.numel()))
            o0 += p.numel()
        bounds[-1] = (bounds[-1][0], off + 1)  # the loss rides in the last bucket

        def assemble(b):
            assembly[b]()
            if b == len(plist) - 1:
                flat[off:off + 1].copy_(loss.detach().reshape(1))

        def finish(b):
            p, (neg_step, bc2s) = plist[b], steps[b]
            st = self.opt.state[p]
            tr._native.check(L.gr_adam_step(p.numel(), tr._native.ptr(p.data), tr._native.ptr(p.grad),
                                            tr._native.ptr(st["exp_avg"]), tr._native.ptr(st["exp_avg_sq"]),
                                            ctypes.c_float(neg_step), ctypes.c_float(bc2s), ctypes.c_double(b1),
                                            ctypes.c_double(b2), ctypes.c_float(eps), stream), "gr_adam_step")

        bucketed_all_reduce([flat[a:b] for a, b in bounds], assemble, finish, self.group)
        return flat[off]

    def _finish_step(self, loss) -> torch.Tensor:
        plist = list(self.params.values())
        for p in plist:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        if self.world > 1:
            flat = torch.cat([p.grad.reshape(-1) for p in plist] + [loss.detach().reshape(1)])
            bounds, off = [], 0
            for p in plist:
                bounds.append((off, off + p.numel()))
                off += p.numel()
            bounds[-1] = (bounds[-1][0], off + 1)
            buckets = [flat[a:b] for a, b in bounds]

            def finish(b):
                p = plist[b]
                p.grad.copy_(buckets[b][:p.numel()].view_as(p))

            bucketed_all_reduce(buckets, lambda b: None, finish, self.group)
            loss_all = flat[off]
        else:
            loss_all = loss.detach()
        self.opt.step()
        return loss_all

    # ---- the fused step as one HIP graph (GR_GRAPH) -------------------------------------------------------------
    def _graph_ok(self, device) -> bool:
        """The graph applies: the fused path with its one-launch parameter update (world size 1), the Python
        schedule without a separate binning stream, and the optimizer state made by an eager step."""
        mode = self._graph_mode()
        if not (mode != "0" and self.world == 1 and device.type == "cuda" and BIN_STREAM == "" and self._direct(device)
                and self.params["means"].shape[0] > 0 and self._fused_step_ok()):
            return False
        if mode in ("batch", "batchgraph") and F32_GRADE:  # (the batched L1 path runs the two-piece mode only)
            return False
        if min(NUM_STREAMS, len(self.my_views)) > tr._native.FIT_MAX_ACC or len(self.params) > tr._native.FIT_MAX_PARAMS:
            return False
        return all(bool(self.opt.state.get(p)) for p in self.params.values())

    def _graph_mode(self) -> str:
        """The effective GR_GRAPH mode of this fit (auto: batch for small views, else 0)."""
        if GRAPH_MODE == "auto":
            return "batch" if self.width * self.height <= GRAPH_AUTO_PIXELS and len(self.my_views) >= 2 else "0"
        return GRAPH_MODE

    def _graph_key(self) -> tuple:
        g = self.opt.param_groups[0]
        plist = list(self.params.values())
        return (tuple((p.data_ptr(), tuple(p.shape)) for p in plist),
                tuple((self.opt.state[p]["exp_avg"].data_ptr(), self.opt.state[p]["exp_avg_sq"].data_ptr()) for p in plist),
                float(g["lr"]), tuple(g["betas"]), float(g["eps"]), tuple(self.my_views), self._depth_grad(),
                self.w_sil, self.w_depth, self.reg_opacity, self.reg_scale, F32_GRADE, FIT_TILE, NUM_STREAMS,
                tuple(t.data_ptr() for t in self.targets), tuple(m.data_ptr() for m in (self.masks or ())),
                tuple(d.data_ptr() for d in (self.depths or ())))

    def _probe_counts(self, device) -> list:
        """Every view of this rank prepared once with host-read plans: [(pairs, slots, core pairs)] per view."""
        with torch.no_grad():
            m, s, c, o = (t.detach().float().contiguous() for t in activations(self.params))
            views = self.my_views
            pins = torch.zeros((max(1, len(views)), 3), dtype=torch.int64, pin_memory=True)
            depth = self._depth_grad()
            for j0 in range(0, len(views), tr._native.PREPARE_MAX_VIEWS):
                js = range(j0, min(len(views), j0 + tr._native.PREPARE_MAX_VIEWS))
                gvs = [tr.make_view(self.cams[views[q]].view, self.cams[views[q]].proj, self.width, self.height,
                                    self._background(device), depth_grad=True) if depth else self._fit_view(views[q], device)
                       for q in js]
                tr.prepare_views_native(m, s, c, o, gvs, [pins[q] for q in js])
            torch.cuda.synchronize(device)
            return [tuple(int(x) for x in r) for r in pins[:len(views)].tolist()]

    @staticmethod
    def _caps_of(counts, old=None) -> list:
        def grow(x):
            return (int(x * GRAPH_MARGIN) + 4096 + 4095) // 4096 * 4096
        caps = []
        for j, (k, _, kc) in enumerate(counts):
            cc, ct = grow(kc), grow(k - kc)
            if old is not None:
                cc, ct = max(cc, int(old[j].num_core_pairs)), max(ct, int(old[j].num_pairs - old[j].num_core_pairs))
            caps.append(tr._native.GrPlan(cc + ct, cc + ct, cc))
        return caps

    def _graph_sched(self, device, t0: int):
        """(neg_step_size, bias_correction2_sqrt) of updates t0+1 .. t0+65536 onward from update 1, as the eager step
        computes them (same expressions, rounded to float32 as its ctypes arguments): index t = updates applied."""
        g = self.opt.param_groups[0]
        lr, (b1, b2) = float(g["lr"]), g["betas"]
        T = max(1 << 16, 2 * (t0 + 1))
        tab = np.empty((T, 2), dtype=np.float32)
        for t in range(T):
            u = float(t + 1)
            tab[t, 0] = -(lr / (1.0 - b1 ** u))
            tab[t, 1] = (1.0 - b2 ** u) ** 0.5
        return torch.from_numpy(tab.reshape(-1)).to(device), T

    def _act_ws_for(self, device) -> torch.Tensor:
        """activations_native's workspace, kept per fitter (made outside any capture: _graph_build asks first)."""
        ws = getattr(self, "_act_ws", None)
        if ws is None or ws.device != device:
            self._act_ws = ws = torch.zeros(int(tr._native.lib().gr_fit_activations_ws_bytes(0)), dtype=torch.uint8,
                                            device=device)
        return ws

    def _activations_fused(self, device):
        """The fused step's activations and (rank 0) regulariser in one launch (activations_native)."""
        ws = self._act_ws_for(device)
        if self.params["means"].shape[0] == 0:
            means, scales, colors, opacities = activations(self.params)
            return means, scales, colors, opacities, None
        return activations_native(self.params, (self.reg_opacity, self.reg_scale) if self.rank == 0 else None, ws)

    def _graph_body(self, gs):
        """The fused step (step()'s first branch, eager) on device-sized views, for capture."""
        with torch.no_grad():
            means, scales, colors, opacities, reg_t = self._activations_fused(self.params["means"].device)
            reg_fn = (lambda: reg_t) if reg_t is not None else None
            mode = self._graph_mode()
            if mode in ("batch", "batchgraph"):  # one launch per kernel for up to 8 views (gr_fit_views_batched), one stream
                reg = reg_fn() if reg_fn else None
                total = self._views_batched(means, scales, colors, opacities, gs)
            elif mode == "exec":  # the native executor with capacities (as step()'s executor branch)
                total = self._views_native(means, scales, colors, opacities, self._depth_grad(), sized=gs)
                rs = getattr(self, "_prep", None) if EXEC_STREAMS else None
                reg = None
                if reg_fn and rs is not None:
                    main = torch.cuda.current_stream(means.device)
                    with torch.cuda.stream(rs):
                        reg = reg_fn()
                    reg.record_stream(main)
                    main.wait_stream(rs)
                elif reg_fn:
                    reg = reg_fn()
            elif self._depth_grad():
                reg = reg_fn() if reg_fn else None
                total = self._views_direct_depth(means, scales, colors, opacities, sized=gs)
            else:
                total, reg = self._views_direct(means, scales, colors, opacities, reg_fn, sized=gs)
            loss = total / len(self.targets)
            if reg is not None:
                loss = loss + reg
        return self._fused_param_step(scales, opacities, loss, sized=gs)

    def _graph_build(self, device, counts=None, old_caps=None):
        """(Re)capture the step: capacities from `counts` (or a probe), the device step counter at the updates applied
        so far (the optimizer's step count), a fresh schedule table when it runs short."""
        gs = getattr(self, "_gs", None)
        if gs is None:
            gs = self._gs = _GraphState()
        gs.graph = None
        n_views = max(1, len(self.my_views))
        t0 = int(float(self.opt.state[next(iter(self.params.values()))]["step"]))
        if counts is None:
            counts = self._probe_counts(device)
        gs.caps = self._caps_of(counts, old_caps)
        gs.caps_arr = (tr._native.GrPlan * max(1, len(gs.caps)))(*gs.caps)
        gs.observed = torch.zeros((n_views, 3), dtype=torch.int64, pin_memory=True)
        gs.flags = torch.zeros(2, dtype=torch.int32, pin_memory=True)
        gs.ovf = torch.zeros(1, dtype=torch.int32, device=device)
        gs.step_dev = torch.tensor([t0], dtype=torch.int32, device=device)
        if gs.sched is None or gs.sched_len < t0 + 1024 or gs.sched_key != self._graph_key()[2:5]:
            gs.sched, gs.sched_len = self._graph_sched(device, t0)
            gs.sched_key = self._graph_key()[2:5]
        gs.done_host = t0
        self._act_ws_for(device)  # (made before any capture)
        torch.cuda.synchronize(device)
        if self._graph_mode() in ("1", "batchgraph"):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="relaxed"):
                gs.loss = self._graph_body(gs)
        else:  # (diagnostics: the device-sized step without the graph, enqueued by the host every step)
            g = _EagerReplay(lambda: self._graph_body(gs), gs)
        gs.graph = g
        gs.builds += 1
        gs.key = self._graph_key()
        gs.n = int(self.params["means"].shape[0])
        gs.inflight = []
        return gs

    def _graph_step(self, device) -> torch.Tensor:
        gs = getattr(self, "_gs", None)
        if gs is None or gs.graph is None or gs.key != self._graph_key():
            self.graph_sync()
            counts = None
            if gs is not None and gs.graph is not None and gs.n == int(self.params["means"].shape[0]):
                counts = [tuple(int(x) for x in r) for r in gs.observed[:len(self.my_views)].tolist()]
            gs = self._graph_build(device, counts)
        elif int(float(self.opt.state[next(iter(self.params.values()))]["step"])) + 2 >= gs.sched_len:
            self.graph_sync()
            gs = self._graph_build(device, [tuple(int(x) for x in r) for r in gs.observed[:len(self.my_views)].tolist()],
                                   gs.caps)
        gs.graph.replay()
        out = gs.loss.detach().clone()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        for p in self.params.values():  # torch.optim.Adam's host step count, as the eager step advances it
            self.opt.state[p]["step"] += 1
        gs.inflight.append((out, ev))
        if len(gs.inflight) > 2:
            gs.inflight.pop(0)
        if len(gs.inflight) == 2:  # the previous step (the GPU is busy with this one meanwhile)
            gs.inflight[0][1].synchronize()
            self._graph_check(device)
        return out

    def _graph_check(self, device) -> None:
        """A replayed step whose views exceeded their capacities updated nothing (and neither did any later one: the
        parameters did not change): grow the capacities from the true counts, recapture, and redo those steps, their
        losses written into the tensors step() returned for them."""
        gs = self._gs
        while int(gs.flags[0]) != 0:
            torch.cuda.synchronize(device)
            done = int(gs.flags[1])
            applied = int(float(self.opt.state[next(iter(self.params.values()))]["step"]))
            lost = applied - done
            redo = gs.inflight[len(gs.inflight) - lost:] if lost > 0 else []
            counts = [tuple(int(x) for x in r) for r in gs.observed[:len(self.my_views)].tolist()]
            for p in self.params.values():
                self.opt.state[p]["step"] -= lost
            gs.overflows += 1
            inflight = gs.inflight
            gs = self._graph_build(device, counts, gs.caps)
            for out, _ in redo:  # (an overflowing redo updates nothing, nor do the ones after it: counted next round)
                gs.graph.replay()
                out.copy_(gs.loss)
                for p in self.params.values():
                    self.opt.state[p]["step"] += 1
            torch.cuda.synchronize(device)
            gs.inflight = inflight

    def _views_batched(self, means, scales, colors, opacities, gs) -> torch.Tensor:
        """The step's views on the current stream, every kernel launched once per batch of up to 8 views
        (gr_fit_views_batched) on device-sized views: the preparations (gr_fwd_prepare_views_sized, 4 views each), the
        batched chain (binning, forward with the loss epilogue or the depth-loss forward, backward, gather), then the
        chain rules of up to 16 views per gr_reduce_sums into one accumulator set.  Per-view workspaces sized by the
        capacities are kept in the graph state across steps."""
        device = means.device
        L = tr._native.lib()
        nat = tr._native
        m, s, c, o = (t.detach().float().contiguous() for t in (means, scales, colors, opacities))
        n = int(m.shape[0])
        views = self.my_views
        depth = self._depth_grad()
        w_sil = self.w_sil if (self.masks is not None and self.w_sil > 0.0) else 0.0
        g_scale = 1.0 / len(self.targets)
        bkey = (n, depth, tuple((int(cp.num_pairs), int(cp.num_core_pairs)) for cp in gs.caps), str(device))
        bw = getattr(gs, "batch_ws", None)
        if bw is None or bw[0] != bkey:
            gvs = []
            for i in views:
                if depth:
                    cam = self.cams[i]
                    gvd = getattr(self, "_gvd_cache", None)
                    if gvd is None:
                        self._gvd_cache = gvd = {}
                    if i not in gvd:
                        gvd[i] = tr.make_view(cam.view, cam.proj, self.width, self.height, self._background(device),
                                              depth_grad=True)
                    gvs.append(tr.sized_view(gvd[i]))
                else:
                    gvs.append(tr.sized_view(self._fit_view(i, device)))
            u8 = dict(dtype=torch.uint8, device=device)
            gb = int(L.gr_geom_bytes(n))
            ws = []
            for j, gv in enumerate(gvs):
                cp = gs.caps[j]
                ws.append(dict(
                    geom=torch.empty((gb,), **u8),
                    bins=torch.empty((int(L.gr_bins_bytes(ctypes.byref(gv), n, ctypes.byref(cp))),), **u8),
                    scratch=torch.empty((int(L.gr_fwd_scratch_bytes(ctypes.byref(gv), n, ctypes.byref(cp))),), **u8),
                    ws=torch.empty((int(L.gr_bwd_bytes(ctypes.byref(gv), n, ctypes.byref(cp))),), **u8),
                    saved=(torch.empty((int(L.gr_saved_floats(ctypes.byref(gv))),), dtype=torch.float32, device=device)
                           if depth else None),
                    sums=torch.empty((n, 8), dtype=torch.float32, device=device),
                    sums3=torch.empty((n,), dtype=torch.float32, device=device) if depth else None))
            gs.batch_ws = bw = (bkey, gvs, ws)
        _, gvs, ws = bw
        losses_v = torch.empty(max(1, len(views)), dtype=torch.float32, device=device)
        # the chain rules in one accumulator set, batches of up to REDUCE_BATCH views (every view is gathered before
        # the first chain rule, so no short tail batch): the same sums in the same order as _views_direct /
        # _views_direct_depth with GR_STREAMS=1 and GR_REDUCE_TAIL=0, so the same parameters bit for bit (one chain-rule
        # launch for up to 16 views, one accumulator for the update to read instead of one per stream)
        ns = 1
        shapes = (ns,) + tuple(tuple(t.shape) for t in (m, s, c, o))
        cached = getattr(self, "_direct_acc", None)
        if cached is None or cached[0] != shapes or cached[1][0][0].device != device:
            self._direct_acc = cached = (shapes, [tuple(torch.empty_like(t) for t in (m, s, c, o)) for _ in range(ns)])
        acc = cached[1]
        stream = ctypes_stream(device)
        cd = tr._color_dim(c)
        for j0 in range(0, len(views), nat.PREPARE_MAX_VIEWS):
            js = range(j0, min(len(views), j0 + nat.PREPARE_MAX_VIEWS))
            k = len(js)
            nat.check(L.gr_fwd_prepare_views_sized(
                k, (nat.GrView * k)(*[gvs[q] for q in js]), n, nat.ptr(m), nat.ptr(s), nat.ptr(c), cd, nat.ptr(o),
                (ctypes.c_void_p * k)(*[ws[q]["geom"].data_ptr() for q in js]), ws[js[0]]["geom"].numel(),
                (nat.GrPlan * k)(*[gs.caps[q] for q in js]),
                (ctypes.c_void_p * k)(*[gs.observed[q].data_ptr() for q in js]), nat.ptr(gs.ovf), stream),
                "gr_fwd_prepare_views_sized")
        for j0 in range(0, len(views), nat.BATCH_MAX_VIEWS):
            js = range(j0, min(len(views), j0 + nat.BATCH_MAX_VIEWS))
            arr = (nat.GrBatchView * len(js))()
            for e, q in zip(arr, js):
                w, i = ws[q], views[q]
                e.view, e.plan = gvs[q], gs.caps[q]
                e.geom, e.bins, e.bins_bytes = w["geom"].data_ptr(), w["bins"].data_ptr(), w["bins"].numel()
                e.scratch, e.scratch_bytes = w["scratch"].data_ptr(), w["scratch"].numel()
                e.ws, e.ws_bytes = w["ws"].data_ptr(), w["ws"].numel()
                e.saved = w["saved"].data_ptr() if depth else None
                e.target_rgb = self.targets[self._vi(i)].data_ptr()
                e.target_mask = self.masks[self._vi(i)].data_ptr() if w_sil > 0.0 else None
                e.target_depth = self.depths[i].data_ptr() if depth else None
                e.sums, e.sums3 = w["sums"].data_ptr(), (w["sums3"].data_ptr() if depth else None)
                e.loss = losses_v[q:q + 1].data_ptr()
            nat.check(L.gr_fit_views_batched(len(js), arr, n, ctypes.c_float(w_sil), ctypes.c_float(self.w_depth if depth else 0.0),
                                             ctypes.c_float(g_scale), stream), "gr_fit_views_batched")
        for k, sizes in enumerate(_batch_sizes(ns, len(views), tail=0)):
            mine = list(range(k, len(views), ns))
            at = 0
            for b in sizes:
                js = mine[at:at + b]
                if js:
                    tr.reduce_sums_native(m, s, c, o,
                                          [(gvs[q], ws[q]["sums"]) + ((ws[q]["sums3"],) if depth else ()) for q in js],
                                          acc[k], accumulate=at > 0)
                at += b
        self._acc_parts = acc[:min(ns, len(views))] if views else [tuple(torch.zeros_like(t) for t in (m, s, c, o))]
        self._native_keep = (m, s, c, o)
        return losses_v[:len(views)].sum() if views else torch.zeros((), device=device)

    def _graph_leave(self) -> None:
        """The step goes eager while replayed steps may still be in flight (the graph's conditions changed, e.g.
        F32_GRADE toggled): settle them first (an overflowed one is redone and its loss rewritten, and the host's Adam
        step count corrected), then drop the graph, so that a later capture counts only its own replays."""
        gs = getattr(self, "_gs", None)
        if gs is None or gs.graph is None:
            return
        self.graph_sync()
        gs.graph = None
        gs.key = None
        gs.inflight = []

    def graph_sync(self) -> None:
        """Wait for the replayed steps and redo any that overflowed (densify, the parameters' readers and the end of a
        fit call this; a no-op without a graph)."""
        gs = getattr(self, "_gs", None)
        if gs is None or gs.graph is None:
            return
        torch.cuda.synchronize(self.params["means"].device)
        self._graph_check(self.params["means"].device)

    def densify_and_prune(self, max_gaussians: int, densify_ratio: float, prune_opacity: float,
                          on_device: Optional[bool] = None) -> None:
        """on_device (default: N >= DEVICE_DENSIFY_MIN): the device-side rule with a device generator
        (densify_and_prune_device); otherwise the host rule with the stub's CPU random stream."""
        self.graph_sync()
        n_now = int(self.params["means"].shape[0])
        if on_device is None:
            on_device = self.params["means"].device.type == "cuda" and n_now >= DEVICE_DENSIFY_MIN
        if on_device and getattr(self, "_dgen", None) is None:
            self._dgen = torch.Generator(device=self.params["means"].device).manual_seed(self.densify_seed)

        def decide():
            base = self.canonical_params()
            if on_device:
                newp = densify_and_prune_device(base, max_gaussians, densify_ratio, prune_opacity, self._dgen)
            else:
                newp = densify_and_prune(base, max_gaussians, densify_ratio, prune_opacity)
            perm = None
            if self.reorder and newp["means"].shape[0] >= 2:
                perm = morton_order(newp["means"])
                newp = {k: torch.nn.Parameter(v.detach()[perm].contiguous()) for k, v in newp.items()}
            return newp, perm

        if self.world > 1:
            # rank 0 decides, everyone receives the new tensors
            dev = self.params["means"].device
            if self.rank == 0:
                newp, perm = decide()
                n = torch.tensor([newp["means"].shape[0], int(perm is not None)], device=dev)
            else:
                n = torch.zeros(2, dtype=torch.int64, device=dev)
            dist.broadcast(n, 0, group=self.group)
            n_new, has_perm = int(n[0].item()), bool(n[1].item())
            if self.rank != 0:
                newp = {k: torch.nn.Parameter(torch.empty((n_new,) + tuple(v.shape[1:]), device=v.device))
                        for k, v in self.params.items()}
                perm = torch.empty(n_new, dtype=torch.int64, device=dev) if has_perm else None
            for k in sorted(newp):
                dist.broadcast(newp[k].data, 0, group=self.group)
            if has_perm:
                dist.broadcast(perm, 0, group=self.group)
            self.params, self.perm = newp, perm
        else:
            self.params, self.perm = decide()
        self.reset_optimizer()


# ------------------------------------------------------------------------------------------------
# CLI: same flags as fit_multiview_stub.py:200-229.
# ------------------------------------------------------------------------------------------------
def _load_image(path: Path, width: int, height: int, gray: bool = False) -> np.ndarray:
    from PIL import Image

    img = Image.open(path).convert("L" if gray else "RGB").resize((width, height), Image.Resampling.BILINEAR)
    return np.asarray(img, dtype=np.float32) / 255.0


def orbit_cameras(num_views: int, width: int, height: int, device) -> list:
    """fit_multiview_stub.py:70-90."""
    proj = tr.perspective(60.0, width / height, 0.01, 100.0, device=device)
    target = torch.tensor([0.0, 0.0, 0.0], dtype=torch.float32, device=device)
    up = torch.tensor([0.0, 1.0, 0.0], dtype=torch.float32, device=device)
    cams = []
    for i in range(num_views):
        yaw = (2.0 * math.pi * i) / max(1, num_views)
        eye = torch.tensor([2.5 * math.cos(0.2) * math.sin(yaw), 2.5 * math.sin(0.2), 2.5 * math.cos(0.2) * math.cos(yaw)],
                           dtype=torch.float32, device=device)
        cams.append(tr.Camera(view=tr.look_at(eye, target, up), proj=proj))
    return cams


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--targets_dir", required=True)
    ap.add_argument("--out_dir", default="outputs/fit_multiview_stub")
    ap.add_argument("--camera_npz", default="")
    ap.add_argument("--masks_dir", default="")
    ap.add_argument("--depth_dir", default="")
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--lr", type=float, default=0.02)
    ap.add_argument("--width", type=int, default=128)
    ap.add_argument("--height", type=int, default=128)
    ap.add_argument("--num_gaussians", type=int, default=800)
    ap.add_argument("--max_gaussians", type=int, default=3000)
    ap.add_argument("--use_sh", action="store_true")
    ap.add_argument("--sh_degree", type=int, default=1, choices=(1, 3), help="with --use_sh: 1 (reference) or 3 (extension)")
    ap.add_argument("--densify_interval", type=int, default=80)
    ap.add_argument("--prune_interval", type=int, default=80)
    ap.add_argument("--densify_ratio", type=float, default=0.15)
    ap.add_argument("--prune_opacity", type=float, default=0.05)
    ap.add_argument("--silhouette_weight", type=float, default=0.2)
    ap.add_argument("--mask_thresh", type=float, default=0.06)
    ap.add_argument("--depth_weight", type=float, default=0.05)
    ap.add_argument("--reg_opacity", type=float, default=0.001)
    ap.add_argument("--reg_scale", type=float, default=0.001)
    ap.add_argument("--seed", type=int, default=None, help="torch.manual_seed before initialisation")
    ap.add_argument("--device", default="", help="cpu: host tensors (cpu_renderer, gloo); default: the HIP device")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    on_host = args.device == "cpu" or not torch.cuda.is_available()
    if world > 1:
        if not on_host:
            torch.cuda.set_device(local_rank)
        dist.init_process_group("gloo" if on_host else "nccl")
    rank = dist.get_rank() if world > 1 else 0
    device = torch.device("cpu") if on_host else torch.device("cuda", local_rank)
    if args.seed is not None:
        torch.manual_seed(args.seed)
    if rank == 0:
        print(f"Using device: {device} (ranks: {world})")

    tdir = Path(args.targets_dir)
    paths = sorted([*tdir.glob("*.png"), *tdir.glob("*.jpg"), *tdir.glob("*.jpeg")])
    if not paths:
        raise FileNotFoundError(f"No target images found in {tdir} (supported: png/jpg/jpeg)")
    targets = [torch.from_numpy(_load_image(p, args.width, args.height)).to(device) for p in paths]
    masks = None
    if args.masks_dir:
        cand = [Path(args.masks_dir) / f"{p.stem}.png" for p in paths]
        if all(c.exists() for c in cand):
            masks = [torch.from_numpy(_load_image(c, args.width, args.height, gray=True)).to(device) for c in cand]
    if masks is None and args.silhouette_weight > 0.0:
        masks = [(t.mean(dim=2) > args.mask_thresh).to(torch.float32) for t in targets]
    depths = None
    if args.depth_dir:
        cand = [Path(args.depth_dir) / f"{p.stem}.png" for p in paths]
        if all(c.exists() for c in cand):
            depths = [torch.from_numpy(_load_image(c, args.width, args.height, gray=True)).to(device) for c in cand]
    if args.camera_npz:
        data = np.load(args.camera_npz)
        if "view" not in data or "proj" not in data:
            raise KeyError("camera npz must contain arrays: view (V,4,4), proj (V,4,4)")
        views, projs = np.asarray(data["view"], np.float32), np.asarray(data["proj"], np.float32)
        if views.shape[0] != len(targets) or projs.shape[0] != len(targets):
            raise ValueError("camera count mismatch with number of target images")
        cams = [tr.Camera(view=torch.from_numpy(views[i]).to(device), proj=torch.from_numpy(projs[i]).to(device))
                for i in range(len(targets))]
    else:
        cams = orbit_cameras(len(targets), args.width, args.height, device)

    params = build_params(args.num_gaussians, device, args.use_sh, args.sh_degree)
    fitter = ViewShardedFitter(params, cams, targets, args.width, args.height, lr=args.lr, masks=masks, depths=depths,
                               silhouette_weight=args.silhouette_weight, depth_weight=args.depth_weight,
                               reg_opacity=args.reg_opacity, reg_scale=args.reg_scale)
    loss_log = []
    pending = []  # the step tensors not yet read: a replayed step found to have overflowed is redone and its loss
    #               rewritten in place one step later (graph_sync), so the host reads them after that
    for it in range(args.iters):
        pending.append(fitter.step())
        if rank == 0 and (it == 0 or (it + 1) % 25 == 0):
            fitter.graph_sync()
            print(f"iter {it+1:4d}  loss={float(pending[-1]):.6f}  N={fitter.params['means'].shape[0]}")
        if (it + 1) % args.prune_interval == 0 or (it + 1) % args.densify_interval == 0 or it + 1 == args.iters:
            fitter.graph_sync()
            loss_log.extend(float(t) for t in pending)
            pending = []
        if (it + 1) % args.prune_interval == 0 or (it + 1) % args.densify_interval == 0:
            fitter.densify_and_prune(args.max_gaussians,
                                     args.densify_ratio if (it + 1) % args.densify_interval == 0 else 0.0,
                                     args.prune_opacity)
    if rank == 0:
        save_outputs(fitter, cams, args, Path(args.out_dir), loss_log)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def save_outputs(fitter: ViewShardedFitter, cams, args, out_dir: Path, loss_log) -> None:
    """gaussians_fitted.npz / loss.txt / preview_view0.png exactly as fit_multiview_stub.py:327-380."""
    from PIL import Image

    out_dir.mkdir(parents=True, exist_ok=True)
    p = fitter.canonical_params()
    means = p["means"]
    scales = torch.nn.functional.softplus(p["scales_raw"]) + 1e-3
    opacities = torch.sigmoid(p["opacities_raw"])
    sh = p.get("sh_raw")
    colors = sh[:, 0, :].clamp(0.0, 1.0) if sh is not None else torch.sigmoid(p["colors_raw"])
    arrays = dict(means=means, scales=scales, colors=colors, opacities=opacities)
    if sh is not None:
        arrays["sh_coeffs"] = sh
    np.savez(out_dir / "gaussians_fitted.npz", **{k: v.detach().cpu().numpy().astype(np.float32) for k, v in arrays.items()})
    (out_dir / "loss.txt").write_text("\n".join(f"{v:.8f}" for v in loss_log), encoding="utf-8")
    with torch.no_grad():
        pred0 = tr.render_gaussians_torch(means, scales, sh if sh is not None else colors, opacities, cams[0],
                                          width=args.width, height=args.height,
                                          background=torch.tensor([0.0, 0.0, 0.0], device=means.device),
                                          max_gaussians=max(args.max_gaussians, means.shape[0]), return_aux=False)
        Image.fromarray((pred0.clamp(0, 1).cpu().numpy() * 255.0).astype(np.uint8), mode="RGB").save(out_dir / "preview_view0.png")
    print(f"Done. Outputs written to: {out_dir}")


if __name__ == "__main__":
    main()
