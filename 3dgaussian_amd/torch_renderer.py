"""Drop-in replacement for the reference's python/torch_renderer.py, backed by gfx950 HIP kernels.

Same module surface as the reference (torch_renderer.py:10-121): ``Camera``, ``get_default_device``,
``perspective``, ``look_at``, ``render_gaussians_torch``; same argument meaning, return values and
exceptions.  The math is the reference's order-independent weighted average
(torch_renderer.py:164-203), evaluated by the tile-binned forward and hand-written backward kernels of
libgr_hip.so through a ``torch.autograd.Function`` — not by torch ops.  Differences that are by design
(DESIGN.md §Semantics):

* a Gaussian is evaluated on the 16x16 tiles where its largest weight is >= o*exp(-cutoff^2/2)
  (cutoff 8 when the depth output may be differentiated, 7 with ``depth_grad=False``;
  ``default_cutoff``); tiles where it stays below o*exp(-core_cutoff^2/2) (default 5.5) are "tail"
  tiles that carry only the weight and depth sums forward and the depth-coupled gradient terms
  backward (only when an upstream depth gradient is given): outputs and gradients agree with the
  dense reference to <=5e-6 relative L2 on its own fixtures, with and without depth gradients, and to
  <=1e-4 on sampled dense checks at configs C4 and C5 (tests/test_scale_gpu.py);
* ``chunk_size`` is accepted and ignored (no chunk loop);
* gradients flow to means, scales, colours/SH, opacities, background and - when their tensors require
  grad, as the reference's autograd gives them (:57-83, 140-150) - to camera.view / camera.proj
  (gr_bwd_camera);
* the op dispatches on the tensors' device like the reference: HIP tensors always run the HIP kernels
  (a missing libgr_hip.so raises ImportError; nothing falls back), CPU tensors run ``cpu_renderer``'s
  dense torch op (config C1, the reference's own CPU plumbing case; no tile cutoff there).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading
import weakref
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

try:  # package import (3dgaussian_amd.torch_renderer) or flat import (drop-in on sys.path)
    from . import _native, cpu_renderer, spatial
except ImportError:  # pragma: no cover
    import _native  # type: ignore
    import cpu_renderer  # type: ignore
    import spatial  # type: ignore

DEFAULT_CUTOFF = 7.0  # tail zone (W and D) when no depth gradient will follow (depth_grad=False)
DEPTH_GRAD_CUTOFF = 8.0  # tail zone when the depth output may be differentiated (the default mode)
DEFAULT_CORE_CUTOFF = 5.5
# Views of the fused fit path (no depth output, no depth gradient: fit_multiview._views_direct) are
# binned with one zone at 5 sigma (SURVEY.md 8(d)'s footprint; elliptical tile culling): no tail zone
# (it only carries W and D), and the dropped weight (<= o e^-12.5 per Gaussian and tile) keeps the
# outputs and gradients within 5e-5 relL2 of the dense reference at configs C4 and C5, also on the
# bench's fit state after several Adam steps (tests/test_scale_gpu.py; 5.5 sigma: 2.5e-5, 10% slower)
FIT_CUTOFF = float(os.environ.get("GR_FIT_CUTOFF", "5.0"))


# depth_grad=True (the default, "a depth gradient may follow") renders lazily: the forward runs in the
# two-piece mode with the no-depth-gradient footprint (what a caller whose loss never differentiates the
# depth output - the reference fit loop without --depth_dir - needs), and a backward that does receive a
# depth gradient re-renders the view at f32 grade with the depth-gradient footprint first (gr_bwd then
# differentiates that render; its outputs equal the returned ones within the parity bar).  A caller that
# knows it will differentiate the depth passes depth_grad="eager" (one f32-grade render).  GR_LAZY_DEPTH=0
# makes True eager.
LAZY_DEPTH = os.environ.get("GR_LAZY_DEPTH", "1") != "0"
# Adaptive laziness: a caller whose loss does differentiate the depth (the reference loop with --depth_dir) would
# pay for every view twice (the lazy render, then the f32-grade re-render in its backward).  After LAZY_ADAPT
# such re-renders in a row, depth_grad=True renders at f32 grade up front (as "eager"); the first backward of such
# a render that receives no depth gradient switches back to lazy.  Results are the eager mode's (within the parity
# bar of the lazy ones).  GR_LAZY_ADAPT=0 never adapts.
LAZY_ADAPT = max(0, int(os.environ.get("GR_LAZY_ADAPT", "2")))
# What the op adapts to is kept per CALLER, keyed by the caller's means tensor (a fit's parameter: the same object
# across its iterations; the reference loop passes params["means"] itself, fit_multiview_stub.py:268): the adaptive
# laziness above and the Morton layout's permutation (below).  Two fits interleaved on one process (one with a depth
# loss, one without) therefore never change each other's renders: each gets exactly what it gets alone.  Within one
# caller the rounding of depth_grad=True renders does depend on its own history (lazy for its first LAZY_ADAPT
# iterations, f32 grade after), within the parity bar either way; GR_LAZY_ADAPT=0 makes it history-free.
# Every piece of module state (callers, the speculation pipelines per device) is guarded by one lock.
_LOCK = threading.RLock()


class _Caller:
    __slots__ = ("rerenders", "eager", "layout", "perm")

    def __init__(self):
        self.rerenders, self.eager, self.layout, self.perm = 0, False, None, None


_CALLERS: dict = {}  # id(means) -> (weakref(means), _Caller)


def _caller_of(means: torch.Tensor) -> _Caller:
    with _LOCK:
        e = _CALLERS.get(id(means))
        if e is not None and e[0]() is means:
            return e[1]
        if len(_CALLERS) >= 256:  # forget callers whose tensors are gone
            for k in [k for k, (r, _) in _CALLERS.items() if r() is None]:
                del _CALLERS[k]
        c = _Caller()
        _CALLERS[id(means)] = (weakref.ref(means), c)
        return c


def lazy_eager(means: torch.Tensor) -> bool:
    """Whether adaptive laziness renders this caller's depth_grad=True views at f32 grade up front."""
    with _LOCK:
        e = _CALLERS.get(id(means))
        return bool(e is not None and e[0]() is means and e[1].eager)


def reset_lazy_depth() -> None:
    """Forget what adaptive laziness learned, for every caller (a new loop / loss)."""
    with _LOCK:
        for _, c in _CALLERS.values():
            c.rerenders, c.eager = 0, False


def default_cutoff(depth_grad: bool = True) -> float:
    """Tail cutoff (in sigma) of a view rendered with/without a depth gradient to follow.  With one, the
    depth-coupled gradient d depth / d w = (z - depth) / (W + 1e-6) amplifies far tails by up to 1e6 on
    near-empty pixels: at config C5 (1080p, empty image sides) 7 sigma leaves the dense reference's
    position/scale gradients 4e-5..4e-4 relL2 away, 8 sigma 2.5e-6 (tests/test_scale_gpu.py,
    tools/probe_cutoff.py).  Without one the tail only feeds the alpha/depth outputs: 7 sigma."""
    return DEPTH_GRAD_CUTOFF if depth_grad else DEFAULT_CUTOFF


def _eager(depth_grad) -> bool:
    """depth_grad (True / False / "eager") -> whether the forward renders at f32 grade up front."""
    if isinstance(depth_grad, str):
        if depth_grad != "eager":
            raise ValueError('depth_grad must be True, False or "eager"')
        return True
    return bool(depth_grad) and not LAZY_DEPTH


@dataclass
class Camera:
    """A camera view; same fields as the reference (torch_renderer.py:10-13)."""

    view: torch.Tensor  # (4,4) float32, row-major world->camera
    proj: torch.Tensor  # (4,4) float32, row-major camera->clip


def get_default_device() -> torch.device:
    """HIP device when one is visible (the reference returns cpu on Linux, torch_renderer.py:16-21)."""
    if torch.cuda.is_available():
        return torch.device("cuda")
    if getattr(torch.backends, "mps", None) is not None and torch.backends.mps.is_available():
        return torch.device("mps")
    return torch.device("cpu")


def perspective(fovy_deg: float, aspect: float, znear: float, zfar: float, device=None) -> torch.Tensor:
    """OpenGL-style projection matrix (torch_renderer.py:24-32), float32."""
    half = torch.tensor(fovy_deg, dtype=torch.float32) * (torch.pi / 180.0) * 0.5
    f = 1.0 / torch.tan(half)
    m = torch.zeros((4, 4), dtype=torch.float32)
    m[0, 0] = f / aspect
    m[1, 1] = f
    m[2, 2] = (zfar + znear) / (znear - zfar)
    m[2, 3] = (2.0 * zfar * znear) / (znear - zfar)
    m[3, 2] = -1.0
    return m.to(device) if device is not None else m


def look_at(eye: torch.Tensor, target: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """Right-handed look-at view matrix (torch_renderer.py:35-54), float32, on eye's device."""
    e = eye.to(dtype=torch.float32)
    fwd = target.to(dtype=torch.float32, device=e.device) - e
    fwd = fwd / (torch.linalg.norm(fwd) + 1e-8)
    upn = up.to(dtype=torch.float32, device=e.device)
    upn = upn / (torch.linalg.norm(upn) + 1e-8)
    side = torch.linalg.cross(fwd, upn)
    side = side / (torch.linalg.norm(side) + 1e-8)
    true_up = torch.linalg.cross(side, fwd)
    rot = torch.eye(4, dtype=torch.float32, device=e.device)
    rot[0, :3] = side
    rot[1, :3] = true_up
    rot[2, :3] = -fwd
    trans = torch.eye(4, dtype=torch.float32, device=e.device)
    trans[:3, 3] = -e
    return rot @ trans


# ------------------------------------------------------------------------------------------------
# Camera -> gr_view (host copy of the 4x4 matrices; cached per tensor version to avoid a D2H copy
# per render call in the fit loop).
# ------------------------------------------------------------------------------------------------
_MAT_CACHE: dict = {}


def _host_copy(t: torch.Tensor, shape) -> np.ndarray:
    """Host copy of a small (camera / background) tensor, cached per tensor and version: reading a
    device tensor waits for the whole stream, so a view built from the same tensors twice must not
    read them twice."""
    key = (id(t), t.data_ptr(), t._version, str(t.device))
    hit = _MAT_CACHE.get(key)
    if hit is not None and hit[0]() is t:
        return hit[1]
    m = t.detach().to(device="cpu", dtype=torch.float32).reshape(shape).numpy().copy()
    if len(_MAT_CACHE) > 4096:
        _MAT_CACHE.clear()
    # a weak reference: the cache never keeps a caller's tensor alive (a dead entry can only miss)
    _MAT_CACHE[key] = (weakref.ref(t), m)
    return m


_ZERO_BG: dict = {}


def _default_background(device: torch.device) -> torch.Tensor:
    """The background=None value (zeros), one persistent tensor per device: its host copy is cached,
    so a caller that passes no background costs no device-to-host read per view."""
    t = _ZERO_BG.get(str(device))
    if t is None:
        t = _ZERO_BG[str(device)] = torch.zeros(3, dtype=torch.float32, device=device)
    return t


def _host_matrix(t: torch.Tensor) -> np.ndarray:
    return _host_copy(t, (4, 4))


def make_view(view, proj, width: int, height: int, background=None, cutoff: Optional[float] = None,
              core_cutoff: float = DEFAULT_CORE_CUTOFF, depth_grad: bool = True, tile: int = 0) -> _native.GrView:
    """Build a gr_view from host (numpy / tensor) matrices.  ``depth_grad=False`` promises that the
    depth output will get no gradient (gr_view.no_depth_grad): W and D are then accumulated within
    2^-16 relative instead of f32-grade, and a depth gradient raises in the backward.
    ``cutoff=None``: ``default_cutoff(depth_grad)``.  ``tile``: gr_view.tile (0/16, or 32 on the fused fit path)."""
    if cutoff is None:
        cutoff = default_cutoff(depth_grad)
    V = view if isinstance(view, np.ndarray) else _host_matrix(view)
    P = proj if isinstance(proj, np.ndarray) else _host_matrix(proj)
    V = np.asarray(V, dtype=np.float32).reshape(4, 4)
    P = np.asarray(P, dtype=np.float32).reshape(4, 4)
    gv = _native.GrView()
    gv.width, gv.height = int(width), int(height)
    gv.view[:] = V.reshape(16).tolist()
    gv.proj[:] = P.reshape(16).tolist()
    gv.background_dev = None
    if background is None:
        bg = [0.0, 0.0, 0.0]
    elif isinstance(background, torch.Tensor) and background.device.type == "cuda":
        # read by the kernels on the device (gr_view.background_dev), stream-ordered: no device-to-host
        # copy per view.  The caller keeps the tensor alive until the view's kernels have run (rasterize
        # saves it for the backward); it must be 3 contiguous float32 values.
        if background.dtype != torch.float32 or background.numel() != 3 or not background.is_contiguous():
            raise ValueError("a device background must be 3 contiguous float32 values")
        gv.background_dev = background.data_ptr()
        bg = [0.0, 0.0, 0.0]
    elif isinstance(background, torch.Tensor):
        bg = background.detach().to(torch.float32).reshape(3).tolist()
    else:
        bg = np.asarray(background, np.float32).reshape(3).tolist()
    gv.background[:] = bg
    # camera centre = inv(view)[:3,3] (torch_renderer.py:81-83); float64 inverse, rounded once.
    cam = np.linalg.inv(V.astype(np.float64))[:3, 3]
    gv.cam_pos[:] = cam.astype(np.float32).tolist()
    gv.cutoff = float(cutoff)
    gv.core_cutoff = float(core_cutoff)
    gv.no_depth_grad = 0 if depth_grad else 1
    gv.tile = int(tile)
    return gv


def _color_dim(colors: torch.Tensor) -> int:
    """gr_hip.h color_dim: 3 (RGB), 12 (the reference's degree-1 basis, (N,4,3)) or 48 (the degree-3
    extension, (N,16,3): unnormalised real spherical-harmonic polynomials continuing the reference's
    degree-1 terms)."""
    return 3 if colors.dim() == 2 else 3 * int(colors.shape[1])


def _ws_round(nbytes) -> int:
    """Workspace sizes that follow the pair count (bins, scratch, backward partials) rounded up to coarse
    classes (1/32 to 1/16 of the size, at least 2 MiB): as a fit moves its Gaussians the pair counts
    drift by fractions of a percent per step, and exact sizes would make the caching allocator reserve a
    new block almost every step (its reserve grew ~0.7 GiB per step at C4) instead of reusing one."""
    nbytes = int(nbytes)
    q = max(1 << 21, 1 << max(0, nbytes.bit_length() - 5))
    return (nbytes + q - 1) // q * q


def _stream(device: torch.device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class RenderState:
    """Device workspaces produced by the forward pass and consumed by the backward pass."""

    __slots__ = ("gv", "n", "plan", "geom", "bins", "saved")

    def __init__(self, gv, n, plan, geom, bins, saved):
        self.gv, self.n, self.plan, self.geom, self.bins, self.saved = gv, n, plan, geom, bins, saved

    @property
    def num_pairs(self) -> int:
        return int(self.plan.num_pairs)


class Prepared:
    """A view whose projection, culling and pair counting (gr_fwd_prepare_async) are enqueued.

    The plan (pair / slot counts) arrives in pinned host memory; ``plan()`` waits for it.  Preparing
    the next view before rendering the current one keeps the device busy while the host reads the
    plan (ViewShardedFitter does this)."""

    __slots__ = ("gv", "n", "geom", "plan_host", "event", "binned", "rendered", "caps")

    def __init__(self, gv, n, geom, plan_host, event, caps=None):
        self.gv, self.n, self.geom, self.plan_host, self.event = gv, n, geom, plan_host, event
        self.binned = None  # (bins, scratch, binned gr_view, event) when the speculation binned it ahead
        self.rendered = None  # (saved sums, event) when the speculation also rendered it ahead (_render_launch)
        self.caps = caps  # device-side sizing (prepare_views_sized): the view's capacities, its plan for every later call

    def plan(self) -> _native.GrPlan:
        if self.caps is not None:  # no host read: the counts stay on the device (gr_view.device_counts)
            return self.caps
        self.event.synchronize()
        pairs, slots, core = (int(x) for x in self.plan_host.tolist())
        if pairs < 0 or slots < 0:
            raise RuntimeError("gr_fwd_prepare: pair count overflows int32")
        return _native.GrPlan(pairs, slots, core)


def prepare_native(means, scales, colors, opacities, gv: _native.GrView, plan_host=None) -> Prepared:
    """Enqueue gr_fwd_prepare_async for one view on the current stream (no host wait).  ``plan_host``: a
    pinned int64 tensor of 3 elements to receive the plan (a fit passes slices of one buffer it keeps)."""
    L = _native.lib()
    dev = means.device
    n = int(means.shape[0])
    cd = _color_dim(colors)
    geom = torch.empty((int(L.gr_geom_bytes(n)),), dtype=torch.uint8, device=dev)
    if plan_host is None:
        plan_host = torch.zeros(3, dtype=torch.int64, pin_memory=True)  # gr_plan {num_pairs, num_slots, num_core_pairs}
    _native.check(L.gr_fwd_prepare_async(ctypes.byref(gv), n, _native.ptr(means), _native.ptr(scales),
                                         _native.ptr(colors), cd, _native.ptr(opacities), _native.ptr(geom),
                                         geom.numel(), ctypes.c_void_p(plan_host.data_ptr()), _stream(dev)),
                  "gr_fwd_prepare_async")
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    return Prepared(gv, n, geom, plan_host, ev)


def prepare_views_native(means, scales, colors, opacities, gvs, plan_hosts) -> list:
    """gr_fwd_prepare_views_async: up to _native.PREPARE_MAX_VIEWS views of the same Gaussians prepared in one
    pass over the parameters, on the current stream; ``plan_hosts``: one pinned int64 tensor of 3 elements
    per view.  Returns one Prepared per view (they share one event)."""
    L = _native.lib()
    k = len(gvs)
    if not 1 <= k <= _native.PREPARE_MAX_VIEWS or len(plan_hosts) != k:
        raise ValueError(f"1 to {_native.PREPARE_MAX_VIEWS} views, one plan buffer each")
    _check_params(means, scales, colors, opacities)
    dev = means.device
    n = int(means.shape[0])
    nbytes = int(L.gr_geom_bytes(n))
    geoms = [torch.empty((nbytes,), dtype=torch.uint8, device=dev) for _ in range(k)]
    views = (_native.GrView * k)(*gvs)
    gptr = (ctypes.c_void_p * k)(*[g.data_ptr() for g in geoms])
    pptr = (ctypes.c_void_p * k)(*[p.data_ptr() for p in plan_hosts])
    _native.check(L.gr_fwd_prepare_views_async(k, views, n, _native.ptr(means), _native.ptr(scales), _native.ptr(colors),
                                               _color_dim(colors), _native.ptr(opacities), gptr, nbytes, pptr,
                                               _stream(dev)), "gr_fwd_prepare_views_async")
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    return [Prepared(gv, n, g, p, ev) for gv, g, p in zip(gvs, geoms, plan_hosts)]


def sized_view(gv: _native.GrView) -> _native.GrView:
    """gv with device_counts = 1 (made once per view structure and kept on it): the view of prepare_views_sized."""
    b = getattr(gv, "_sized_copy", None)
    if b is None:
        b = _native.GrView.from_buffer_copy(gv)
        b.device_counts = 1
        gv._sized_copy = b
    return b


def prepare_views_sized(means, scales, colors, opacities, gvs, caps, observed, overflow) -> list:
    """gr_fwd_prepare_views_sized on the current stream: as prepare_views_native for views with device_counts = 1
    (sized_view) against per-view capacities ``caps`` (GrPlan each; num_pairs / num_core_pairs bound the view's pairs
    / core pairs); ``observed``: one pinned int64 tensor of 3 elements per view (or None) receiving the true counts;
    ``overflow``: a device int32 raised when a view exceeds its capacity (it then renders without pairs).  The
    returned Prepared hand out their capacities as plans: no host wait anywhere after this call (the fit step can be
    captured in a graph)."""
    L = _native.lib()
    k = len(gvs)
    if not 1 <= k <= _native.PREPARE_MAX_VIEWS or len(caps) != k or len(observed) != k:
        raise ValueError(f"1 to {_native.PREPARE_MAX_VIEWS} views, one capacity and one observed buffer each")
    _check_params(means, scales, colors, opacities)
    dev = means.device
    n = int(means.shape[0])
    nbytes = int(L.gr_geom_bytes(n))
    geoms = [torch.empty((nbytes,), dtype=torch.uint8, device=dev) for _ in range(k)]
    views = (_native.GrView * k)(*gvs)
    capa = (_native.GrPlan * k)(*caps)
    gptr = (ctypes.c_void_p * k)(*[g.data_ptr() for g in geoms])
    optr = (ctypes.c_void_p * k)(*[o.data_ptr() if o is not None else None for o in observed])
    _native.check(L.gr_fwd_prepare_views_sized(k, views, n, _native.ptr(means), _native.ptr(scales), _native.ptr(colors),
                                               _color_dim(colors), _native.ptr(opacities), gptr, nbytes, capa, optr,
                                               _native.ptr(overflow), _stream(dev)), "gr_fwd_prepare_views_sized")
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    return [Prepared(gv, n, g, o, ev, caps=c) for gv, g, o, c in zip(gvs, geoms, observed, caps)]


def _bin_launch(L, gv, n, plan, prepared, bin_stream, dev):
    """gr_fwd_bin of a prepared view on ``bin_stream`` (after the preparation's event), into bins and scratch
    allocated there.  Returns (bins, scratch, the gr_view with binned = 1, the binning's end event)."""
    with torch.cuda.stream(bin_stream):
        bins = torch.empty((_ws_round(L.gr_bins_bytes(ctypes.byref(gv), n, ctypes.byref(plan))),), dtype=torch.uint8,
                           device=dev)
        scratch = torch.empty((_ws_round(L.gr_fwd_scratch_bytes(ctypes.byref(gv), n, ctypes.byref(plan))),),
                              dtype=torch.uint8, device=dev)
        bin_stream.wait_event(prepared.event)
        prepared.geom.record_stream(bin_stream)
        _native.check(L.gr_fwd_bin(ctypes.byref(gv), n, ctypes.byref(plan), _native.ptr(prepared.geom), _native.ptr(bins),
                                   bins.numel(), _native.ptr(scratch), scratch.numel(),
                                   ctypes.c_void_p(bin_stream.cuda_stream)), "gr_fwd_bin")
        done = torch.cuda.Event()
        done.record(bin_stream)
    return bins, scratch, _binned(gv), done


def _render_launch(L, prepared: Prepared, stream, dev) -> None:
    """The splat of a speculatively prepared view, ahead of its call, on ``stream``: its binning (_bin_launch, unless
    done) and gr_fwd_render_saved into saved sums; the call then only composes the outputs with its own background
    (forward_native).  Sets ``prepared.binned`` and ``prepared.rendered``."""
    plan = prepared.plan()
    if prepared.binned is None:
        prepared.binned = _bin_launch(L, prepared.gv, prepared.n, plan, prepared, stream, dev)
    bins, scratch, bgv, done = prepared.binned
    with torch.cuda.stream(stream):
        stream.wait_event(done)
        saved = torch.empty((int(L.gr_saved_floats(ctypes.byref(bgv))),), dtype=torch.float32, device=dev)
        _native.check(L.gr_fwd_render_saved(ctypes.byref(bgv), prepared.n, ctypes.byref(plan), _native.ptr(prepared.geom),
                                            _native.ptr(bins), bins.numel(), _native.ptr(scratch), scratch.numel(),
                                            _native.ptr(saved), ctypes.c_void_p(stream.cuda_stream)), "gr_fwd_render_saved")
        ev = torch.cuda.Event()
        ev.record(stream)
    prepared.rendered = (saved, ev)


def _bin_ahead(L, gv, n, plan, prepared, bin_stream, dev):
    """The bins and forward scratch of a render (allocated for the current stream); with ``bin_stream``
    filled by gr_fwd_bin there (_bin_launch), or already binned (``prepared.binned``, the speculation's),
    the current stream waiting for the binning.  Returns (bins, scratch, the gr_view to render with)."""
    pre = getattr(prepared, "binned", None) if prepared is not None else None
    if pre is None and bin_stream is None:
        bins = torch.empty((_ws_round(L.gr_bins_bytes(ctypes.byref(gv), n, ctypes.byref(plan))),), dtype=torch.uint8,
                           device=dev)
        scratch = torch.empty((_ws_round(L.gr_fwd_scratch_bytes(ctypes.byref(gv), n, ctypes.byref(plan))),),
                              dtype=torch.uint8, device=dev)
        return bins, scratch, gv
    if pre is not None and pre[2].cutoff == gv.cutoff and pre[2].no_depth_grad == gv.no_depth_grad:
        bins, scratch, _, done = pre
    else:
        bins, scratch, _, done = _bin_launch(L, gv, n, plan, prepared, bin_stream or torch.cuda.current_stream(dev), dev)
    # this render's own view (its background pointer), not the one the binning was launched with
    rv = _binned(gv)
    cur = torch.cuda.current_stream(dev)
    cur.wait_event(done)
    bins.record_stream(cur)
    scratch.record_stream(cur)
    return bins, scratch, rv


def forward_native(means, scales, colors, opacities, gv: _native.GrView, prepared: Optional[Prepared] = None,
                   want_depth: bool = True, images: bool = True, bin_stream=None):
    """Run gr_fwd_prepare(_async) + gr_fwd_render.  Returns (out, alpha, depth, RenderState).
    ``want_depth=False`` on a no_depth_grad view: no depth output (None) and no depth sums (gr_fwd_render
    with out_depth = NULL: the forward skips its depth channel).  ``images=False``: no output images at
    all (None, None, None; the saved sums for the backward only, as the fit loop needs).  ``bin_stream``
    (with ``prepared``): the view's binning runs there (gr_fwd_bin), beside whatever the current stream
    still has queued, and only the splat on the current stream."""
    L = _native.lib()
    dev = means.device
    n = int(means.shape[0])
    H, W = gv.height, gv.width
    s = _stream(dev)
    if prepared is None:
        prepared = prepare_native(means, scales, colors, opacities, gv)
    elif (prepared.n != n or prepared.gv.width != W or prepared.gv.height != H or prepared.gv.cutoff != gv.cutoff
          or prepared.gv.core_cutoff != gv.core_cutoff):
        raise ValueError("prepared view does not match this render (Gaussian count, image size or cutoffs)")
    geom = prepared.geom
    plan = prepared.plan()
    ahead = getattr(prepared, "rendered", None)
    if ahead is not None and images and prepared.binned[2].no_depth_grad == gv.no_depth_grad:
        # rendered ahead (the speculation's gr_fwd_render_saved): only the outputs, with this call's background
        saved, ev = ahead
        bins = prepared.binned[0]
        cur = torch.cuda.current_stream(dev)
        cur.wait_event(ev)
        for t in (saved, bins, geom):
            t.record_stream(cur)
        out = torch.empty((H, W, 3), dtype=torch.float32, device=dev)
        alpha = torch.empty((H, W), dtype=torch.float32, device=dev)
        depth = torch.empty((H, W), dtype=torch.float32, device=dev)
        _native.check(L.gr_fwd_compose(ctypes.byref(gv), _native.ptr(saved), _native.ptr(out), _native.ptr(alpha),
                                       _native.ptr(depth), s), "gr_fwd_compose")
        return out, alpha, depth, RenderState(gv, n, plan, geom, bins, saved)
    bins, scratch, rv = _bin_ahead(L, gv, n, plan, prepared, bin_stream, dev)
    out = torch.empty((H, W, 3), dtype=torch.float32, device=dev) if images else None
    alpha = torch.empty((H, W), dtype=torch.float32, device=dev) if images else None
    depth = (torch.empty((H, W), dtype=torch.float32, device=dev)
             if images and (want_depth or not gv.no_depth_grad) else None)
    saved = torch.empty((int(L.gr_saved_floats(ctypes.byref(gv))),), dtype=torch.float32, device=dev)
    # scratch is released when this function returns; the caching allocator keeps it stream-ordered
    _native.check(L.gr_fwd_render(ctypes.byref(rv), n, ctypes.byref(plan), _native.ptr(geom), _native.ptr(bins),
                                  bins.numel(), _native.ptr(scratch), scratch.numel(), _native.ptr(out), _native.ptr(alpha),
                                  _native.ptr(depth), _native.ptr(saved), s), "gr_fwd_render")
    del scratch
    return out, alpha, depth, RenderState(gv, n, plan, geom, bins, saved)


def backward_native(means, scales, colors, opacities, st: RenderState, g_out, g_alpha, g_depth, want_ws: bool = False,
                    index=None):
    """Run gr_bwd.  Returns (d_means, d_scales, d_colors, d_opacities) (+ the backward workspace with
    ``want_ws``: it holds the per-Gaussian sums camera_grad_native reads).  ``index`` (int32 device, n): the
    render was of a permuted copy; means .. opacities and the gradients are in the caller's order and index[r] is
    the rendered position of the caller's row r (gr_bwd_indexed)."""
    L = _native.lib()
    dev = means.device
    cd = _color_dim(colors)
    ws = torch.empty((_ws_round(L.gr_bwd_bytes(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan))),), dtype=torch.uint8,
                     device=dev)
    dm = torch.empty_like(means)
    ds = torch.empty_like(scales)
    dc = torch.empty_like(colors)
    do = torch.empty_like(opacities)
    if index is None:
        _native.check(L.gr_bwd(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan), _native.ptr(means), _native.ptr(scales),
                               _native.ptr(colors), cd, _native.ptr(opacities), _native.ptr(st.geom), _native.ptr(st.bins),
                               _native.ptr(st.saved), _native.ptr(g_out), _native.ptr(g_alpha), _native.ptr(g_depth),
                               _native.ptr(dm), _native.ptr(ds), _native.ptr(dc), _native.ptr(do), _native.ptr(ws),
                               ws.numel(), _stream(dev)), "gr_bwd")
    else:
        _native.check(L.gr_bwd_indexed(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan), _native.ptr(means),
                                       _native.ptr(scales), _native.ptr(colors), cd, _native.ptr(opacities),
                                       _native.ptr(st.geom), _native.ptr(st.bins), _native.ptr(st.saved), _native.ptr(g_out),
                                       _native.ptr(g_alpha), _native.ptr(g_depth), _native.ptr(index), _native.ptr(dm),
                                       _native.ptr(ds), _native.ptr(dc), _native.ptr(do), _native.ptr(ws), ws.numel(),
                                       _stream(dev)), "gr_bwd_indexed")
    return (dm, ds, dc, do, ws) if want_ws else (dm, ds, dc, do)


def camera_grad_native(means, scales, colors, opacities, st: RenderState, ws, depth: bool) -> torch.Tensor:
    """gr_bwd_camera on the current stream, after backward_native(..., want_ws=True) of the same render:
    (35,) device floats = d view (16, row-major), d proj (16), d cam_pos (3, SH colours only)."""
    L = _native.lib()
    out = torch.empty((_native.CAMERA_GRADS,), dtype=torch.float32, device=means.device)
    _native.check(L.gr_bwd_camera(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan), _native.ptr(means), _native.ptr(scales),
                                  _native.ptr(colors), _color_dim(colors), _native.ptr(opacities), _native.ptr(ws), ws.numel(),
                                  1 if depth else 0, _native.ptr(out), _stream(means.device)), "gr_bwd_camera")
    return out


def _camera_grads(d: torch.Tensor, view: Optional[torch.Tensor], proj: Optional[torch.Tensor], need_view: bool,
                  need_proj: bool, sh: bool):
    """gr_bwd_camera's 35 floats -> (d view, d proj) in the camera tensors' dtype and device.  With SH colours the
    camera centre cam = inv(view)[:3,3] (torch_renderer.py:81-83) also depends on view:
    d view += -inv(view)^T G inv(view)^T with G = d cam in column 3 (the inverse's differential)."""
    dview = dproj = None
    if need_view:
        dv = d[:16].view(4, 4).double()
        if sh:
            Vi = torch.linalg.inv(view.detach().to(device=d.device, dtype=torch.float64))
            G = torch.zeros((4, 4), dtype=torch.float64, device=d.device)
            G[:3, 3] = d[32:35].double()
            dv = dv - Vi.t() @ G @ Vi.t()
        dview = dv.to(dtype=view.dtype, device=view.device)
    if need_proj:
        dproj = d[16:32].view(4, 4).to(dtype=proj.dtype, device=proj.device)
    return dview, dproj


def backward_l1_native(means, scales, colors, opacities, st: RenderState, target, mask, w_sil: float, g_scale: float,
                       loss_out, grads, accumulate: bool) -> None:
    """gr_bwd_l1 on the current stream: the backward of the fit loop's view loss
    ``mean|out - target| + w_sil mean|alpha - mask|`` (mask may be None) scaled by ``g_scale``, written
    (accumulate=False) or added (accumulate=True) into ``grads`` = (d_means, d_scales, d_colors,
    d_opacities); the unscaled view loss goes to the 0-d / 1-element device tensor ``loss_out``."""
    L = _native.lib()
    dev = means.device
    ws = torch.empty((_ws_round(L.gr_bwd_bytes(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan))),), dtype=torch.uint8,
                     device=dev)
    dm, ds, dc, do = grads
    _native.check(L.gr_bwd_l1(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan), _native.ptr(means), _native.ptr(scales),
                              _native.ptr(colors), _color_dim(colors), _native.ptr(opacities), _native.ptr(st.geom),
                              _native.ptr(st.bins), _native.ptr(st.saved), _native.ptr(target), _native.ptr(mask),
                              ctypes.c_float(w_sil), ctypes.c_float(g_scale), _native.ptr(loss_out), _native.ptr(dm),
                              _native.ptr(ds), _native.ptr(dc), _native.ptr(do), 1 if accumulate else 0,
                              _native.ptr(ws), ws.numel(), _stream(dev)), "gr_bwd_l1")


def backward_fit_native(means, scales, colors, opacities, st: RenderState, target, mask, w_sil: float, depth_target,
                        w_depth: float, g_scale: float, loss_out, grads, accumulate: bool) -> None:
    """gr_bwd_fit on the current stream: as ``backward_l1_native`` with the fit loop's depth term
    ``w_depth mean|depth / (max(depth) + 1e-6) - depth_target|`` (the view rendered with depth_grad=True)."""
    L = _native.lib()
    dev = means.device
    _check_params(means, scales, colors, opacities)
    _check_operand(target, (st.gv.height, st.gv.width, 3), "target", dev)
    _check_operand(mask, (st.gv.height, st.gv.width), "mask", dev)
    _check_operand(depth_target, (st.gv.height, st.gv.width), "depth_target", dev)
    ws = torch.empty((_ws_round(L.gr_bwd_bytes(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan))),), dtype=torch.uint8,
                     device=dev)
    dm, ds, dc, do = grads
    _native.check(L.gr_bwd_fit(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan), _native.ptr(means), _native.ptr(scales),
                               _native.ptr(colors), _color_dim(colors), _native.ptr(opacities), _native.ptr(st.geom),
                               _native.ptr(st.bins), _native.ptr(st.saved), _native.ptr(target), _native.ptr(mask),
                               ctypes.c_float(w_sil), _native.ptr(depth_target), ctypes.c_float(w_depth),
                               ctypes.c_float(g_scale), _native.ptr(loss_out), _native.ptr(dm), _native.ptr(ds),
                               _native.ptr(dc), _native.ptr(do), 1 if accumulate else 0, _native.ptr(ws), ws.numel(),
                               _stream(dev)), "gr_bwd_fit")


def _check_operand(t, shape, name: str, dev) -> None:
    """A tensor the C ABI reads through its raw pointer (the fused fit path's targets, masks, depths and
    parameters): exactly ``shape``, float32, contiguous, on ``dev`` - anything else would be read as the
    wrong bytes, so it raises instead.  None passes (an optional operand)."""
    if t is None:
        return
    if (not isinstance(t, torch.Tensor) or tuple(t.shape) != tuple(shape) or t.dtype != torch.float32
            or not t.is_contiguous() or t.device != dev):
        got = (tuple(t.shape), t.dtype, t.device, t.is_contiguous()) if isinstance(t, torch.Tensor) else type(t)
        raise ValueError(f"{name}: expected a contiguous float32 tensor of shape {tuple(shape)} on {dev}, got {got}")


def _check_params(means, scales, colors, opacities) -> None:
    n, dev = int(means.shape[0]), means.device
    _check_operand(means, (n, 3), "means", dev)
    _check_operand(scales, (n, 3), "scales", dev)
    _check_operand(colors, (n,) + tuple(colors.shape[1:]), "colors", dev)
    _check_operand(opacities, (n,), "opacities", dev)


def _binned(gv: _native.GrView) -> _native.GrView:
    """gv with binned = 1 (made once per view structure and kept on it)."""
    b = getattr(gv, "_binned_copy", None)
    if b is None:
        b = _native.GrView.from_buffer_copy(gv)
        b.binned = 1
        gv._binned_copy = b
    return b


def forward_l1_native(means, scales, colors, opacities, gv: _native.GrView, prepared: Prepared, target, mask,
                      w_sil: float, g_scale: float, loss_out, bin_stream=None, out=None, alpha=None):
    """gr_fwd_render_l1 on the current stream (the fused fit path; gv with no_depth_grad, no depth output):
    the forward of one view whose epilogue evaluates the fit loss ``mean|out - target| + w_sil
    mean|alpha - mask|`` (mask may be None) into ``loss_out`` and its upstream gradients (scaled by
    ``g_scale``) into the backward workspace.  No image is written.  Returns (RenderState, workspace):
    pass them to ``backward_splat_native`` and then ``reduce_views_native``.  ``bin_stream``: run the
    view's binning (gr_fwd_bin) on that stream (after the preparation's event) and only the splat on the
    current one, which waits for it.  ``out`` (H,W,3) / ``alpha`` (H,W): float32 device tensors the render also
    writes its images into (tests; the fit path renders none)."""
    L = _native.lib()
    dev = means.device
    n = int(means.shape[0])
    if (prepared.n != n or prepared.gv.width != gv.width or prepared.gv.height != gv.height
            or prepared.gv.cutoff != gv.cutoff or prepared.gv.core_cutoff != gv.core_cutoff
            or prepared.gv.tile != gv.tile):
        raise ValueError("prepared view does not match this render (Gaussian count, image size, cutoffs or tile)")
    if out is not None:
        _check_operand(out, (gv.height, gv.width, 3), "out", dev)
    if alpha is not None:
        _check_operand(alpha, (gv.height, gv.width), "alpha", dev)
    _check_operand(target, (gv.height, gv.width, 3), "target", dev)
    _check_operand(mask, (gv.height, gv.width), "mask", dev)
    plan = prepared.plan()
    bins, scratch, rv = _bin_ahead(L, gv, n, plan, prepared, bin_stream, dev)
    ws = torch.empty((_ws_round(L.gr_bwd_bytes(ctypes.byref(gv), n, ctypes.byref(plan))),), dtype=torch.uint8, device=dev)
    _native.check(L.gr_fwd_render_l1(ctypes.byref(rv), n, ctypes.byref(plan), _native.ptr(prepared.geom),
                                     _native.ptr(bins), bins.numel(), _native.ptr(scratch), scratch.numel(),
                                     _native.ptr(target), _native.ptr(mask), ctypes.c_float(w_sil), ctypes.c_float(g_scale),
                                     _native.ptr(loss_out), _native.ptr(out) if out is not None else None,
                                     _native.ptr(alpha) if alpha is not None else None, _native.ptr(ws), ws.numel(),
                                     _stream(dev)),
                  "gr_fwd_render_l1")
    del scratch
    return RenderState(gv, n, plan, prepared.geom, bins, None), ws


def backward_splat_native(st: RenderState, ws) -> None:
    """gr_bwd_splat on the current stream: the backward splat of a view rendered by forward_l1_native;
    its per-pair gradient partials stay in ``ws`` for reduce_views_native."""
    L = _native.lib()
    _native.check(L.gr_bwd_splat(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan), _native.ptr(st.geom),
                                 _native.ptr(st.bins), _native.ptr(ws), ws.numel(), _stream(ws.device)), "gr_bwd_splat")


def reduce_views_native(means, scales, colors, opacities, batch, grads, accumulate: bool) -> None:
    """gr_reduce_views on the current stream: ``batch`` = [(RenderState, workspace) of views through
    forward_l1_native + backward_splat_native, ...] (at most _native.REDUCE_MAX_VIEWS); their summed gradient is written
    (accumulate=False) or added (accumulate=True) to ``grads`` = (d_means, d_scales, d_colors, d_opacities)."""
    L = _native.lib()
    if len(batch) > _native.REDUCE_MAX_VIEWS:
        raise ValueError(f"at most {_native.REDUCE_MAX_VIEWS} views per gr_reduce_views batch")
    _check_params(means, scales, colors, opacities)
    for g, p, nm in zip(grads, (means, scales, colors, opacities), ("d_means", "d_scales", "d_colors", "d_opacities")):
        _check_operand(g, tuple(p.shape), nm, means.device)
    arr = (_native.GrReduceView * max(1, len(batch)))()
    for k, (st, ws) in enumerate(batch):
        arr[k].view = st.gv
        arr[k].plan = st.plan
        arr[k].geom = st.geom.data_ptr()
        arr[k].bins = st.bins.data_ptr()
        arr[k].ws = ws.data_ptr()
    dm, ds, dc, do = grads
    _native.check(L.gr_reduce_views(len(batch), arr, int(means.shape[0]), _native.ptr(means), _native.ptr(scales),
                                    _native.ptr(colors), _color_dim(colors), _native.ptr(opacities), _native.ptr(dm),
                                    _native.ptr(ds), _native.ptr(dc), _native.ptr(do), 1 if accumulate else 0,
                                    _stream(means.device)), "gr_reduce_views")


def gather_view_native(st: RenderState, ws, sums=None):
    """gr_gather_view on the current stream: the per-Gaussian sums (n, 8) of a view's pair partials right
    after its backward_splat_native; the view's bins / geom / workspace may be dropped once it is enqueued
    (stream-ordered reuse).  Returns the sums tensor."""
    L = _native.lib()
    dev = ws.device
    if sums is None:
        sums = torch.empty((st.n, 8), dtype=torch.float32, device=dev)
    _check_operand(sums, (st.n, 8), "sums", dev)
    _native.check(L.gr_gather_view(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan), _native.ptr(st.geom),
                                   _native.ptr(st.bins), _native.ptr(ws), _native.ptr(sums), _stream(dev)),
                  "gr_gather_view")
    return sums


def backward_fit_gather_native(st: RenderState, target, mask, w_sil: float, depth_target, w_depth: float,
                               g_scale: float, loss_out):
    """gr_bwd_fit_gather on the current stream: the depth-loss backward of a view rendered with depth_grad=True up to
    its per-Gaussian sums; returns (sums (n, 8), depth sums (n,)) for reduce_sums_native (the view's geom, bins and
    saved sums are free after it)."""
    L = _native.lib()
    dev = st.saved.device
    _check_operand(target, (st.gv.height, st.gv.width, 3), "target", dev)
    _check_operand(mask, (st.gv.height, st.gv.width), "mask", dev)
    _check_operand(depth_target, (st.gv.height, st.gv.width), "depth_target", dev)
    ws = torch.empty((_ws_round(L.gr_bwd_bytes(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan))),), dtype=torch.uint8,
                     device=dev)
    sums = torch.empty((st.n, 8), dtype=torch.float32, device=dev)
    sums3 = torch.empty((st.n,), dtype=torch.float32, device=dev)
    _native.check(L.gr_bwd_fit_gather(ctypes.byref(st.gv), st.n, ctypes.byref(st.plan), _native.ptr(st.geom),
                                      _native.ptr(st.bins), _native.ptr(st.saved), _native.ptr(target), _native.ptr(mask),
                                      ctypes.c_float(w_sil), _native.ptr(depth_target), ctypes.c_float(w_depth),
                                      ctypes.c_float(g_scale), _native.ptr(loss_out), _native.ptr(ws), ws.numel(),
                                      _native.ptr(sums), _native.ptr(sums3), _stream(dev)), "gr_bwd_fit_gather")
    return sums, sums3


def reduce_sums_native(means, scales, colors, opacities, batch, grads, accumulate: bool) -> None:
    """gr_reduce_sums on the current stream: ``batch`` = [(gr_view, sums from gather_view_native), ...] or
    [(gr_view, sums, depth sums from backward_fit_gather_native), ...] (at most _native.REDUCE_MAX_VIEWS); the views'
    chain rules summed, written (accumulate=False) or added to ``grads`` = (d_means, d_scales, d_colors,
    d_opacities)."""
    L = _native.lib()
    if len(batch) > _native.REDUCE_MAX_VIEWS:
        raise ValueError(f"at most {_native.REDUCE_MAX_VIEWS} views per gr_reduce_sums batch")
    _check_params(means, scales, colors, opacities)
    n = int(means.shape[0])
    arr = (_native.GrSumsView * max(1, len(batch)))()
    for k, item in enumerate(batch):
        gv, sums = item[0], item[1]
        sums3 = item[2] if len(item) > 2 else None
        _check_operand(sums, (n, 8), "sums", means.device)
        _check_operand(sums3, (n,), "sums3", means.device)
        arr[k].view = gv
        arr[k].sums = sums.data_ptr()
        arr[k].sums3 = sums3.data_ptr() if sums3 is not None else None
    for g, p, nm in zip(grads, (means, scales, colors, opacities), ("d_means", "d_scales", "d_colors", "d_opacities")):
        _check_operand(g, tuple(p.shape), nm, means.device)
    dm, ds, dc, do = grads
    _native.check(L.gr_reduce_sums(len(batch), arr, n, _native.ptr(means), _native.ptr(scales), _native.ptr(colors),
                                   _color_dim(colors), _native.ptr(opacities), _native.ptr(dm), _native.ptr(ds),
                                   _native.ptr(dc), _native.ptr(do), 1 if accumulate else 0, _stream(means.device)),
                  "gr_reduce_sums")


def _grad_background(st: RenderState, background: torch.Tensor, g_out: torch.Tensor) -> torch.Tensor:
    """d(out)/d(bg) = sum_p g_out * [0<=out_r<=1] / (1+W)  (torch_renderer.py:194-196)."""
    HW = st.gv.width * st.gv.height
    acc = st.saved[: 4 * HW].view(HW, 4)
    den = 1.0 + acc[:, 0:1]
    out_r = (background.view(1, 3) + acc[:, 1:4]) / den
    mask = (out_r >= 0) & (out_r <= 1)
    return (g_out.reshape(HW, 3) * mask / den).sum(0)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means, scales, colors, opacities, background, view, proj, gv, prepared, gv_depth=None,
                bin_stream=None, layout=None, adapted=False, caller=None):
        """view / proj: the camera tensors (their gradients, gr_bwd_camera) or None; the render itself uses gv's
        host copy of them.  gv_depth: the f32-grade view a lazily rendered gv (two-piece mode) re-renders with
        when a depth gradient arrives (LAZY_DEPTH), else None.  bin_stream: see forward_native.  layout: a
        _Layout of the inputs (their Morton-ordered copy, rendered instead; the gradients return in the inputs'
        order), or None."""
        ctx.caller = caller  # the caller's adaptive state (_Caller) or None
        callers_t = (means, scales, colors, opacities) if layout is not None else (None,) * 4
        if layout is not None:
            means, scales, colors, opacities = layout.tensors
        out, alpha, depth, st = forward_native(means, scales, colors, opacities, gv, prepared, bin_stream=bin_stream)
        # an output the loss does not use gets a None gradient instead of zeros, so an unused depth
        # output lets the backward skip the tail pairs (gr_bwd with g_depth = NULL)
        ctx.set_materialize_grads(False)
        ctx.meta = (st.gv, st.n, st.plan)
        ctx.gv_depth = gv_depth
        ctx.adapted = adapted  # rendered at f32 grade because earlier backwards all differentiated the depth
        # the render state's device buffers are saved tensors: autograd releases them after this node's backward
        # unless the graph is retained (a second backward through it then finds them)
        ctx.save_for_backward(means, scales, colors, opacities, background, view, proj, st.geom, st.bins, st.saved,
                              layout.index if layout is not None else None, *callers_t)
        return out, alpha, depth

    @staticmethod
    def backward(ctx, g_out, g_alpha, g_depth):
        means, scales, colors, opacities, background, view, proj, geom, bins, saved, index, *caller = ctx.saved_tensors
        st = RenderState(*ctx.meta, geom, bins, saved)
        if g_out is None:
            g_out = torch.zeros((st.gv.height, st.gv.width, 3), dtype=torch.float32, device=means.device)
        g_out = g_out.contiguous().float()
        g_alpha = None if g_alpha is None else g_alpha.contiguous().float()
        g_depth = None if g_depth is None else g_depth.contiguous().float()
        if g_depth is not None and st.gv.no_depth_grad:
            if ctx.gv_depth is None:
                raise RuntimeError("the depth output was rendered with depth_grad=False and cannot be differentiated; "
                                   "render with depth_grad=True")
            # lazy default: the depth is differentiated after all - re-render at f32 grade with the
            # depth-gradient footprint and differentiate that render
            _, _, _, st = forward_native(means, scales, colors, opacities, ctx.gv_depth, images=False)
            if ctx.caller is not None:
                with _LOCK:
                    ctx.caller.rerenders += 1
                    if LAZY_ADAPT and ctx.caller.rerenders >= LAZY_ADAPT:
                        ctx.caller.eager = True
        elif g_depth is None and (ctx.gv_depth is not None or ctx.adapted) and ctx.caller is not None:
            with _LOCK:
                ctx.caller.rerenders, ctx.caller.eager = 0, False  # this loss has no depth term (any more)
        need_view, need_proj = ctx.needs_input_grad[5], ctx.needs_input_grad[6]
        # with a layout: the chain rule in the caller's order (its tensors; the rendered copy's sums gathered by index)
        dm, ds, dc, do, ws = backward_native(*(caller if index is not None else (means, scales, colors, opacities)), st,
                                             g_out, g_alpha, g_depth, want_ws=True, index=index)
        dbg = _grad_background(st, background, g_out) if ctx.needs_input_grad[4] else None
        dview = dproj = None
        if need_view or need_proj:
            d = camera_grad_native(means, scales, colors, opacities, st, ws, g_depth is not None)
            dview, dproj = _camera_grads(d, view, proj, need_view, need_proj, colors.dim() == 3)
        return dm, ds, dc, do, dbg, dview, dproj, None, None, None, None, None, None, None


def _device_inputs(means, scales, colors, opacities):
    dev = means.device
    if dev.type != "cuda":
        raise RuntimeError("the MI355X renderer needs tensors on a HIP device (got %s); there is no CPU path" % dev)
    return (means.to(torch.float32).contiguous(), scales.to(device=dev, dtype=torch.float32).contiguous(),
            colors.to(device=dev, dtype=torch.float32).contiguous(),
            opacities.to(device=dev, dtype=torch.float32).contiguous())


def prepare_view(means, scales, colors, opacities, view, proj, width, height, background=None,
                 cutoff=None, core_cutoff=DEFAULT_CORE_CUTOFF, depth_grad=True, plan_host=None) -> Prepared:
    """Enqueue the preparation of one view (see ``Prepared``); pass it to ``rasterize(prepared=...)``
    with the same tensors, cutoffs and ``depth_grad``.  The tensors' values must not change in between.
    depth_grad=True prepares the view rasterize renders first in the lazy default (the no-depth-gradient
    footprint); "eager" the f32-grade view."""
    if depth_grad is True and not _eager(depth_grad) and cutoff is None:
        gv = make_view(view, proj, width, height, background, None, core_cutoff, False)
    else:
        gv = make_view(view, proj, width, height, background, cutoff, core_cutoff, bool(depth_grad))
    return prepare_native(*_device_inputs(means, scales, colors, opacities), gv, plan_host)


# ------------------------------------------------------------------------------------------------
# Preparation ahead for callers that render view after view through the autograd op (the reference fit
# loop, fit_multiview_stub.py:277-290, calls render_gaussians_torch once per camera with the same
# activation tensors).  A render needs its view's pair count on the host before the binning can be
# enqueued; without help that is one host wait per view for a preparation enqueued just before it.
# The op learns the camera order and keeps a two-deep pipeline of the cameras expected next, with the same
# input tensors, on a stream of its own: after rendering camera A the preparation of the camera two ahead is
# enqueued, and on entering the render of A the camera after A (prepared one render ago: its plan is on the
# host) is binned, before A's splat is enqueued, so the binning runs beside A's splat.  A render uses its
# pipeline entry when camera and tensors match (the same live tensor objects at the same versions: weak
# references, so a freed tensor never matches) and otherwise drops the pipeline.  A transition that missed
# is not speculated the next time.  GR_SPECULATE=0 turns this off; GR_SPEC_BIN=0 keeps the binning in the
# render.
# ------------------------------------------------------------------------------------------------
SPECULATE = os.environ.get("GR_SPECULATE", "1") != "0"
SPEC_BIN = os.environ.get("GR_SPEC_BIN", "1") != "0"
# the camera after the one being rendered is also splatted ahead (gr_fwd_render_saved), so its call only composes
# the outputs with the background it passes (gr_fwd_compose): the splats of consecutive calls run back to back on the
# speculation stream while the host runs the caller's per-view code
SPEC_RENDER = os.environ.get("GR_SPEC_RENDER", "1") != "0"
# cameras prepared ahead: with the render-ahead, the one after the next is prepared before the next one's splat is
# enqueued, so taking its plan never waits behind a splat
SPEC_DEPTH = 3 if SPEC_RENDER else 2


class _Speculation:
    __slots__ = ("key", "refs", "versions", "prepared", "src")

    def __init__(self, key, tensors, prepared, src):
        self.key, self.prepared, self.src = key, prepared, src
        self.refs = tuple(weakref.ref(t) for t in tensors)
        self.versions = tuple(t._version for t in tensors)

    def matches(self, key, tensors) -> bool:
        return key == self.key and all(r() is t and t._version == v
                                       for r, t, v in zip(self.refs, tensors, self.versions))


# hit / miss counters over all devices; the learned camera order and the pipeline per device (_spec_of)
_SPEC: dict = {"hits": 0, "misses": 0}


def _spec_of(dev: torch.device) -> dict:
    key = ("dev", str(dev))
    d = _SPEC.get(key)
    if d is None:
        d = _SPEC[key] = {"last": None, "next": {}, "views": {}, "cold": set(), "pipe": [], "stream": None}
    return d


def _view_key(gv: _native.GrView) -> tuple:
    return (bytes(gv.view), bytes(gv.proj), gv.width, gv.height, gv.cutoff, gv.core_cutoff, gv.no_depth_grad)


def _spec_take(key, tensors) -> Optional[Prepared]:
    """The speculative preparation of this view, if the pipeline's head is exactly these inputs; then the
    next entry is binned on the speculation stream (before this view's kernels are enqueued)."""
    D = _spec_of(tensors[0].device)
    pipe = D["pipe"]
    if not pipe:
        return None
    sp = pipe.pop(0)
    if not sp.matches(key, tensors):
        _SPEC["misses"] += 1
        D["cold"].add((sp.src, sp.key))
        pipe.clear()
        return None
    _SPEC["hits"] += 1
    D["cold"].discard((sp.src, key))
    if pipe and pipe[0].prepared.rendered is None and (SPEC_RENDER or (SPEC_BIN and pipe[0].prepared.binned is None)):
        nx = pipe[0].prepared
        dev = tensors[0].device
        if SPEC_RENDER:  # the next camera's binning and splat, beside this view's compose, losses and host work
            _render_launch(_native.lib(), nx, _spec_stream(dev), dev)
        else:
            nx.binned = _bin_launch(_native.lib(), nx.gv, nx.n, nx.plan(), nx, _spec_stream(dev), dev)
    return sp.prepared


def _spec_stream(dev: torch.device) -> "torch.cuda.Stream":
    D = _spec_of(dev)
    if D["stream"] is None:
        D["stream"] = torch.cuda.Stream(dev)
    return D["stream"]


def _spec_after(key, gv, tensors, inputs_ready) -> None:
    """Learn the camera order and fill the pipeline with the cameras expected next: their preparations on a
    stream of their own that waits only for the input tensors (``inputs_ready``, recorded before this
    view's kernels), so they run beside this view's render."""
    D = _spec_of(tensors[0].device)
    last = D["last"]
    if last is not None:
        D["next"][last] = key
    D["last"] = key
    D["views"][key] = gv
    if len(D["views"]) > 4096:
        D["views"].clear()
        D["next"].clear()
    pipe = D["pipe"]
    ps = None
    while len(pipe) < SPEC_DEPTH:
        src = pipe[-1].key if pipe else key
        nxt = D["next"].get(src)
        if nxt is None or (src, nxt) in D["cold"] or nxt == key:
            return
        if ps is None:
            ps = _spec_stream(tensors[0].device)
            ps.wait_event(inputs_ready)
            for t in tensors:  # read on ps: not reused by the allocator before ps is done with them
                t.record_stream(ps)
        with torch.cuda.stream(ps):
            pv = prepare_native(*tensors, D["views"][nxt])
        pipe.append(_Speculation(nxt, tensors, pv, src))


# ------------------------------------------------------------------------------------------------
# Spatial layout of the drop-in op.  A caller's Gaussians come in its own order (the reference fit loop's are in
# random order, fit_multiview_stub.py:114-137); the tile sort, the splats' record gathers and the per-Gaussian
# gathers all run several times faster on Morton-ordered Gaussians (spatial.py).  The op renders a Morton-ordered
# copy of its inputs - made once per set of input tensors (the same live tensors at the same versions: a fit
# loop's activations, shared by all the views of an iteration) - and gr_bwd_indexed writes each Gaussian's
# gradients back to the caller's row, so nothing outside sees the copy (results differ from an unpermuted render
# only in float summation order).  The permutation itself is kept per means tensor (a fit's parameter, updated in
# place) and recomputed every LAYOUT_EVERY input sets.  GR_DROPIN_LAYOUT=0 turns this off.
# ------------------------------------------------------------------------------------------------
LAYOUT = os.environ.get("GR_DROPIN_LAYOUT", "1") != "0"
LAYOUT_MIN = 32768  # Gaussians from which the copy pays for itself
LAYOUT_EVERY = 16   # input sets rendered with one permutation before it is recomputed


class _Layout:
    """tensors: the rendered (Morton-ordered) copy; index: int32, the rendered position of each caller row."""
    __slots__ = ("refs", "versions", "tensors", "index")

    def __init__(self, inputs, tensors, index):
        self.refs = tuple(weakref.ref(t) for t in inputs)
        self.versions = tuple(t._version for t in inputs)
        self.tensors, self.index = tensors, index

    def matches(self, inputs) -> bool:
        return all(r() is t and t._version == v for r, t, v in zip(self.refs, inputs, self.versions))


def _layout_of(caller: _Caller, m, s, c, o) -> _Layout:
    """The Morton-ordered copy of these input tensors (cached: one entry per caller)."""
    e = caller.layout
    if e is not None and e.matches((m, s, c, o)):
        return e
    pc = caller.perm  # [weakref(means), n, perm int64, inverse int32, uses]
    if pc is None or pc[0]() is not m or pc[1] != m.shape[0] or pc[4] >= LAYOUT_EVERY:
        perm = spatial.morton_order(m)
        inv = torch.empty_like(perm, dtype=torch.int32)
        inv[perm] = torch.arange(perm.numel(), dtype=torch.int32, device=perm.device)
        pc = caller.perm = [weakref.ref(m), m.shape[0], perm, inv, 0]
    pc[4] += 1
    with torch.no_grad():
        tensors = tuple(t.detach().index_select(0, pc[2]).contiguous() for t in (m, s, c, o))
    e = caller.layout = _Layout((m, s, c, o), tensors, pc[3])
    return e


def rasterize(means, scales, colors, opacities, view, proj, width, height, background=None, cutoff=None,
              prepared: Optional[Prepared] = None, core_cutoff=DEFAULT_CORE_CUTOFF, depth_grad=True):
    """Differentiable render of one view on the HIP device: returns (rgb (H,W,3), alpha (H,W), depth (H,W)).

    ``prepared`` (from ``prepare_view`` with the same inputs) skips the preparation step;
    ``depth_grad``: True (default: the depth may be differentiated; rendered lazily, see LAZY_DEPTH),
    "eager" (f32-grade render up front), False (see ``make_view``)."""
    dev = means.device
    if dev.type != "cuda":
        # tensors on the host: the dense CPU op (config C1; cpu_renderer.py).  HIP tensors never take it.
        if background is None:
            background = torch.zeros(3, dtype=torch.float32, device=dev)
        return cpu_renderer.render(means, scales, colors, opacities, view, proj, width, height,
                                   background.to(dtype=torch.float32, device=dev))
    with _LOCK:  # the op's adaptive state (per caller) and speculation pipeline (per device)
        return _rasterize_hip(means, scales, colors, opacities, view, proj, width, height, background, cutoff, prepared,
                              core_cutoff, depth_grad)


def _rasterize_hip(means, scales, colors, opacities, view, proj, width, height, background, cutoff, prepared,
                   core_cutoff, depth_grad):
    dev = means.device
    caller = _caller_of(means)
    m, s, c, o = _device_inputs(means, scales, colors, opacities)
    if background is None:
        background = _default_background(dev)
    background = background.to(dtype=torch.float32, device=dev).reshape(3).contiguous()
    gv_depth = None
    adapted = depth_grad is True and not _eager(depth_grad) and cutoff is None and caller.eager
    if depth_grad is True and not _eager(depth_grad) and cutoff is None and not adapted:
        # lazy default: two-piece render with the no-depth-gradient footprint now, f32 grade only if needed
        gv_depth = make_view(view, proj, width, height, background, None, core_cutoff, True)
        gv = make_view(view, proj, width, height, background, None, core_cutoff, False)
    else:
        gv = make_view(view, proj, width, height, background, cutoff, core_cutoff, bool(depth_grad))
    if prepared is not None and (prepared.gv.cutoff != gv.cutoff or prepared.gv.no_depth_grad != gv.no_depth_grad):
        # a preparation made for the other mode (prepare_view(depth_grad="eager"), GR_LAZY_DEPTH=0, or adaptive
        # laziness switched since): render the prepared view
        gv, gv_depth = prepared.gv, None
        adapted = False
    # the camera tensors enter the autograd op only when a gradient is wanted for them (gr_bwd_camera)
    cam_v = view if isinstance(view, torch.Tensor) and view.requires_grad else None
    cam_p = proj if isinstance(proj, torch.Tensor) and proj.requires_grad else None
    if prepared is not None:  # a preparation made by prepare_view is of the caller's own order: render that
        return _RasterizeGaussians.apply(m, s, c, o, background, cam_v, cam_p, gv, prepared, gv_depth, None, None, adapted,
                                         caller)
    # the rendered tensors: the Morton-ordered copy of the inputs
    layout = _layout_of(caller, m, s, c, o) if LAYOUT and m.shape[0] >= LAYOUT_MIN else None
    if not SPECULATE:
        return _RasterizeGaussians.apply(m, s, c, o, background, cam_v, cam_p, gv, None, gv_depth, None, layout, adapted,
                                         caller)
    rt = layout.tensors if layout is not None else (m, s, c, o)
    key = _view_key(gv)
    pv = _spec_take(key, rt)
    stream = torch.cuda.current_stream(dev)
    if pv is not None:
        stream.wait_event(pv.event)
        pv.geom.record_stream(stream)
    ready = torch.cuda.Event()
    ready.record(stream)
    res = _RasterizeGaussians.apply(m, s, c, o, background, cam_v, cam_p, gv, pv, gv_depth, None, layout, adapted, caller)
    _spec_after(key, gv, rt, ready)
    return res


def render_gaussians_torch(
    means: torch.Tensor,  # (N,3) float32
    scales: torch.Tensor,  # (N,3) float32
    colors: torch.Tensor,  # (N,3) or SH coeffs (N,4,3); extension: degree-3 coefficients (N,16,3)
    opacities: torch.Tensor,  # (N,)  float32
    camera: Camera,
    width: int,
    height: int,
    background: Optional[torch.Tensor] = None,  # (3,)
    max_gaussians: int = 10000,
    chunk_size: int = 256,
    return_aux: bool = False,
    cutoff: Optional[float] = None,
    prepared: Optional[Prepared] = None,
    core_cutoff: float = DEFAULT_CORE_CUTOFF,
    depth_grad=True,
):
    """Differentiable Gaussian splat; signature, results and errors of torch_renderer.py:109-203.

    Returns ``out`` (H,W,3) or ``(out, alpha, depth)`` when ``return_aux``; ``n == 0`` returns a
    single zero image even with ``return_aux`` (torch_renderer.py:135-136).  ``cutoff``,
    ``core_cutoff``, ``prepared`` (see ``prepare_view``) and ``depth_grad`` (see ``make_view``) are
    extensions; the reference has none.
    """
    if background is None:
        background = _default_background(means.device)
    background = background.to(dtype=torch.float32, device=means.device)

    if means.ndim != 2 or means.shape[1] != 3:
        raise ValueError("means must be (N,3)")
    n = means.shape[0]
    if n == 0:
        return torch.zeros((height, width, 3), dtype=torch.float32, device=means.device)
    if n > max_gaussians:
        raise ValueError(f"N={n} too large for torch reference renderer. Increase max_gaussians or downsample.")
    if not ((colors.ndim == 2 and colors.shape[1] == 3) or (colors.ndim == 3 and colors.shape[1] in (4, 16) and colors.shape[2] == 3)):
        raise ValueError("colors must be (N,3) or SH coeffs (N,4,3)")

    out, alpha, depth = rasterize(means, scales, colors, opacities, camera.view, camera.proj, width, height,
                                  background=background, cutoff=cutoff, prepared=prepared, core_cutoff=core_cutoff,
                                  depth_grad=depth_grad)
    if not return_aux:
        return out
    return out, alpha, depth


__all__ = ["Camera", "get_default_device", "perspective", "look_at", "render_gaussians_torch", "rasterize",
           "make_view", "prepare_view", "prepare_native", "Prepared", "forward_native", "backward_native",
           "backward_l1_native", "backward_fit_native", "backward_fit_gather_native", "forward_l1_native", "backward_splat_native", "reduce_views_native",
           "gather_view_native", "reduce_sums_native",
           "DEFAULT_CUTOFF", "DEPTH_GRAD_CUTOFF", "DEFAULT_CORE_CUTOFF", "FIT_CUTOFF", "default_cutoff"]
