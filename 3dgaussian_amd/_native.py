"""ctypes binding of the in-tree HIP library libgr_hip.so (C ABI declared in include/gr_hip.h).

This is the Python side of the drop-in boundary: it replaces the reference's pybind11 module
(src/bindings.cpp) and the pure-torch math of python/torch_renderer.py with calls into hand-written
gfx950 kernels.  There is no fallback: if the library is missing or cannot be loaded, importing the
renderer raises, so a GPU test can never pass on a silent CPU/eager path.

torch is imported first on purpose: the wheel ships its own libamdhip64.so (SONAME libamdhip64.so.7),
and loading it before libgr_hip.so makes our library bind to the same HIP runtime instance as torch,
so torch device pointers and streams are valid inside our calls.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load; see module docstring)

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GR_HIP_LIB", os.path.join(_PKG_DIR, "libgr_hip.so"))

TILE = 16

GR_OK = 0
GR_ERR_INVALID_ARGUMENT = 1
GR_ERR_HIP = 2
GR_ERR_WORKSPACE = 3
GR_ERR_OVERFLOW = 4


class GrView(ctypes.Structure):
    """gr_view (include/gr_hip.h)."""

    _fields_ = [
        ("width", ctypes.c_int),
        ("height", ctypes.c_int),
        ("view", ctypes.c_float * 16),
        ("proj", ctypes.c_float * 16),
        ("background", ctypes.c_float * 3),
        ("cam_pos", ctypes.c_float * 3),
        ("cutoff", ctypes.c_float),
        ("core_cutoff", ctypes.c_float),
        ("no_depth_grad", ctypes.c_int),
        ("background_dev", ctypes.c_void_p),  # optional device pointer to the 3 background floats
        ("binned", ctypes.c_int),  # 1: gr_fwd_bin already built the bins; the render launches only the splat
        ("tile", ctypes.c_int),  # screen tile edge: 0/16 (default) or 32 (fused fit path)
        ("device_counts", ctypes.c_int),  # 1: plans are capacities, the counts stay on the device (sized preparation)
        ("chunk", ctypes.c_int),  # work-item length in pairs (0: the default 2048)
        ("row0", ctypes.c_int),  # a band of tile rows [row0, row0 + rows) (rows 0: the whole view)
        ("rows", ctypes.c_int),
    ]


class GrRenderParams(ctypes.Structure):
    """gr_render_params (include/gr_hip.h); same field order as gr::RenderParams
    (include/gr/gaussian_types.h:24-46)."""

    _fields_ = [
        ("width", ctypes.c_int),
        ("height", ctypes.c_int),
        ("view", ctypes.c_float * 16),
        ("proj", ctypes.c_float * 16),
        ("background", ctypes.c_float * 3),
        ("enable_depth_sort", ctypes.c_int),
        ("depth_slices", ctypes.c_int),
        ("force_cpu", ctypes.c_int),
    ]


class GrPlan(ctypes.Structure):
    """gr_plan (include/gr_hip.h): sizes produced by gr_fwd_prepare."""

    _fields_ = [("num_pairs", ctypes.c_int64), ("num_slots", ctypes.c_int64), ("num_core_pairs", ctypes.c_int64)]


CAMERA_GRADS = 35  # GR_CAMERA_GRADS: d view (16), d proj (16), d cam_pos (3)
REDUCE_MAX_VIEWS = 16  # GR_REDUCE_MAX_VIEWS
PREPARE_MAX_VIEWS = 8  # GR_PREPARE_MAX_VIEWS


class GrReduceView(ctypes.Structure):
    """gr_reduce_view (include/gr_hip.h): one view of a gr_reduce_views batch."""

    _fields_ = [("view", GrView), ("plan", GrPlan), ("geom", ctypes.c_void_p), ("bins", ctypes.c_void_p),
                ("ws", ctypes.c_void_p)]


class GrSumsView(ctypes.Structure):
    """gr_sums_view (include/gr_hip.h): one view of a gr_reduce_sums batch."""

    _fields_ = [("view", GrView), ("sums", ctypes.c_void_p), ("sums3", ctypes.c_void_p)]


class GrFitTarget(ctypes.Structure):
    """gr_fit_target (include/gr_hip.h): one view of a gr_fit_views call."""

    _fields_ = [("view", GrView), ("target_rgb", ctypes.c_void_p), ("target_mask", ctypes.c_void_p),
                ("target_depth", ctypes.c_void_p)]


class GrFitConfig(ctypes.Structure):
    """gr_fit_config (include/gr_hip.h): the native fit executor's schedule."""

    _fields_ = [("num_streams", ctypes.c_int), ("prep_ahead", ctypes.c_int), ("prep_group", ctypes.c_int),
                ("prep_first", ctypes.c_int), ("reduce_batch", ctypes.c_int), ("reduce_tail", ctypes.c_int),
                ("render_streams", ctypes.POINTER(ctypes.c_void_p)), ("prep_stream", ctypes.c_void_p),
                ("caps", ctypes.POINTER(GrPlan)), ("observed", ctypes.c_void_p), ("overflow", ctypes.c_void_p)]


FIT_MAX_ACC = 8      # GR_FIT_MAX_ACC
FIT_MAX_PARAMS = 8   # GR_FIT_MAX_PARAMS


class GrParamStep(ctypes.Structure):
    """gr_param_step (include/gr_hip.h): one parameter tensor of a gr_fit_param_steps launch."""

    _fields_ = [("count", ctypes.c_int64), ("act", ctypes.c_int), ("num_accs", ctypes.c_int), ("param", ctypes.c_void_p),
                ("grad", ctypes.c_void_p), ("accs", ctypes.c_void_p * FIT_MAX_ACC), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("reg", ctypes.c_float), ("neg_step_size", ctypes.c_float),
                ("bias_correction2_sqrt", ctypes.c_float)]


BATCH_MAX_VIEWS = 8  # GR_BATCH_MAX_VIEWS


class GrBatchView(ctypes.Structure):
    """gr_batch_view (include/gr_hip.h): one view of a gr_fit_views_batched call."""

    _fields_ = [("view", GrView), ("plan", GrPlan), ("geom", ctypes.c_void_p), ("bins", ctypes.c_void_p),
                ("bins_bytes", ctypes.c_size_t), ("scratch", ctypes.c_void_p), ("scratch_bytes", ctypes.c_size_t),
                ("ws", ctypes.c_void_p), ("ws_bytes", ctypes.c_size_t), ("saved", ctypes.c_void_p),
                ("target_rgb", ctypes.c_void_p), ("target_mask", ctypes.c_void_p), ("target_depth", ctypes.c_void_p),
                ("sums", ctypes.c_void_p), ("sums3", ctypes.c_void_p), ("loss", ctypes.c_void_p)]


class NativeLibraryError(ImportError):
    pass


_lib = None

_P = ctypes.c_void_p
_VP = ctypes.POINTER(GrView)
_PP = ctypes.POINTER(GrPlan)
_SIG = {
    "gr_geom_bytes": (ctypes.c_size_t, [ctypes.c_int]),
    "gr_fwd_prepare": (ctypes.c_int, [_VP, ctypes.c_int, _P, _P, _P, ctypes.c_int, _P, _P, ctypes.c_size_t, _PP, _P]),
    "gr_fwd_prepare_async": (ctypes.c_int, [_VP, ctypes.c_int, _P, _P, _P, ctypes.c_int, _P, _P, ctypes.c_size_t, _P, _P]),
    "gr_fwd_prepare_views_async": (ctypes.c_int, [ctypes.c_int, _VP, ctypes.c_int, _P, _P, _P, ctypes.c_int, _P,
                                                  ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                                  ctypes.POINTER(ctypes.c_void_p), _P]),
    "gr_fwd_prepare_views_sized": (ctypes.c_int, [ctypes.c_int, _VP, ctypes.c_int, _P, _P, _P, ctypes.c_int, _P,
                                                  ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, _PP,
                                                  ctypes.POINTER(ctypes.c_void_p), _P, _P]),
    "gr_fit_views_batched": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(GrBatchView), ctypes.c_int, ctypes.c_float,
                                            ctypes.c_float, ctypes.c_float, _P]),
    "gr_bins_bytes": (ctypes.c_size_t, [_VP, ctypes.c_int, _PP]),
    "gr_saved_floats": (ctypes.c_size_t, [_VP]),
    "gr_fwd_scratch_bytes": (ctypes.c_size_t, [_VP, ctypes.c_int, _PP]),
    "gr_fwd_render": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, ctypes.c_size_t, _P, ctypes.c_size_t, _P, _P, _P, _P, _P]),
    "gr_fwd_render_saved": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, ctypes.c_size_t, _P, ctypes.c_size_t, _P, _P]),
    "gr_fwd_compose": (ctypes.c_int, [_VP, _P, _P, _P, _P, _P]),
    "gr_fwd_bin": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, ctypes.c_size_t, _P, ctypes.c_size_t, _P]),
    "gr_bwd_bytes": (ctypes.c_size_t, [_VP, ctypes.c_int, _PP]),
    "gr_bwd": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, _P, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P,
                              _P, _P, _P, _P, _P, ctypes.c_size_t, _P]),
    "gr_bwd_indexed": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, _P, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _P,
                                      _P, _P, _P, _P, _P, ctypes.c_size_t, _P]),
    "gr_bwd_camera": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, _P, ctypes.c_int, _P, _P, ctypes.c_size_t, ctypes.c_int,
                                     _P, _P]),
    "gr_bwd_l1": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, _P, ctypes.c_int, _P, _P, _P, _P, _P, _P,
                                 ctypes.c_float, ctypes.c_float, _P, _P, _P, _P, _P, ctypes.c_int, _P, ctypes.c_size_t,
                                 _P]),
    "gr_bwd_fit": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, _P, ctypes.c_int, _P, _P, _P, _P, _P, _P,
                                  ctypes.c_float, _P, ctypes.c_float, ctypes.c_float, _P, _P, _P, _P, _P, ctypes.c_int, _P,
                                  ctypes.c_size_t, _P]),
    "gr_fit_param_step": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, _P, _P, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                         ctypes.c_float, ctypes.c_int, _P,
                                         _P, ctypes.c_float, ctypes.c_float, ctypes.c_double, ctypes.c_double, ctypes.c_float,
                                         _P]),
    "gr_adam_step": (ctypes.c_int, [ctypes.c_int64, _P, _P, _P, _P, ctypes.c_float, ctypes.c_float, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_float, _P]),
    "gr_fit_param_steps": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(GrParamStep), ctypes.c_double, ctypes.c_double,
                                          ctypes.c_float, _P]),
    "gr_fit_param_steps_sched": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(GrParamStep), ctypes.c_double, ctypes.c_double,
                                                ctypes.c_float, _P, _P, _P, _P, _P]),
    "gr_fit_activations_ws_bytes": (ctypes.c_size_t, [ctypes.c_int64]),
    "gr_fit_activations": (ctypes.c_int, [ctypes.c_int64, _P, _P, _P, ctypes.c_int64, _P, _P, _P, ctypes.c_float,
                                          ctypes.c_float, _P, _P, ctypes.c_size_t, _P]),
    "gr_fwd_render_l1": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, ctypes.c_size_t, _P, ctypes.c_size_t, _P, _P,
                                        ctypes.c_float, ctypes.c_float, _P, _P, _P, _P, ctypes.c_size_t, _P]),
    "gr_bwd_splat": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, _P, ctypes.c_size_t, _P]),
    "gr_reduce_views": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(GrReduceView), ctypes.c_int, _P, _P, _P, ctypes.c_int,
                                       _P, _P, _P, _P, _P, ctypes.c_int, _P]),
    "gr_view_sums_floats": (ctypes.c_size_t, [ctypes.c_int]),
    "gr_gather_view": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, _P, _P, _P]),
    "gr_bwd_fit_gather": (ctypes.c_int, [_VP, ctypes.c_int, _PP, _P, _P, _P, _P, _P, ctypes.c_float, _P, ctypes.c_float,
                                         ctypes.c_float, _P, _P, ctypes.c_size_t, _P, _P, _P]),
    "gr_reduce_sums": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(GrSumsView), ctypes.c_int, _P, _P, _P, ctypes.c_int,
                                      _P, _P, _P, _P, _P, ctypes.c_int, _P]),
    "gr_executor_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "gr_executor_destroy": (None, [_P]),
    "gr_fit_views": (ctypes.c_int, [_P, ctypes.POINTER(GrFitConfig), ctypes.c_int, ctypes.POINTER(GrFitTarget), ctypes.c_int,
                                    _P, _P, _P, ctypes.c_int, _P, ctypes.c_float, ctypes.c_float, ctypes.c_float, _P,
                                    ctypes.POINTER(ctypes.c_void_p), _P]),
    "gr_render_u8": (ctypes.c_int, [ctypes.POINTER(GrRenderParams), ctypes.c_int, _P, _P, _P, _P, _P]),
    "gr_geom_layout": (None, [ctypes.c_int, ctypes.POINTER(ctypes.c_size_t)]),
    "gr_bins_layout": (None, [_VP, ctypes.c_int, _PP, ctypes.POINTER(ctypes.c_size_t)]),
    "gr_profile_begin": (None, []),
    "gr_profile_end": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
    "gr_l1_loss_ws_bytes": (ctypes.c_size_t, []),
    "gr_l1_loss_fwd": (ctypes.c_int, [_P, _P, ctypes.c_int64, _P, _P, ctypes.c_int64, ctypes.c_float, _P, _P,
                                      ctypes.c_size_t, _P]),
    "gr_l1_loss_bwd": (ctypes.c_int, [_P, _P, ctypes.c_int64, _P, _P, ctypes.c_int64, ctypes.c_float, _P, _P, _P, _P]),
    "gr_last_error": (ctypes.c_char_p, []),
    "gr_version": (ctypes.c_char_p, []),
}


def lib() -> ctypes.CDLL:
    """Load libgr_hip.so (once).  Raises NativeLibraryError when it is absent: no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"HIP extension {LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C 3dgaussian_amd/csrc`) first")
    try:
        handle = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the box
        raise NativeLibraryError(f"cannot load HIP extension {LIB_PATH}: {e}") from e
    for name, (res, args) in _SIG.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    _lib = handle
    return _lib


def check(status: int, what: str = "") -> None:
    """Map a gr_status to the reference's exception types (bindings.cpp raises RuntimeError,
    torch_renderer.py raises ValueError for argument errors)."""
    if status == GR_OK:
        return
    msg = lib().gr_last_error().decode("utf-8", "replace")
    if what:
        msg = f"{what}: {msg}"
    if status == GR_ERR_INVALID_ARGUMENT:
        raise ValueError(msg)
    raise RuntimeError(msg)


def ptr(t) -> ctypes.c_void_p:
    """Device/host pointer of a tensor (None -> NULL)."""
    if t is None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(t.data_ptr())


def profile_begin() -> None:
    lib().gr_profile_begin()


PROFILE_STAGES = ("raster_fwd", "raster_bwd", "reduce_bwd", "binning")


def profile_end():
    """Returns {stage: (total_ms, launches)} for PROFILE_STAGES."""
    ms = (ctypes.c_double * 4)()
    n = (ctypes.c_int * 4)()
    check(lib().gr_profile_end(ms, n), "gr_profile_end")
    return {k: (ms[i], n[i]) for i, k in enumerate(PROFILE_STAGES)}


def version() -> str:
    return lib().gr_version().decode()


GEOM_PARTS = 6


def geom_layout(n: int):
    """[records ((n+1) x 32 B, then z_abs[n+1]), rect, counts (core | tail << 32, u64), their exclusive
    scan, device plan, end of the fixed part] (gr_hip.h gr_geom_layout)."""
    out = (ctypes.c_size_t * GEOM_PARTS)()
    lib().gr_geom_layout(int(n), out)
    return list(out)


def bins_layout(gv: GrView, n: int, num_pairs: int):
    """[keys (radix path), sorted Gaussian ids int[K], ranges int2[2 tiles], pos_of int[K]]."""
    out = (ctypes.c_size_t * 4)()
    plan = GrPlan(int(num_pairs), 0, 0)
    lib().gr_bins_layout(ctypes.byref(gv), int(n), ctypes.byref(plan), out)
    return list(out)


_EXECUTORS: dict = {}


def executor(device: int) -> ctypes.c_void_p:
    """The native fit executor of a device (gr_executor_create), created once per process."""
    ex = _EXECUTORS.get(device)
    if ex is None:
        ex = ctypes.c_void_p()
        check(lib().gr_executor_create(int(device), ctypes.byref(ex)), "gr_executor_create")
        _EXECUTORS[device] = ex
    return ex
