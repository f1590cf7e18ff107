"""Legacy uint8 surface: drop-in for the reference's pybind11 module ``gaussian_renderer``
(src/bindings.cpp:27-100), backed by gr_render_u8 in libgr_hip.so (HIP-only dispatch, replacing
src/renderer_dispatch.cpp and src/renderer.cu).

``render_gaussians(means, scales, colors, opacities, width=800, height=600, view, proj,
background=None) -> np.ndarray (H,W,4) uint8`` with the binding's validation and messages
(RuntimeError).  Semantics are renderer_cpu.cpp's: 3-sigma box, w < 1e-5 skip, no clamps, uint8
round-half-up, alpha 255.  ``enable_depth_sort=1`` (an extension argument; RenderParams field at
gaussian_types.h:37) gives exact per-pixel front-to-back compositing in camera-z order.  ``force_cpu=1`` (an
extension argument, RenderParams.force_cpu: renderer_dispatch.cpp:12-13) asks for the CPU renderer's contract, which
this HIP path already follows except at n == 0: the background with alpha 255 (renderer_cpu.cpp:219-240) instead of
the CUDA renderer's all-zero image (renderer.cu:279-281).
"""
from __future__ import annotations

import ctypes

import numpy as np

try:
    from . import _native
except ImportError:  # pragma: no cover
    import _native  # type: ignore


def _require_contiguous_f32(arr, name: str) -> None:
    # bindings.cpp:15-25
    if not isinstance(arr, np.ndarray):
        raise RuntimeError(f"{name} must be a numpy array")
    if arr.dtype.kind != "f" or arr.itemsize != 4:
        raise RuntimeError(f"{name} must be float32")
    if not arr.flags["C_CONTIGUOUS"]:
        raise RuntimeError(f"{name} must be C-contiguous")


_MISSING = object()


def render_gaussians(means, scales, colors, opacities, width=800, height=600, view=_MISSING, proj=_MISSING,
                     background=None, enable_depth_sort=0, force_cpu=0):
    if view is _MISSING or proj is _MISSING:
        raise TypeError("render_gaussians() missing required arguments: 'view' and 'proj'")
    _require_contiguous_f32(means, "means")
    _require_contiguous_f32(scales, "scales")
    _require_contiguous_f32(colors, "colors")
    _require_contiguous_f32(opacities, "opacities")
    _require_contiguous_f32(view, "view")
    _require_contiguous_f32(proj, "proj")
    # bindings.cpp:48-53
    if means.ndim != 2 or means.shape[1] != 3:
        raise RuntimeError("means must be (N,3)")
    if scales.ndim != 2 or scales.shape[1] != 3:
        raise RuntimeError("scales must be (N,3)")
    if colors.ndim != 2 or colors.shape[1] != 3:
        raise RuntimeError("colors must be (N,3)")
    if opacities.ndim != 1:
        raise RuntimeError("opacities must be (N,)")
    if view.ndim != 2 or view.shape != (4, 4):
        raise RuntimeError("view must be (4,4)")
    if proj.ndim != 2 or proj.shape != (4, 4):
        raise RuntimeError("proj must be (4,4)")
    if background is None:
        bg = np.zeros((3,), np.float32)
    else:
        bg = background
        _require_contiguous_f32(bg, "background")
        if bg.ndim != 1 or bg.shape[0] != 3:
            raise RuntimeError("background must be (3,)")
    n = int(means.shape[0])
    if scales.shape[0] != n or colors.shape[0] != n or opacities.shape[0] != n:
        raise RuntimeError("means/scales/colors/opacities must have matching N")

    p = _native.GrRenderParams()
    p.width, p.height = int(width), int(height)
    p.view[:] = view.reshape(16).tolist()
    p.proj[:] = proj.reshape(16).tolist()
    p.background[:] = bg.reshape(3).tolist()
    p.enable_depth_sort = int(enable_depth_sort)
    p.depth_slices = 16
    p.force_cpu = int(force_cpu)
    out = np.empty((int(height), int(width), 4), np.uint8)
    L = _native.lib()
    st = L.gr_render_u8(ctypes.byref(p), n, means.ctypes.data_as(ctypes.c_void_p), scales.ctypes.data_as(ctypes.c_void_p),
                        colors.ctypes.data_as(ctypes.c_void_p), opacities.ctypes.data_as(ctypes.c_void_p),
                        out.ctypes.data_as(ctypes.c_void_p))
    if st != _native.GR_OK:
        raise RuntimeError(L.gr_last_error().decode("utf-8", "replace"))
    return out


__doc_module__ = "3D Gaussian renderer core bindings"  # bindings.cpp:28 m.doc()
