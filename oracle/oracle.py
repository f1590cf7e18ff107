"""TEST INFRASTRUCTURE ONLY — numpy/ctypes front end of the CPU oracle (oracle/gr_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product package (3dgaussian_amd/) never does.  The oracle restates the reference render op:

  * dense forward/backward: python/torch_renderer.py:57-203 (+ autograd, fit_multiview_stub.py:310)
  * binned forward/backward: the same math restricted to the 16x16 tiles a Gaussian's
    cutoff*sigma box overlaps (the HIP product's semantics; rectangles bit-exact)
  * uint8 surface: src/renderer_cpu.cpp:34-260 (OIT and depth-sorted modes)

It is pinned against tests/golden/*.npz (tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

TILE = 16


class GrView(ctypes.Structure):
    """Mirror of gr_view (include/gr_hip.h)."""

    _fields_ = [
        ("width", ctypes.c_int),
        ("height", ctypes.c_int),
        ("view", ctypes.c_float * 16),
        ("proj", ctypes.c_float * 16),
        ("background", ctypes.c_float * 3),
        ("cam_pos", ctypes.c_float * 3),
        ("cutoff", ctypes.c_float),
        ("core_cutoff", ctypes.c_float),
        ("no_depth_grad", ctypes.c_int),  # product precision mode; the oracle always computes in float64
        ("background_dev", ctypes.c_void_p),  # product only (device background); the oracle reads background
        ("binned", ctypes.c_int),  # product only (gr_fwd_bin ran); the oracle always bins
        ("tile", ctypes.c_int),  # tile edge of the binned semantics: 0/16 or 32
        ("device_counts", ctypes.c_int),  # (the HIP path's device-side sizing; the oracle ignores it)
        ("chunk", ctypes.c_int),  # (the HIP path's work-item length; the oracle ignores it)
        ("row0", ctypes.c_int),  # a band of tile rows [row0, row0 + rows) (rows 0: the whole view)
        ("rows", ctypes.c_int),
    ]


class GrRenderParams(ctypes.Structure):
    """Mirror of gr_render_params (include/gr_hip.h) == gr::RenderParams (gaussian_types.h:24-46)."""

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


def build() -> str:
    """Compile liboracle.so (gcc) if missing or stale; return its path."""
    import subprocess

    so = os.path.join(_HERE, "liboracle.so")
    src = os.path.join(_HERE, "gr_oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return so


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(build())
        f = ctypes.c_void_p
        _LIB.gro_preprocess.argtypes = [ctypes.POINTER(GrView), ctypes.c_int, f, f, f, ctypes.c_int, f, f, f, f]
        _LIB.gro_bin.argtypes = [ctypes.POINTER(GrView), ctypes.c_int] + [f] * 7
        _LIB.gro_bin.restype = ctypes.c_int64
        _LIB.gro_forward.argtypes = [ctypes.POINTER(GrView), ctypes.c_int, f, f, f, ctypes.c_int, f, ctypes.c_int] + [f] * 4
        _LIB.gro_backward.argtypes = [ctypes.POINTER(GrView), ctypes.c_int, f, f, f, ctypes.c_int, f, ctypes.c_int] + [f] * 7
        _LIB.gro_render_u8.argtypes = [ctypes.POINTER(GrRenderParams), ctypes.c_int] + [f] * 5
        _LIB.gro_dense_pixels.argtypes = [ctypes.POINTER(GrView), ctypes.c_int, f, f, f, ctypes.c_int, f, ctypes.c_int] + [f] * 4
        _LIB.gro_dense_grads_sel.argtypes = ([ctypes.POINTER(GrView), ctypes.c_int, f, f, f, ctypes.c_int, f] + [f] * 3
                                             + [ctypes.c_int] + [f] * 5)
    return _LIB


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


@dataclass
class Scene:
    means: np.ndarray  # (N,3)
    scales: np.ndarray  # (N,3)
    colors: np.ndarray  # (N,3) or (N,4,3)
    opacities: np.ndarray  # (N,)

    def arrays(self):
        return _f32(self.means), _f32(self.scales), _f32(self.colors), _f32(self.opacities)


def camera_position(view: np.ndarray) -> np.ndarray:
    return np.linalg.inv(np.asarray(view, dtype=np.float64))[:3, 3].astype(np.float32)


def make_view(view, proj, width, height, background=None, cutoff=7.0, core_cutoff=0.0, tile=0) -> GrView:
    """core_cutoff <= 0 (default) = one zone; the product's default is DEFAULT_CORE_CUTOFF (5.5).  tile: the binned
    semantics' tile edge (0/16, or 32 as the fit path's gr_view.tile)."""
    v = GrView()
    v.width, v.height = int(width), int(height)
    v.view[:] = [float(x) for x in np.asarray(view, dtype=np.float32).reshape(16)]
    v.proj[:] = [float(x) for x in np.asarray(proj, dtype=np.float32).reshape(16)]
    bg = np.zeros(3, np.float32) if background is None else np.asarray(background, np.float32).reshape(3)
    v.background[:] = [float(x) for x in bg]
    v.cam_pos[:] = [float(x) for x in camera_position(view)]
    v.cutoff = float(cutoff)
    v.core_cutoff = float(core_cutoff)
    v.tile = int(tile)
    return v


def color_dim(colors: np.ndarray) -> int:
    if colors.ndim == 2 and colors.shape[1] == 3:
        return 3
    if colors.ndim == 3 and colors.shape[1:] == (4, 3):
        return 12
    if colors.ndim == 3 and colors.shape[1:] == (16, 3):  # degree-3 extension (build only)
        return 48
    raise ValueError("colors must be (N,3) or SH coeffs (N,4,3)")


def preprocess(v: GrView, scene: Scene):
    m, s, c, o = scene.arrays()
    n = m.shape[0]
    rec = np.zeros((n, 12), np.float32)
    rect = np.zeros((n, 4), np.int32)
    counts = np.zeros((n,), np.int32)
    lib().gro_preprocess(ctypes.byref(v), n, _p(m), _p(s), _p(c), color_dim(c), _p(o), _p(rec), _p(rect), _p(counts))
    return rec, rect, counts


def bin_pairs(v: GrView, rec: np.ndarray, rect: np.ndarray, counts: np.ndarray):
    """Stable (virtual tile, Gaussian) pair lists, virtual tile = 2*tile + (1 for a tail pair);
    rec/rect/counts from preprocess().  ranges: (2*tiles, 2)."""
    n = counts.shape[0]
    rec = np.ascontiguousarray(rec, np.float32)
    te = 32 if v.tile == 32 else TILE
    tiles = math.ceil(v.width / te) * math.ceil(v.height / te)
    offsets = np.zeros((n + 1,), np.int32)
    rect = np.ascontiguousarray(rect, np.int32)
    counts = np.ascontiguousarray(counts, np.int32)
    K = lib().gro_bin(ctypes.byref(v), n, _p(rec), _p(rect), _p(counts), _p(offsets), None, None, None)
    keys = np.zeros((max(K, 1),), np.uint32)
    vals = np.zeros((max(K, 1),), np.int32)
    ranges = np.zeros((2 * tiles, 2), np.int32)
    lib().gro_bin(ctypes.byref(v), n, _p(rec), _p(rect), _p(counts), _p(offsets), _p(keys), _p(vals), _p(ranges))
    return offsets, keys[:K], vals[:K], ranges


def forward(v: GrView, scene: Scene, binned: bool = False, return_saved: bool = False):
    m, s, c, o = scene.arrays()
    n = m.shape[0]
    H, W = v.height, v.width
    out = np.zeros((H, W, 3), np.float32)
    alpha = np.zeros((H, W), np.float32)
    depth = np.zeros((H, W), np.float32)
    saved = np.zeros((H * W, 5), np.float32) if return_saved else None
    lib().gro_forward(ctypes.byref(v), n, _p(m), _p(s), _p(c), color_dim(c), _p(o), int(binned), _p(out), _p(alpha), _p(depth), _p(saved))
    if return_saved:
        return out, alpha, depth, saved
    return out, alpha, depth


def backward(v: GrView, scene: Scene, g_rgb, g_alpha=None, g_depth=None, binned: bool = False):
    m, s, c, o = scene.arrays()
    n = m.shape[0]
    g_rgb = _f32(g_rgb)
    g_alpha = None if g_alpha is None else _f32(g_alpha)
    g_depth = None if g_depth is None else _f32(g_depth)
    dm = np.zeros_like(m)
    ds = np.zeros_like(s)
    dc = np.zeros_like(c)
    do = np.zeros_like(o)
    lib().gro_backward(ctypes.byref(v), n, _p(m), _p(s), _p(c), color_dim(c), _p(o), int(binned), _p(g_rgb), _p(g_alpha), _p(g_depth), _p(dm), _p(ds), _p(dc), _p(do))
    return dm, ds, dc, do


def dense_pixels(v: GrView, scene: Scene, pix: np.ndarray):
    """Dense (no cutoff, every Gaussian) float64 out (P,3), alpha (P,), depth (P,) at pixel indices y*W+x."""
    m, s, c, o = scene.arrays()
    pix = np.ascontiguousarray(pix, np.int32)
    P = pix.shape[0]
    out = np.zeros((P, 3), np.float32)
    alpha = np.zeros((P,), np.float32)
    depth = np.zeros((P,), np.float32)
    lib().gro_dense_pixels(ctypes.byref(v), m.shape[0], _p(m), _p(s), _p(c), color_dim(c), _p(o), P, _p(pix),
                           _p(out), _p(alpha), _p(depth))
    return out, alpha, depth


def dense_grads_sel(v: GrView, scene: Scene, sel: np.ndarray, g_rgb, g_alpha=None, g_depth=None):
    """Exact gradients of the selected Gaussians over the whole image (no cutoff), per-pixel sums from the
    binned forward: (d_means, d_scales, d_colors, d_opac) rows in sel order."""
    m, s, c, o = scene.arrays()
    sel = np.ascontiguousarray(sel, np.int32)
    k = sel.shape[0]
    g_rgb = _f32(g_rgb)
    g_alpha = None if g_alpha is None else _f32(g_alpha)
    g_depth = None if g_depth is None else _f32(g_depth)
    dm = np.zeros((k, 3), np.float32)
    ds = np.zeros((k, 3), np.float32)
    dc = np.zeros((k,) + c.shape[1:], np.float32)
    do = np.zeros((k,), np.float32)
    lib().gro_dense_grads_sel(ctypes.byref(v), m.shape[0], _p(m), _p(s), _p(c), color_dim(c), _p(o), _p(g_rgb),
                              _p(g_alpha), _p(g_depth), k, _p(sel), _p(dm), _p(ds), _p(dc), _p(do))
    return dm, ds, dc, do


def render_u8(width, height, view, proj, scene: Scene, background=None, enable_depth_sort=0) -> np.ndarray:
    """Restatement of gr::render_gaussians_cpu (renderer_cpu.cpp:34-260): (H,W,4) uint8."""
    m, s, c, o = scene.arrays()
    p = GrRenderParams()
    p.width, p.height = int(width), int(height)
    p.view[:] = [float(x) for x in np.asarray(view, np.float32).reshape(16)]
    p.proj[:] = [float(x) for x in np.asarray(proj, np.float32).reshape(16)]
    bg = np.zeros(3, np.float32) if background is None else np.asarray(background, np.float32).reshape(3)
    p.background[:] = [float(x) for x in bg]
    p.enable_depth_sort = int(enable_depth_sort)
    p.depth_slices = 16
    out = np.zeros((height, width, 4), np.uint8)
    lib().gro_render_u8(ctypes.byref(p), m.shape[0], _p(m), _p(s), _p(c), _p(o), _p(out))
    return out


# ---------------------------------------------------------------------------------------------
# Camera helpers restating torch_renderer.py:24-54 and fit_multiview_stub.py:70-90 in numpy
# (float32), so tests and the bench can build views without the product package.
# ---------------------------------------------------------------------------------------------
def perspective(fovy_deg, aspect, znear, zfar) -> np.ndarray:
    f = np.float32(1.0) / np.tan(np.float32(fovy_deg) * np.float32(math.pi) / np.float32(180.0) * np.float32(0.5))
    m = np.zeros((4, 4), np.float32)
    m[0, 0] = f / np.float32(aspect)
    m[1, 1] = f
    m[2, 2] = (zfar + znear) / (znear - zfar)
    m[2, 3] = (2.0 * zfar * znear) / (znear - zfar)
    m[3, 2] = -1.0
    return m


def look_at(eye, target, up) -> np.ndarray:
    eye = np.asarray(eye, np.float32)
    target = np.asarray(target, np.float32)
    up = np.asarray(up, np.float32)
    f = target - eye
    f = f / (np.linalg.norm(f) + np.float32(1e-8))
    u = up / (np.linalg.norm(up) + np.float32(1e-8))
    s = np.cross(f, u)
    s = s / (np.linalg.norm(s) + np.float32(1e-8))
    u2 = np.cross(s, f)
    m = np.eye(4, dtype=np.float32)
    m[0, :3] = s
    m[1, :3] = u2
    m[2, :3] = -f
    t = np.eye(4, dtype=np.float32)
    t[:3, 3] = -eye
    return (m @ t).astype(np.float32)


def orbit_cameras(num_views, width, height, radius=2.5, pitch=0.2):
    proj = perspective(60.0, width / height, 0.01, 100.0)
    cams = []
    for i in range(num_views):
        yaw = (2.0 * math.pi * i) / max(1, num_views)
        eye = [radius * math.cos(pitch) * math.sin(yaw), radius * math.sin(pitch), radius * math.cos(pitch) * math.cos(yaw)]
        cams.append((look_at(eye, [0, 0, 0], [0, 1, 0]), proj))
    return cams


def synthetic_scene(n, seed=0, scale=None, sh=False) -> Scene:
    """Seeded synthetic scene of SURVEY.md §8(d) (numpy generator; stub init distributions)."""
    rng = np.random.default_rng(seed)
    means = ((rng.random((n, 3), dtype=np.float32) - 0.5) * 1.2).astype(np.float32)
    if scale is None:
        scale = 0.1061 * (1200.0 / max(n, 1)) ** (1.0 / 3.0)
    scales = np.full((n, 3), scale, np.float32)
    opac = np.full((n,), 1.0 / (1.0 + math.exp(2.2)), np.float32)
    if sh:
        colors = np.zeros((n, 4, 3), np.float32)
        colors[:, 0, :] = 0.1 * rng.random((n, 3), dtype=np.float32)
    else:
        colors = (1.0 / (1.0 + np.exp(-0.1 * rng.random((n, 3), dtype=np.float32)))).astype(np.float32)
    return Scene(means, scales, colors, opac)


def rel_l2(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.linalg.norm(b.ravel())
    num = np.linalg.norm((a - b).ravel())
    if den == 0.0:
        return float(num)
    return float(num / den)


def psnr(a, b, peak=1.0) -> float:
    mse = float(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2))
    if mse == 0.0:
        return float("inf")
    return 10.0 * math.log10(peak * peak / mse)
