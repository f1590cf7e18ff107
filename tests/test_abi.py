"""CPU: the C-ABI library loads and exports every function include/gr_hip.h declares (no GPU
compute calls here); the host-only introspection entry points work."""
from __future__ import annotations

import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "gr_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-zA-Z_][\w\s\*]*?\b(gr_\w+)\s*\(", text, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("gr_fwd_prepare", "gr_fwd_render", "gr_bwd", "gr_render_u8", "gr_last_error", "gr_geom_bytes",
                 "gr_bins_bytes", "gr_bwd_bytes", "gr_fwd_scratch_bytes", "gr_saved_floats"):
        assert must in names


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg._native.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_every_declared_symbol_has_a_ctypes_signature(pkg):
    """_native binds exactly the header's entry points (argument and result types set before any call)."""
    assert sorted(pkg._native._SIG) == declared_functions()


def test_version_and_error_string(pkg):
    assert "gfx950" in pkg._native.version()
    assert isinstance(pkg._native.lib().gr_last_error(), bytes)


def test_layouts_are_aligned_and_ordered(pkg):
    off = pkg._native.geom_layout(1000)
    assert off == sorted(off) and all(o % 256 == 0 for o in off)
    gv = pkg.torch_renderer.make_view(__import__("numpy").eye(4, dtype="float32"),
                                      __import__("numpy").eye(4, dtype="float32"), 800, 800)
    b = pkg._native.bins_layout(gv, 1000, 12345)
    assert b == sorted(b) and all(o % 256 == 0 for o in b)
    assert b[2] - b[1] >= 4 * 12345  # sorted Gaussian ids
    assert b[3] > b[2]  # pos_of after the ranges


def test_struct_sizes_match_header(pkg):
    # gr_view: 2 ints + 16 + 16 + 3 + 3 + 2 floats + 1 int, then the background_dev pointer (8-aligned);
    # gr_render_params: RenderParams' layout
    from oracle import oracle as orc
    # then binned, tile, device_counts, chunk, row0, rows
    assert ctypes.sizeof(pkg._native.GrView) == 4 * (2 + 16 + 16 + 3 + 3 + 2 + 1) + 4 + 8 + 24
    assert [f[0] for f in pkg._native.GrView._fields_] == [f[0] for f in orc.GrView._fields_]
    assert ctypes.sizeof(pkg._native.GrRenderParams) == 4 * (2 + 16 + 16 + 3 + 3)
    # gr_param_step: int64, 2 ints, 2 pointers, GR_FIT_MAX_ACC pointers, 2 pointers, 3 floats (+ tail padding)
    assert ctypes.sizeof(pkg._native.GrParamStep) == 8 + 8 + 16 + 8 * 8 + 16 + 16


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No silent fallback: pointing GR_HIP_LIB at nothing makes the loader raise."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("_native_probe", os.path.join(REPO, "3dgaussian_amd", "_native.py"))
    mod = importlib.util.module_from_spec(spec)
    monkeypatch.setenv("GR_HIP_LIB", str(tmp_path / "nope.so"))
    spec.loader.exec_module(mod)
    with pytest.raises(ImportError):
        mod.lib()


def _integration_snippet() -> str:
    """The ctypes example of INTEGRATION.md §4 (the second python block of the file)."""
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", text, flags=re.S)
    snip = [b for b in blocks if "gr_fwd_prepare" in b]
    assert len(snip) == 1
    return snip[0].replace('ctypes.CDLL("3dgaussian_amd/libgr_hip.so")',
                           'ctypes.CDLL(os.path.join(REPO, "3dgaussian_amd", "libgr_hip.so"))')


def test_integration_ctypes_example_plan_layout(pkg):
    """The example's GrPlan has the 24-byte layout of gr_plan (the library writes three int64)."""
    ns = {}
    snip = _integration_snippet()
    cls = snip[snip.index("class GrPlan"):snip.index("lib.gr_geom_bytes")]
    exec("import ctypes\n" + cls, ns)
    assert ctypes.sizeof(ns["GrPlan"]) == 24 == ctypes.sizeof(pkg._native.GrPlan)


@pytest.mark.gpu
def test_integration_ctypes_example_runs(pkg):
    """INTEGRATION.md §4's ctypes snippet, run as written against the built library: the plan it
    reads back equals the one the package's own binding gets."""
    import numpy as np
    import torch

    from oracle import oracle as orc

    sc = orc.synthetic_scene(2000, seed=4, scale=0.04)
    view, proj = orc.orbit_cameras(4, 96, 64)[1]
    means, scales, colors, opac = (torch.from_numpy(a).cuda() for a in sc.arrays())
    n = means.shape[0]
    gv = pkg.torch_renderer.make_view(view, proj, 96, 64)
    ns = {"os": os, "REPO": REPO, "torch": torch, "view": gv, "n": n, "means": means, "scales": scales,
          "colors": colors, "opac": opac, "GrRenderParams": pkg._native.GrRenderParams}
    exec(_integration_snippet(), ns)
    torch.cuda.synchronize()
    ref = pkg.torch_renderer.prepare_native(means, scales, colors, opac, gv).plan()
    got = ns["plan"]
    assert (got.num_pairs, got.num_core_pairs) == (int(ref.num_pairs), int(ref.num_core_pairs))
    assert got.num_pairs > 0 and np.isfinite(got.num_pairs)


def test_u8_force_cpu_empty_scene_is_the_cpu_background(pkg):
    """gr_render_u8 with n == 0 runs on the host only (no device call): the CUDA renderer's contract gives an all-zero
    image (renderer.cu:279-281); RenderParams.force_cpu = 1 the CPU renderer's (renderer_cpu.cpp:219-240: the finalized
    background, alpha 255), bit-exact against its compiled-reference goldens, both modes."""
    import numpy as np

    from conftest import golden

    gr = pkg.gaussian_renderer
    for name in ("u8_n0_17x13_sort0", "u8_n0_17x13_sort1"):
        d = golden(name)
        args = (d["means"], d["scales"], d["colors"], d["opacities"], int(d["width"]), int(d["height"]),
                np.ascontiguousarray(d["view"]), np.ascontiguousarray(d["proj"]), np.ascontiguousarray(d["background"]))
        assert not gr.render_gaussians(*args, enable_depth_sort=int(d["sort"])).any()
        np.testing.assert_array_equal(gr.render_gaussians(*args, enable_depth_sort=int(d["sort"]), force_cpu=1), d["rgba"])
