"""CPU: pin the oracle (oracle/gr_oracle.c) against the reference's own golden vectors.

Goldens (tests/golden/make_golden.py): F1 edge cases and F2 (the C1 scene) from the reference's
python/torch_renderer.py (float32 forward + autograd backward); F3 uint8 from the reference's
src/renderer_cpu.cpp compiled from source.  The oracle accumulates in float64, so for tensors
where the reference's own float32 rounding exceeds 1e-4 (ill-conditioned sums) the bar is the
larger of 1e-4 and 1.5 x what an independent float32 evaluation could be expected to deviate.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import golden, golden_names
from oracle import oracle as orc

FLOAT_GOLDENS = golden_names("f1_") + golden_names("f2_")
KEYS = ("out_rgb", "out_alpha", "out_depth", "d_means", "d_scales", "d_colors", "d_opacities")


CUTOFF = 7.0  # product defaults (3dgaussian_amd/torch_renderer.py DEFAULT_CUTOFF, DEFAULT_CORE_CUTOFF)
CORE = 5.5


def _run(d, binned, cutoff=CUTOFF, core=CORE, depth=True):
    v = orc.make_view(d["view"], d["proj"], int(d["width"]), int(d["height"]), d["background"], cutoff=cutoff,
                      core_cutoff=core)
    sc = orc.Scene(d["means"], d["scales"], d["colors"], d["opacities"])
    out, a, dep = orc.forward(v, sc, binned=binned)
    dm, ds, dc, do = orc.backward(v, sc, d["g_rgb"], d["g_alpha"], d["g_depth"] if depth else None, binned=binned)
    return dict(zip(KEYS, (out, a, dep, dm, ds, dc, do)))


@pytest.mark.parametrize("name", FLOAT_GOLDENS)
def test_dense_oracle_matches_reference(name):
    d = golden(name)
    if d["means"].shape[0] == 0:
        assert not d["out_rgb"].any()  # reference returns zeros for N == 0 (torch_renderer.py:135-136)
        return
    r = _run(d, binned=False)
    for k in KEYS:
        err = orc.rel_l2(r[k], d[k])
        # f1_n1 d_opacities: one cancelling sum where float32 torch is 2.4e-4 from exact
        tol = 3e-4 if (name == "f1_n1_17x13" and k == "d_opacities") else 1e-4
        assert err <= tol, f"{name} {k}: {err:.3e}"


@pytest.mark.parametrize("name", FLOAT_GOLDENS)
def test_binned_two_zone_matches_reference(name):
    """The product's semantics (7-sigma elliptical tile footprint, 5.5-sigma core) against the dense
    reference."""
    d = golden(name)
    if d["means"].shape[0] == 0:
        return
    r = _run(d, binned=True)
    for k in KEYS:
        err = orc.rel_l2(r[k], d[k])
        tol = 3e-4 if (name == "f1_n1_17x13" and k == "d_opacities") else 1e-4
        assert err <= tol, f"{name} {k}: {err:.3e}"
    assert orc.psnr(r["out_rgb"], d["out_rgb"]) >= 60.0


def test_6sigma_is_not_enough_with_depth_gradients():
    """Why the footprint is 7 sigma: with upstream depth gradients, d depth/d w is amplified by
    1/(W+1e-6) on near-empty pixels, and 6-sigma tails (weight o*e^-18) break the 1e-4 bar; at
    7 sigma (o*e^-24.5) the error is <1e-6.  One zone here (core = cutoff)."""
    d = golden("f2_c1_view3")
    r6 = _run(d, binned=True, cutoff=6.0, core=0.0)
    r7 = _run(d, binned=True, cutoff=7.0, core=0.0)
    assert orc.rel_l2(r6["d_means"], d["d_means"]) > 1e-4
    assert orc.rel_l2(r7["d_means"], d["d_means"]) < 2e-6


@pytest.mark.parametrize("depth", [True, False])
@pytest.mark.parametrize("name", ["f1_n300_64x48", "f1_n64_32x32_sh", "f2_c1_view0", "f2_c1_view3"])
def test_two_zone_core_radius(name, depth):
    """Why the core radius is 5.5 sigma: colour channels (and, without an upstream depth gradient, the
    whole backward) are cut at the core; the dropped tail weighs <= o*e^-15.1 per pixel.  Against the
    exact dense answer (float64) the two-zone result stays within 1e-5 at 5.5 sigma on every tensor;
    at 4.5 sigma the C1 scene without depth gradients is past 1e-4."""
    d = golden(name)
    exact = _run(d, binned=False, depth=depth)
    r = _run(d, binned=True, core=5.5, depth=depth)
    for k in KEYS:
        assert orc.rel_l2(r[k], exact[k]) <= 1e-5, k
    if name.startswith("f2") and not depth:
        r45 = _run(d, binned=True, core=4.5, depth=depth)
        assert max(orc.rel_l2(r45[k], exact[k]) for k in KEYS) > 1e-4


@pytest.mark.parametrize("name", golden_names("u8_"))
def test_u8_restatement_bit_exact(name):
    d = golden(name)
    sc = orc.Scene(d["means"], d["scales"], d["colors"], d["opacities"])
    out = orc.render_u8(int(d["width"]), int(d["height"]), d["view"], d["proj"], sc, d["background"], int(d["sort"]))
    np.testing.assert_array_equal(out, d["rgba"])


def test_binning_is_stable_and_consistent():
    sc = orc.synthetic_scene(3000, seed=9, scale=0.05)
    view, proj = orc.orbit_cameras(5, 160, 96)[3]
    v = orc.make_view(view, proj, 160, 96, cutoff=CUTOFF, core_cutoff=CORE)
    rec, rect, counts = orc.preprocess(v, sc)
    offsets, keys, vals, ranges = orc.bin_pairs(v, rec, rect, counts)
    assert offsets[-1] == counts.sum() == len(vals)
    assert np.all(np.diff(keys.astype(np.int64)) >= 0)  # sorted by virtual tile (2 * tile + tail)
    assert 0 < np.count_nonzero(keys & 1) < len(keys)  # both zones present
    for t in range(ranges.shape[0]):
        seg = vals[ranges[t, 0]:ranges[t, 1]]
        assert np.all(np.diff(seg) > 0)  # Gaussian-index order inside a tile (stable)
    # every pair's tile lies in its Gaussian's rectangle; culling keeps at most the rectangle
    assert np.all(counts <= (rect[:, 2] - rect[:, 0] + 1) * (rect[:, 3] - rect[:, 1] + 1))
    r = rect[vals]
    tx, ty = (keys >> 1) % 10, (keys >> 1) // 10
    assert np.all((tx >= r[:, 0]) & (tx <= r[:, 2]) & (ty >= r[:, 1]) & (ty <= r[:, 3]))


def test_camera_helpers_match_golden_views():
    d = golden("f2_c1_view1")
    view, proj = orc.orbit_cameras(4, 128, 128)[1]
    np.testing.assert_array_equal(view, d["view"])
    np.testing.assert_array_equal(proj, d["proj"])
