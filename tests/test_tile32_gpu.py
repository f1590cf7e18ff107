"""GPU: 32-pixel tiles (gr_view.tile = 32), the fused fit path's binning and splats (k_fwd32_l1, k_bwd32).

* the integer binning is bit-exact against the oracle's binned semantics at the same tile size (rectangles, counts,
  per-tile pair lists with their emission indices), on ragged images whose edges cut tiles;
* one view through the fused path (gr_fwd_render_l1 -> gr_bwd_splat -> gr_gather_view -> gr_reduce_sums) against
  the float64 binned oracle at tile 32 with the same L1 upstream (the HIP images' signs at the kink, as
  test_chain_gpu.py): images, loss and all four gradients;
* the 32- and 16-pixel fused paths against each other (each is within the footprint error of the dense reference).
"""
from __future__ import annotations

import importlib

import numpy as np
import pytest
import torch

from oracle import oracle as orc

pytestmark = pytest.mark.gpu

CASES = {
    # name: (n, W, H, camera index, seed, scale)
    "c2_512": (100_000, 512, 512, 5, 3, None),
    "ragged_200x120_big_sigma": (2000, 200, 120, 1, 4, 0.4),
    "ragged_333x215": (30_000, 333, 215, 2, 5, None),
    "hd_1920x1080": (60_000, 1920, 1080, 3, 6, None),
}


def _setup(case, cuda):
    n, W, H, ci, seed, scale = CASES[case]
    sc = orc.synthetic_scene(n, seed=seed, scale=scale)
    view, proj = orc.orbit_cameras(8, W, H)[ci]
    t = [torch.from_numpy(a).to(cuda).contiguous() for a in sc.arrays()]
    return sc, view, proj, W, H, t


def _fused_view(tr, t, view, proj, W, H, tile, target, mask, w_sil, g_scale, cuda):
    """One view through the fused fit path at `tile`: (loss, out, alpha, grads, RenderState)."""
    gv = tr.make_view(view, proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF, depth_grad=False, tile=tile)
    prep = tr.prepare_native(*t, gv)
    loss = torch.zeros(1, device=cuda)
    out = torch.empty((H, W, 3), device=cuda)
    alpha = torch.empty((H, W), device=cuda)
    st, ws = tr.forward_l1_native(*t, gv, prep, target, mask, w_sil, g_scale, loss, out=out, alpha=alpha)
    tr.backward_splat_native(st, ws)
    sums = tr.gather_view_native(st, ws)
    grads = tuple(torch.empty_like(x) for x in t)
    tr.reduce_sums_native(*t, [(st.gv, sums)], grads, accumulate=False)
    torch.cuda.synchronize()
    return float(loss), out, alpha, grads, st


@pytest.mark.parametrize("case", list(CASES))
def test_bins_bit_exact_tile32(pkg, cuda, case):
    tr, nat = pkg.torch_renderer, pkg._native
    sc, view, proj, W, H, t = _setup(case, cuda)
    tgt = torch.zeros((H, W, 3), device=cuda)
    *_, st = _fused_view(tr, t, view, proj, W, H, 32, tgt, None, 0.0, 1.0, cuda)
    n = t[0].shape[0]
    g_off = nat.geom_layout(n)
    geom = st.geom.cpu().numpy()
    rect = geom[g_off[1]: g_off[1] + 16 * n].view(np.int32).reshape(n, 4)
    c64 = geom[g_off[2]: g_off[2] + 8 * n].view(np.uint64)
    core = (c64 & 0xFFFFFFFF).astype(np.int64)
    gv = st.gv
    K = st.num_pairs
    b_off = nat.bins_layout(gv, n, K)
    bins = st.bins.cpu().numpy()
    tiles = ((W + 31) // 32) * ((H + 31) // 32)
    ids = bins[b_off[1]: b_off[1] + 4 * K].view(np.int32)
    pos_of = bins[b_off[3]: b_off[3] + 4 * K].view(np.int32)
    emit = np.full(K, -1, np.int64)
    emit[pos_of] = np.arange(K)
    ranges = bins[b_off[2]: b_off[2] + 16 * tiles].view(np.int32).reshape(2 * tiles, 2)

    v = orc.make_view(view, proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF, tile=32)
    rec, orect, counts = orc.preprocess(v, sc)
    np.testing.assert_array_equal(core, counts)  # one zone: every kept pair is a core pair
    np.testing.assert_array_equal(rect[counts > 0], orect[counts > 0])
    _, keys, vals, oranges = orc.bin_pairs(v, rec, orect, counts)
    assert K == len(vals) and not (keys & 1).any()
    order = np.lexsort((keys >> 1, vals))
    oemit = np.empty(K, np.int64)
    oemit[order] = np.arange(K)
    lens = oranges[:, 1] - oranges[:, 0]
    np.testing.assert_array_equal(np.maximum(ranges[:, 1] - ranges[:, 0], 0), lens)
    for tt in np.nonzero(lens)[0]:
        a, b = ranges[tt]
        np.testing.assert_array_equal(ids[a:b], vals[oranges[tt, 0]:oranges[tt, 1]])
        np.testing.assert_array_equal(emit[a:b], oemit[oranges[tt, 0]:oranges[tt, 1]])
    v16 = orc.make_view(view, proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF)
    k16 = int(orc.preprocess(v16, sc)[2].sum())
    print(f"{case}: {K} pairs at 32-pixel tiles, {k16} at 16 ({K / max(k16, 1):.2f}x)")


@pytest.mark.parametrize("case", list(CASES))
def test_fused_view_tile32_vs_oracle(pkg, cuda, case):
    tr = pkg.torch_renderer
    sc, view, proj, W, H, t = _setup(case, cuda)
    g = torch.Generator(device=cuda).manual_seed(12)
    target = torch.rand((H, W, 3), generator=g, device=cuda)
    mask = (target.mean(dim=2) > 0.5).float().contiguous()
    w_sil, g_scale, HW = 0.2, 0.25, H * W
    loss, out, alpha, grads, _ = _fused_view(tr, t, view, proj, W, H, 32, target, mask, w_sil, g_scale, cuda)
    v = orc.make_view(view, proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF, tile=32)
    o_out, o_alpha, _ = orc.forward(v, sc, binned=True)
    h_out, h_alpha = out.cpu().numpy().astype(np.float64), alpha.cpu().numpy().astype(np.float64)
    tn, mn = target.cpu().numpy(), mask.cpu().numpy()
    o_loss = np.abs(o_out.astype(np.float64) - tn).mean() + w_sil * np.abs(o_alpha.astype(np.float64) - mn).mean()
    # upstream of the L1 kink from the HIP images' signs (near-ties depend on the last float bit)
    g_rgb = (np.sign(h_out - tn) * (g_scale / (3 * HW))).astype(np.float32)
    g_a = (np.sign(h_alpha - mn) * (w_sil * g_scale / HW)).astype(np.float32)
    ora = orc.backward(v, sc, g_rgb, g_a, None, binned=True)
    errs = {"out": orc.rel_l2(h_out, o_out), "alpha": orc.rel_l2(h_alpha, o_alpha), "loss": abs(loss - o_loss) / o_loss}
    for name, h, o in zip(("d_means", "d_scales", "d_colors", "d_opac"), grads, ora):
        h = h.cpu().numpy()
        if name == "d_scales":  # no z column in the render's scale gradient
            h, o = h[:, :2], o[:, :2]
        errs[name] = orc.rel_l2(h, o)
    print(f"{case} tile 32 fused view vs float64 binned oracle:", {k: f"{e:.2e}" for k, e in errs.items()})
    assert errs["out"] <= 2e-5 and errs["alpha"] <= 2e-5, errs
    assert errs["loss"] <= 1e-5, errs
    for k in ("d_means", "d_scales", "d_colors", "d_opac"):
        assert errs[k] <= 1e-4, (k, errs[k])


def test_tile32_vs_tile16_fused_path(pkg, cuda):
    """The same C2-size view at both tile sizes: the footprints differ (per-tile culling of the 5-sigma zone), each
    within the parity bar of the dense reference, so of each other."""
    tr = pkg.torch_renderer
    sc, view, proj, W, H, t = _setup("c2_512", cuda)
    g = torch.Generator(device=cuda).manual_seed(13)
    target = torch.rand((H, W, 3), generator=g, device=cuda)
    r16 = _fused_view(tr, t, view, proj, W, H, 16, target, None, 0.0, 1.0, cuda)
    r32 = _fused_view(tr, t, view, proj, W, H, 32, target, None, 0.0, 1.0, cuda)
    assert abs(r16[0] - r32[0]) <= 1e-5 * abs(r16[0])
    assert float((r16[1] - r32[1]).norm() / r16[1].norm()) <= 2e-5
    for a, b in zip(r16[3], r32[3]):
        assert float((a - b).norm() / a.norm()) <= 1e-4


def test_tile32_rejected_outside_fit_path(pkg, cuda):
    tr = pkg.torch_renderer
    sc, view, proj, W, H, t = _setup("ragged_333x215", cuda)
    gv = tr.make_view(view, proj, W, H, None, depth_grad=False, tile=32)  # two zones (7 / 5.5 sigma)
    with pytest.raises(ValueError, match="32-pixel tiles"):
        tr.forward_native(*t, gv, want_depth=False)
    gv.tile = 24
    with pytest.raises(ValueError, match="tile must be"):
        tr.prepare_native(*t, gv)


@pytest.mark.parametrize("opac_range", [(1e-4, 1e-3), (100.0, 3000.0), (3000.0, 6000.0), (0.0, 1e5), "mixed_negative"])
def test_tile32_f16_operand_range(pkg, cuda, opac_range):
    """k_fwd32_l1 multiplies on f16 pieces pre-scaled like k_raster_fwd_mfma<4> (f16_sa_of): tiny, huge and mixed
    large-negative / live opacities stay finite and within the parity bar vs the float64 binned oracle at tile 32."""
    from test_scale_gpu import _opacities

    tr = pkg.torch_renderer
    rng = np.random.default_rng(7)
    sc = orc.synthetic_scene(3000, seed=3, scale=0.05)
    sc = orc.Scene(sc.means, sc.scales, sc.colors, _opacities(rng, opac_range, sc.opacities.shape))
    view, proj = orc.orbit_cameras(4, 160, 120)[2]
    W, H = 160, 120
    t = [torch.from_numpy(a).to(cuda).contiguous() for a in sc.arrays()]
    g = torch.Generator(device=cuda).manual_seed(14)
    target = torch.rand((H, W, 3), generator=g, device=cuda)
    loss, out, alpha, grads, _ = _fused_view(tr, t, view, proj, W, H, 32, target, None, 0.0, 1.0, cuda)
    v = orc.make_view(view, proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF, tile=32)
    o_out, o_alpha, _ = orc.forward(v, sc, binned=True)
    h_out = out.cpu().numpy().astype(np.float64)
    g_rgb = (np.sign(h_out - target.cpu().numpy()) / (3 * H * W)).astype(np.float32)
    ora = orc.backward(v, sc, g_rgb, np.zeros((H, W), np.float32), None, binned=True)
    errs = {"out": orc.rel_l2(h_out, o_out), "alpha": orc.rel_l2(alpha.cpu().numpy(), o_alpha)}
    for name, h, o in zip(("d_means", "d_scales", "d_colors", "d_opac"), grads, ora):
        h = h.cpu().numpy()
        if name == "d_scales":
            h, o = h[:, :2], o[:, :2]
        errs[name] = orc.rel_l2(h, o)
    live = int((sc.opacities > 0).sum())
    print(f"opacities {opac_range}: {live} live;", {k: f"{e:.2e}" for k, e in errs.items()})
    assert live > 0 and np.isfinite(h_out).all() and float(np.abs(h_out).sum()) > 0.0
    for k, e in errs.items():
        assert e <= 1e-4, (k, e)
