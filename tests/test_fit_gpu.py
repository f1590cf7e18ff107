"""GPU: the fit driver (3dgaussian_amd/fit_multiview.py, HIP render op) reproduces the loss curve
of the reference's unchanged fit_multiview_stub.py (golden F4: torch.manual_seed(1234), 300
Gaussians, 48x48, 3 synthetic targets, 6 iterations with densify/prune every 3)."""
from __future__ import annotations

import importlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden

pytestmark = pytest.mark.gpu


def test_fit_curve_matches_reference_stub(tmp_path, cuda):
    d = golden("f4_fit_curve")
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    fm.main(["--targets_dir", os.path.join(GOLDEN, "fit_targets"), "--out_dir", str(tmp_path), "--iters", str(int(d["iters"])),
             "--width", str(int(d["width"])), "--height", str(int(d["width"])), "--num_gaussians", str(int(d["num_gaussians"])),
             "--max_gaussians", str(int(d["max_gaussians"])), "--densify_interval", str(int(d["densify_interval"])),
             "--prune_interval", str(int(d["densify_interval"])), "--seed", str(int(d["seed"]))])
    losses = np.array([float(x) for x in (tmp_path / "loss.txt").read_text().split()])
    np.testing.assert_allclose(losses, d["losses"], rtol=1e-4)
    npz = np.load(tmp_path / "gaussians_fitted.npz")
    assert set(npz.files) == {"means", "scales", "colors", "opacities"}
    assert (tmp_path / "preview_view0.png").exists()


def test_streams_and_precision_mode_do_not_change_the_step(cuda):
    """The fit driver's multi-stream rotation and its depth_grad=False forward/backward give the same
    parameters after a step as one stream with the default (f32-grade) precision, within the
    two-piece mode's error."""
    import torch

    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W = H = 128
    cams = fm.orbit_cameras(6, W, H, cuda)
    g = torch.Generator(device=cuda).manual_seed(3)
    targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in cams]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]

    def one_step(streams):
        saved = fm.NUM_STREAMS
        fm.NUM_STREAMS = streams
        try:
            params = bench.synthetic_params(20_000, cuda)
            f = fm.ViewShardedFitter(params, cams, targets, W, H, masks=masks)
            loss = float(f.step())
            grads = {k: v.grad.detach().clone() for k, v in f.params.items()}
        finally:
            fm.NUM_STREAMS = saved
        return loss, grads

    l1, g1 = one_step(1)
    l3, g3 = one_step(3)
    l3b, g3b = one_step(3)
    assert abs(l1 - l3) <= 1e-6 * abs(l1)
    for k in g1:
        # one accumulator per stream: the views' gradients are summed in another order with 3 streams
        torch.testing.assert_close(g3[k], g1[k], rtol=1e-5, atol=1e-6 * float(g1[k].abs().max())), k
        assert torch.equal(g3[k], g3b[k]), k  # deterministic for a given stream count
    assert l3 == l3b


@pytest.mark.parametrize("sh", [False, True])
def test_direct_path_matches_autograd_path(cuda, sh):
    """The fused fit path (gr_bwd_l1: L1 + silhouette loss and render backward in one pass, gradients
    accumulated per stream, one autograd pass through the activations) gives the loss and gradients
    of the autograd path (per-view autograd: l1_loss -> gr_bwd -> autograd's gradient sums)."""
    import torch

    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W, H = 160, 128
    cams = fm.orbit_cameras(7, W, H, cuda)
    g = torch.Generator(device=cuda).manual_seed(4)
    targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in cams]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]

    def one_step(direct):
        saved = fm.DIRECT_BACKWARD
        fm.DIRECT_BACKWARD = direct
        try:
            params = bench.synthetic_params(30_000, cuda)
            if sh:
                shc = torch.zeros((30_000, 4, 3), device=cuda)
                shc[:, 0, :] = torch.sigmoid(params.pop("colors_raw").detach())
                gs = torch.Generator(device=cuda).manual_seed(5)  # the same coefficients for both paths
                shc[:, 1:, :] = 0.05 * torch.randn((30_000, 3, 3), generator=gs, device=cuda)
                params["sh_raw"] = torch.nn.Parameter(shc)
            f = fm.ViewShardedFitter(params, cams, targets, W, H, masks=masks)
            loss = float(f.step())
            grads = {k: v.grad.detach().clone() for k, v in f.params.items()}
        finally:
            fm.DIRECT_BACKWARD = saved
        return loss, grads

    la, ga = one_step(False)
    ld, gd = one_step(True)
    assert abs(la - ld) <= 1e-6 * abs(la)
    for k in ga:
        # the two paths bin with different footprints (fused path: one FIT_CUTOFF zone; autograd path:
        # 7 / 5.5 sigma): each is within the parity bar of the dense reference, so of each other
        err = float((gd[k] - ga[k]).norm() / ga[k].norm())
        assert err <= 1e-4, (k, err)


def test_batched_reduce_matches_per_view_reduce(cuda):
    """The fused fit path's calls (gr_fwd_render_l1, gr_bwd_splat, gr_gather_view + gr_reduce_sums or
    gr_reduce_views) against gr_fwd_render + gr_bwd_l1 per view: the same view losses bit for bit, a one-view
    two-stage batch the per-view gradient exactly (gr_reduce_views within summation order), a batch the sum of the per-view gradients within float summation order; the fit
    step is the same for every REDUCE_BATCH and deterministic for each."""
    import torch

    tr = importlib.import_module("3dgaussian_amd.torch_renderer")
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W, H = 144, 112
    n = 25_000
    cams = fm.orbit_cameras(5, W, H, cuda)
    g = torch.Generator(device=cuda).manual_seed(6)
    targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in cams]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    p = bench.synthetic_params(n, cuda)
    m, s, c, o = (t.detach().contiguous() for t in fm.activations(p))
    per_view, batch = [], []
    loss = torch.zeros(len(cams), device=cuda)
    loss2 = torch.zeros(len(cams), device=cuda)
    for i, cam in enumerate(cams):
        gv = tr.make_view(cam.view, cam.proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF, depth_grad=False)
        _, _, _, st = tr.forward_native(m, s, c, o, gv, want_depth=False)
        grads = tuple(torch.empty_like(t) for t in (m, s, c, o))
        tr.backward_l1_native(m, s, c, o, st, targets[i], masks[i], 0.2, 0.25, loss[i:i + 1], grads, accumulate=False)
        per_view.append(grads)
        prep = tr.prepare_native(m, s, c, o, gv)
        st2, ws = tr.forward_l1_native(m, s, c, o, gv, prep, targets[i], masks[i], 0.2, 0.25, loss2[i:i + 1])
        tr.backward_splat_native(st2, ws)
        batch.append((st2, ws))
    assert torch.equal(loss, loss2)  # the forward-epilogue loss is the backward's (same per-tile sums)
    one = tuple(torch.empty_like(t) for t in (m, s, c, o))
    # the per-view backward reduces through the same two stages (gather + chain rule of one view): exact
    tr.reduce_sums_native(m, s, c, o, [(batch[0][0].gv, tr.gather_view_native(*batch[0]))], one, accumulate=False)
    for a, b in zip(one, per_view[0]):
        assert torch.equal(a, b)
    # the one-pass gr_reduce_views (f64 row sums) within float summation order
    tr.reduce_views_native(m, s, c, o, batch[:1], one, accumulate=False)
    for a, b in zip(one, per_view[0]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6 * float(b.abs().max()))
    # two-stage batches of 1..5 views (k_reduce_sums groups a Gaussian's views over 1, 2 or 4 waves by the
    # batch size) against the sum of the per-view gradients
    sums = [(st.gv, tr.gather_view_native(st, ws)) for st, ws in batch]
    for k in range(1, len(batch) + 1):
        got = tuple(torch.empty_like(t) for t in (m, s, c, o))
        tr.reduce_sums_native(m, s, c, o, sums[:k], got, accumulate=False)
        for q in range(4):
            ref = sum(pv[q] for pv in per_view[:k])
            torch.testing.assert_close(got[q], ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max()))
    tot = tuple(torch.empty_like(t) for t in (m, s, c, o))
    tr.reduce_views_native(m, s, c, o, batch, tot, accumulate=False)
    tr.reduce_views_native(m, s, c, o, batch[:2], tot, accumulate=True)  # accumulate adds
    for q in range(4):
        ref = sum(pv[q] for pv in per_view) + per_view[0][q] + per_view[1][q]
        torch.testing.assert_close(tot[q], ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max()))

    def one_step(rb):
        saved = fm.REDUCE_BATCH
        fm.REDUCE_BATCH = rb
        try:
            f = fm.ViewShardedFitter(bench.synthetic_params(n, cuda), cams, targets, W, H, masks=masks)
            lv = float(f.step())
            return lv, {k: v.grad.detach().clone() for k, v in f.params.items()}
        finally:
            fm.REDUCE_BATCH = saved

    l1, g1 = one_step(1)
    for rb in (2, 8, 8):
        lb, gb = one_step(rb)
        assert lb == l1
        for k in g1:
            torch.testing.assert_close(gb[k], g1[k], rtol=1e-5, atol=1e-6 * float(g1[k].abs().max())), k
    _, g8 = one_step(8)
    _, g8b = one_step(8)
    for k in g8:
        assert torch.equal(g8[k], g8b[k]), k


@pytest.mark.parametrize("sh", [False, True])
def test_direct_depth_path_matches_autograd_path(cuda, sh):
    """The fused path with the depth term (gr_bwd_fit: L1 + silhouette + depth loss
    w_depth mean|depth / (max depth + 1e-6) - t| and the render backward, gradients accumulated per stream)
    gives the loss and gradients of the autograd path (torch ops for the loss, gr_bwd, autograd sums)."""
    import torch

    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W, H = 96, 80
    cams = fm.orbit_cameras(5, W, H, cuda)
    g = torch.Generator(device=cuda).manual_seed(7)
    targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in cams]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    depths = [torch.rand((H, W), generator=g, device=cuda) for _ in cams]

    def one_step(direct):
        saved = fm.DIRECT_BACKWARD
        fm.DIRECT_BACKWARD = direct
        try:
            params = bench.synthetic_params(8000, cuda)
            if sh:
                shc = torch.zeros((8000, 16, 3), device=cuda)
                shc[:, 0, :] = torch.sigmoid(params.pop("colors_raw").detach())
                gs = torch.Generator(device=cuda).manual_seed(5)
                shc[:, 1:, :] = 0.03 * torch.randn((8000, 15, 3), generator=gs, device=cuda)
                params["sh_raw"] = torch.nn.Parameter(shc)
            f = fm.ViewShardedFitter(params, cams, targets, W, H, masks=masks, depths=depths)
            loss = float(f.step())
            grads = {k: v.grad.detach().clone() for k, v in f.params.items()}
        finally:
            fm.DIRECT_BACKWARD = saved
        return loss, grads

    la, ga = one_step(False)
    ld, gd = one_step(True)
    assert abs(la - ld) <= 2e-6 * abs(la)
    for k in ga:
        err = float((gd[k] - ga[k]).norm() / ga[k].norm())
        assert err <= 1e-5, (k, err)


@pytest.mark.parametrize("path", ["python", "native", "autograd"])
@pytest.mark.parametrize("with_depth", [False, True])
def test_fit_loss_value_vs_torch_loss_many_tiles(cuda, path, with_depth):
    """The fit step's loss value (the fused paths' device loss: gr_fwd_render_l1 / gr_bwd_fit_gather's
    tile sums finished by the last tile, k_pixel_grads with a depth target) against the stub's torch loss
    (fit_multiview_stub.py:293-308) on the drop-in op's images, at 320x320 = 400 tiles: more than the 256
    threads of the last tile's reduction (its scratch was 1 KiB short past 128 tiles)."""
    import torch

    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W = H = 320
    cams = fm.orbit_cameras(3, W, H, cuda)
    g = torch.Generator(device=cuda).manual_seed(11)
    targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in cams]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    depths = [torch.rand((H, W), generator=g, device=cuda) for _ in cams] if with_depth else None
    saved = (fm.DIRECT_BACKWARD, fm.NATIVE_EXEC)
    fm.DIRECT_BACKWARD = path != "autograd"
    fm.NATIVE_EXEC = "1" if path == "native" else "0"
    try:
        f = fm.ViewShardedFitter(bench.synthetic_params(40_000, cuda), cams, targets, W, H, masks=masks, depths=depths)
        with torch.no_grad():
            m, s, c, o = fm.activations(f.params)
            ref = 0.0
            for i, cam in enumerate(cams):
                pred, alpha, depth = fm.hip_render(m, s, c, o, cam, W, H, f._background(cuda))
                li = torch.mean(torch.abs(pred - targets[i])) + f.w_sil * torch.mean(torch.abs(alpha - masks[i]))
                if with_depth:
                    li = li + f.w_depth * torch.mean(torch.abs(depth / (depth.max() + 1e-6) - depths[i]))
                ref += float(li)
            ref = ref / len(cams) + float(f.reg_opacity * o.mean() + f.reg_scale * s.mean())
        loss = float(f.step())
    finally:
        fm.DIRECT_BACKWARD, fm.NATIVE_EXEC = saved
    print(f"loss {loss:.8f} torch {ref:.8f} rel {abs(loss - ref) / ref:.2e}")
    assert abs(loss - ref) <= 1e-5 * abs(ref), (loss, ref)


def test_fused_param_step_matches_torch_adam(cuda):
    """gr_fit_param_step (gradients through the activations + regulariser, Adam's update) against torch's
    autograd + torch.optim.Adam on the same views, over three steps (Adam's bias corrections move)."""
    import torch

    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W, H = 128, 96
    cams = fm.orbit_cameras(4, W, H, cuda)
    g = torch.Generator(device=cuda).manual_seed(9)
    targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in cams]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]

    def run(fused):
        saved = fm.FUSED_STEP
        fm.FUSED_STEP = fused
        try:
            f = fm.ViewShardedFitter(bench.synthetic_params(20_000, cuda), cams, targets, W, H, masks=masks)
            losses = [float(f.step()) for _ in range(3)]
            return losses, {k: v.detach().clone() for k, v in f.params.items()}
        finally:
            fm.FUSED_STEP = saved

    la, pa = run(False)
    lf, pf = run(True)
    np.testing.assert_allclose(lf, la, rtol=2e-6)
    for k in pa:
        err = float((pf[k] - pa[k]).norm() / pa[k].norm())
        assert err <= 1e-6, (k, err)


@pytest.mark.parametrize("sh", [False, True])
def test_grouped_prepare_matches_single_view_prepare(cuda, sh):
    """gr_fwd_prepare_views_async (parameters read once for up to 8 views) writes, per view, exactly the geom
    workspace (records, depths, rectangles, counts, the pair totals, plan) and the pinned-host plan that
    gr_fwd_prepare_async writes for that view alone (the Gaussians' offsets are the binning's: k_emit_cols)."""
    import torch

    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    tr = importlib.import_module("3dgaussian_amd.torch_renderer")
    bench = importlib.import_module("bench")
    W, H = 160, 120
    params = bench.synthetic_params(30_000, cuda)
    if sh:
        g = torch.Generator(device=cuda).manual_seed(4)
        params["sh_raw"] = torch.nn.Parameter(0.1 * torch.randn((30_000, 16, 3), generator=g, device=cuda))
        del params["colors_raw"]
    with torch.no_grad():
        acts = [a.contiguous() for a in fm.activations(params)]
    cams = fm.orbit_cameras(8, W, H, cuda)
    gvs = [tr.make_view(c.view, c.proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF, depth_grad=False)
           for c in cams]
    pins = torch.zeros((16, 3), dtype=torch.int64, pin_memory=True)
    for k in (8, 5, 4, 3, 2):
        grouped = tr.prepare_views_native(*acts, gvs[:k], [pins[q] for q in range(k)])
        single = [tr.prepare_native(*acts, gv, plan_host=pins[8 + q]) for q, gv in enumerate(gvs[:k])]
        for q, (a, b) in enumerate(zip(grouped, single)):
            pa, pb = a.plan(), b.plan()
            assert (pa.num_pairs, pa.num_slots, pa.num_core_pairs) == (pb.num_pairs, pb.num_slots, pb.num_core_pairs)
            assert pa.num_pairs > 0
            n = acts[0].shape[0]
            off = tr._native.geom_layout(n)
            parts = [(off[0], (n + 1) * 36), (off[1], n * 16), (off[2], (n + 1) * 8), (off[3] + 8 * n, 8),
                     (off[4], 24 + ((n + 256) // 256) * 8)]  # records + depths, rects, counts, totals, plan + block scan
            for o, nb in parts:
                assert torch.equal(a.geom[o:o + nb], b.geom[o:o + nb]), (k, q, o)


def test_binning_on_another_stream_is_exact(cuda):
    """gr_fwd_bin on a second stream followed by the splat with gr_view.binned = 1 (the drop-in op's
    speculative binning, torch_renderer._bin_ahead) gives bit-identical outputs and saved sums to the one-call
    gr_fwd_render, in the default and the no-depth-gradient modes."""
    import torch

    tr = importlib.import_module("3dgaussian_amd.torch_renderer")
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W, H = 160, 120
    p = bench.synthetic_params(20_000, cuda)
    m, s, c, o = (t.detach().contiguous() for t in fm.activations(p))
    cam = fm.orbit_cameras(3, W, H, cuda)[1]
    side = torch.cuda.Stream(cuda)
    for depth_grad in (True, False):
        gv = tr.make_view(cam.view, cam.proj, W, H, None, depth_grad=depth_grad)
        res = []
        for bs in (None, side):
            prep = tr.prepare_native(m, s, c, o, gv)
            out, alpha, depth, st = tr.forward_native(m, s, c, o, gv, prep, bin_stream=bs)
            torch.cuda.synchronize()
            res.append((out.clone(), alpha.clone(), depth.clone(), st.saved.clone()))
        for a, b in zip(*res):
            assert torch.equal(a, b), depth_grad
