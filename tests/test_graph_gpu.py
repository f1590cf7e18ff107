"""GPU: device-side sizing (gr_fwd_prepare_views_sized, gr_view.device_counts) and the fit step captured once as a HIP
graph and replayed (fit_multiview.GRAPH, ViewShardedFitter._graph_step).

* test_sized_view_matches_host_sized: one view prepared against capacities (the counts stay on the device) through the
  fused fit path (32-pixel tiles) and through the depth-loss path (two zones, 16-pixel tiles) gives bit-identical
  losses and per-Gaussian sums to the host-sized view; with capacities below the counts the overflow word is raised,
  the true counts still reach the observed plan, and the view renders as one without pairs (every sum zero).
* test_graph_steps_bit_identical_to_eager: steps replayed from the graph (the first step eager, the second captures)
  leave bit-identical parameters, Adam moments, gradients and losses to the same steps run eagerly, with and without
  the depth term, and across an in-place Morton re-sort.
* test_graph_overflow_and_redo: capacities forced below the counts at capture: the replayed step overflows, updates
  nothing, and is redone with grown capacities; the fit stays bit-identical to the eager one.
* test_batched_steps_bit_identical_to_eager: the views' kernels launched once per batch of up to 8 views
  (gr_fit_views_batched, GR_GRAPH=batch, and that step captured, batchgraph) give the eager schedule's parameters,
  moments, gradients and losses bit for bit (every block computes what it computes in its own view's launch; the chain
  rules run in the single-stream schedule's grouping without its tail batch), for the fit path at 32- and 16-pixel tiles and the depth loss.
"""
from __future__ import annotations

import importlib

import pytest
import torch

pytestmark = pytest.mark.gpu


def _scene(bench, fm, cuda, n, views, W, H, depth=False, sh=False, seed=3):
    params = bench.synthetic_params(n, cuda)
    if sh:
        g = torch.Generator().manual_seed(2)
        shc = torch.zeros((n, 16, 3))
        shc[:, 0, :] = torch.sigmoid(0.1 * torch.rand((n, 3), generator=g))
        shc[:, 1:, :] = 0.02 * torch.randn((n, 15, 3), generator=g)
        del params["colors_raw"]
        params["sh_raw"] = torch.nn.Parameter(shc.to(cuda))
    cams = fm.orbit_cameras(views, W, H, cuda)
    g = torch.Generator(device=cuda).manual_seed(seed)
    targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in range(views)]
    masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
    depths = [torch.rand((H, W), generator=g, device=cuda) for _ in range(views)] if depth else None
    return params, cams, targets, masks, depths


@pytest.mark.parametrize("mode", ["fit32", "depth16"])
def test_sized_view_matches_host_sized(cuda, mode):
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    tr = importlib.import_module("3dgaussian_amd.torch_renderer")
    bench = importlib.import_module("bench")
    W, H = 256, 192
    params, cams, targets, masks, depths = _scene(bench, fm, cuda, 60_000, 1, W, H, depth=True)
    m, s, c, o = (t.detach().float().contiguous() for t in fm.activations(params))
    if mode == "fit32":
        gv = tr.make_view(cams[0].view, cams[0].proj, W, H, None, cutoff=tr.FIT_CUTOFF, core_cutoff=tr.FIT_CUTOFF,
                          depth_grad=False, tile=32)
    else:
        gv = tr.make_view(cams[0].view, cams[0].proj, W, H, None, depth_grad=True)

    def run(prep):
        loss = torch.zeros(1, device=cuda)
        if mode == "fit32":
            st, ws = tr.forward_l1_native(m, s, c, o, prep.gv, prep, targets[0], masks[0], 0.2, 0.5, loss)
            tr.backward_splat_native(st, ws)
            sums, sums3 = tr.gather_view_native(st, ws), None
        else:
            _, _, _, st = tr.forward_native(m, s, c, o, prep.gv, prep, images=False)
            sums, sums3 = tr.backward_fit_gather_native(st, targets[0], masks[0], 0.2, depths[0], 0.05, 0.5, loss)
        torch.cuda.synchronize()
        return float(loss), sums, sums3

    pin = torch.zeros(3, dtype=torch.int64, pin_memory=True)
    (ph,) = tr.prepare_views_native(m, s, c, o, [gv], [pin])
    ref = run(ph)
    K, _, Kc = (int(x) for x in pin.tolist())
    assert K > 0
    obs = torch.zeros(3, dtype=torch.int64, pin_memory=True)
    ovf = torch.zeros(1, dtype=torch.int32, device=cuda)
    caps = tr._native.GrPlan(K + (K - Kc) + 70_000, K + (K - Kc) + 70_000, Kc + 50_000)  # roomy, uneven
    (pz,) = tr.prepare_views_sized(m, s, c, o, [tr.sized_view(gv)], [caps], [obs], ovf)
    got = run(pz)
    assert int(ovf.item()) == 0
    assert [int(x) for x in obs.tolist()] == [K, K, Kc]
    assert got[0] == ref[0]
    assert torch.equal(got[1], ref[1])
    if ref[2] is not None:
        assert torch.equal(got[2], ref[2])
    print(f"{mode}: {K} pairs ({Kc} core), sized view bit-identical")
    # capacities below the counts: the overflow word, the true counts observed, a view without pairs
    small = tr._native.GrPlan(Kc // 2 + (K - Kc), Kc // 2 + (K - Kc), Kc // 2)
    obs.zero_()
    (pz,) = tr.prepare_views_sized(m, s, c, o, [tr.sized_view(gv)], [small], [obs], ovf)
    over = run(pz)
    assert int(ovf.item()) == 1
    assert [int(x) for x in obs.tolist()] == [K, K, Kc]
    assert float(over[1].abs().sum()) == 0.0
    assert over[0] > 0.0 and torch.isfinite(torch.tensor(over[0]))


def _set_mode(fm, mode):
    """fit_multiview's GR_GRAPH mode ("0", "1", "sized", "exec", "batch", "batchgraph", "auto")."""
    fm.GRAPH_MODE = mode


def _run(fm, params_fn, cams, targets, masks, depths, W, H, steps, graph, resort=0):
    saved = fm.GRAPH_MODE, fm.RESORT_EVERY
    _set_mode(fm, graph if isinstance(graph, str) else ("1" if graph else "0"))
    fm.RESORT_EVERY = resort
    try:
        f = fm.ViewShardedFitter(params_fn(), cams, targets, W, H, lr=0.02, masks=masks, depths=depths)
        losses = [f.step() for _ in range(steps)]
        f.graph_sync()
        torch.cuda.synchronize()
        out = {k: v.detach().clone() for k, v in f.params.items()}
        mom = {k: (f.opt.state[v]["exp_avg"].clone(), f.opt.state[v]["exp_avg_sq"].clone(), float(f.opt.state[v]["step"]))
               for k, v in f.params.items()}
        grads = {k: v.grad.detach().clone() for k, v in f.params.items()}
        gs = getattr(f, "_gs", None)
        return [float(x) for x in losses], out, mom, grads, f.perm.clone() if f.perm is not None else None, gs
    finally:
        _set_mode(fm, saved[0])
        fm.RESORT_EVERY = saved[1]


def _assert_same(a, b):
    la, pa, ma, ga, perm_a, _ = a
    lb, pb, mb, gb, perm_b, _ = b
    assert la == lb, (la, lb)
    for k in pa:
        assert torch.equal(pa[k], pb[k]), k
        assert torch.equal(ga[k], gb[k]), k
        assert torch.equal(ma[k][0], mb[k][0]) and torch.equal(ma[k][1], mb[k][1]) and ma[k][2] == mb[k][2], k
    assert (perm_a is None) == (perm_b is None) and (perm_a is None or torch.equal(perm_a, perm_b))


@pytest.mark.parametrize("case", ["fit", "depth_sh3", "fit_resort"])
def test_graph_steps_bit_identical_to_eager(cuda, case):
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W, H = 192, 160
    depth = case == "depth_sh3"
    _, cams, targets, masks, depths = _scene(bench, fm, cuda, 40_000, 5, W, H, depth=depth, sh=depth)

    def params_fn():
        return _scene(bench, fm, cuda, 40_000, 5, W, H, depth=depth, sh=depth)[0]

    resort = 2 if case == "fit_resort" else 0
    eager = _run(fm, params_fn, cams, targets, masks, depths, W, H, 6, False, resort)
    graph = _run(fm, params_fn, cams, targets, masks, depths, W, H, 6, True, resort)
    gs = graph[5]
    assert gs is not None and gs.graph is not None and gs.overflows == 0  # replayed, no redo
    _assert_same(eager, graph)
    print(f"{case}: 6 steps, graph replays bit-identical to eager; losses {graph[0]}")


def test_graph_overflow_and_redo(cuda, monkeypatch):
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W, H = 192, 160
    _, cams, targets, masks, depths = _scene(bench, fm, cuda, 40_000, 4, W, H)

    def params_fn():
        return _scene(bench, fm, cuda, 40_000, 4, W, H)[0]

    eager = _run(fm, params_fn, cams, targets, masks, depths, W, H, 6, False)
    real = fm.ViewShardedFitter._caps_of
    calls = []

    def short_caps(counts, old=None):
        calls.append(old is None)
        if old is None:  # the first capture: capacities at 60% of the probed counts (every view overflows)
            return [tr_plan(int(0.6 * k), int(0.6 * kc)) for k, _, kc in counts]
        return real(counts, old)

    tr = importlib.import_module("3dgaussian_amd.torch_renderer")

    def tr_plan(k, kc):
        return tr._native.GrPlan(k, k, kc)

    monkeypatch.setattr(fm.ViewShardedFitter, "_caps_of", staticmethod(short_caps))
    graph = _run(fm, params_fn, cams, targets, masks, depths, W, H, 6, True)
    gs = graph[5]
    assert gs.overflows >= 1 and calls[0] and not all(calls)
    _assert_same(eager, graph)
    print(f"overflow and redo: {gs.overflows} redo(s), capacities grown to "
          f"{[int(c.num_pairs) for c in gs.caps]}; bit-identical to eager")


@pytest.mark.parametrize("case", ["fit32", "fit16", "depth_sh3", "fit32_graph", "depth_graph"])
def test_batched_steps_bit_identical_to_eager(cuda, case, monkeypatch):
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    W, H = 192, 160
    depth = case.startswith("depth")
    if case == "fit16":
        monkeypatch.setattr(fm, "FIT_TILE", 16)
    V = 11  # two batches of views (8 + 3), three streams' reduction groupings
    _, cams, targets, masks, depths = _scene(bench, fm, cuda, 40_000, V, W, H, depth=depth, sh=depth)

    def params_fn():
        return _scene(bench, fm, cuda, 40_000, V, W, H, depth=depth, sh=depth)[0]

    # the batched step reduces in the single-stream schedule's grouping, without the short tail batch
    monkeypatch.setattr(fm, "NUM_STREAMS", 1)
    monkeypatch.setattr(fm, "REDUCE_TAIL", 0)
    eager = _run(fm, params_fn, cams, targets, masks, depths, W, H, 5, False)
    batched = _run(fm, params_fn, cams, targets, masks, depths, W, H, 5, "batchgraph" if case.endswith("graph") else "batch")
    assert batched[5] is not None and batched[5].overflows == 0
    _assert_same(eager, batched)
    print(f"{case}: 5 steps of {V} views batched, bit-identical to eager; losses {batched[0]}")


@pytest.mark.parametrize("world", [5, 8])
@pytest.mark.parametrize("schedule", ["python", "native"])
def test_band_split_adds_up_to_the_views(cuda, world, schedule, monkeypatch):
    """Multi-GPU view sharding with the leftover views cut into bands of tile rows (BAND_SPLIT, gr_view.row0 / rows;
    round 6: the ranks in one group per leftover view, one band per rank): every emulated rank's loss and gradient (this
    process playing each rank in turn, no collective) sum to the single-process step's, within float summation order;
    each band renders only its rows (a band's pairs are those of its tile rows).  11 views: 5 ranks cut view 10 in
    five bands; 8 ranks cut views 8, 9, 10 over groups of 2, 3 and 3."""
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    bench = importlib.import_module("bench")
    monkeypatch.setattr(fm, "BAND_OVERHEAD", 0.0)  # bands whatever they cost
    W, H, V = 256, 224, 11  # 7 tile rows of 32 pixels
    params, cams, targets, masks, _ = _scene(bench, fm, cuda, 50_000, V, W, H)
    f = fm.ViewShardedFitter(params, cams, targets, W, H, lr=0.02, masks=masks)
    acts = [a.detach().float().contiguous() for a in fm.activations(f.params)]

    def run():
        with torch.no_grad():
            if schedule == "native":
                total = f._views_native(*acts, False)
            else:
                total, _ = f._views_direct(*acts)
            parts = f._acc_parts
            acc = [sum(p[q] for p in parts[1:]) + parts[0][q] if len(parts) > 1 else parts[0][q].clone() for q in range(4)]
        torch.cuda.synchronize()
        return float(total), acc

    ref_loss, ref = run()
    tot_loss, tot = 0.0, [torch.zeros_like(a) for a in ref]
    seen = []
    for r in range(world):
        f.rank, f.world = r, world
        f._rr_views = list(range(r, V, world))
        views = f.my_views
        assert len([v for v in views if v >= V]) == 1  # one band per rank (7 tile rows >= every group's size)
        seen += views
        loss, acc = run()
        tot_loss += loss
        tot = [a + b for a, b in zip(tot, acc)]
    f.rank, f.world = 0, 1
    assert sorted(v for v in seen if v < V) == list(range(V - V % world))
    assert abs(tot_loss - ref_loss) <= 1e-6 * abs(ref_loss), (tot_loss, ref_loss)
    for k, (a, b) in enumerate(zip(tot, ref)):
        err = float((a - b).norm() / b.norm())
        assert err <= 1e-5, (k, err)
    print(f"world {world} ({schedule}): bands of views {list(range(V - V % world, V))} add up: loss {tot_loss:.7f} "
          f"vs {ref_loss:.7f}")
