"""GPU: gr_fit_param_steps (every parameter tensor's gradient and Adam update in one launch) gives exactly what one
gr_fit_param_step per tensor gives, for each activation and with one to three stream accumulators, on both of its
paths (float4 when the count is a multiple of 4 and every array 16-byte aligned, scalar otherwise)."""
from __future__ import annotations

import ctypes
import importlib

import pytest
import torch


@pytest.mark.gpu
def test_param_steps_equal_per_tensor_steps(pkg, cuda):
    nat = pkg._native
    L = nat.lib()
    # (count, activation, accumulators, regulariser, element offset of every array): identity / softplus / sigmoid,
    # sizes across block boundaries; offset 1 misaligns a count that is a multiple of 4 (the scalar path)
    specs = [(3 * 1000, 0, 3, 0.0, 0), (3 * 777, 1, 2, 1e-4, 0), (1_000_003, 2, 1, 2e-6, 0), (255, 2, 0, 0.0, 0),
             (4_000_000, 1, 3, 1e-5, 0), (4096, 2, 2, 0.0, 1), (48 * 50_000, 0, 1, 0.0, 0)]
    b1, b2, eps = 0.9, 0.999, 1e-15
    runs = []
    for fused in (False, True):
        state = []
        for q, (n, act, na, reg, off) in enumerate(specs):
            gg = torch.Generator(device=cuda).manual_seed(10 + q)
            p = (torch.randn(n + off, generator=gg, device=cuda) * 3.0)[off:]
            m = (torch.randn(n + off, generator=gg, device=cuda) * 1e-3)[off:]
            v = (torch.rand(n + off, generator=gg, device=cuda) * 1e-6)[off:]
            accs = [torch.randn(n + off, generator=gg, device=cuda)[off:] for _ in range(na)]
            state.append((p, torch.empty(n + off, device=cuda)[off:], accs, m, v, act, reg, -(1e-3 / (1 - b1 ** (q + 2))),
                          (1 - b2 ** (q + 2)) ** 0.5))
        stream = ctypes.c_void_p(torch.cuda.current_stream(cuda).cuda_stream)
        if fused:
            arr = (nat.GrParamStep * len(state))()
            for e, (p, gr, accs, m, v, act, reg, ns, bc) in zip(arr, state):
                e.count, e.act, e.num_accs = p.numel(), act, len(accs)
                e.param, e.grad = p.data_ptr(), gr.data_ptr()
                for j, x in enumerate(accs):
                    e.accs[j] = x.data_ptr()
                e.exp_avg, e.exp_avg_sq = m.data_ptr(), v.data_ptr()
                e.reg, e.neg_step_size, e.bias_correction2_sqrt = reg, ns, bc
            nat.check(L.gr_fit_param_steps(len(state), arr, ctypes.c_double(b1), ctypes.c_double(b2), ctypes.c_float(eps),
                                           stream), "gr_fit_param_steps")
        else:
            for p, gr, accs, m, v, act, reg, ns, bc in state:
                ptrs = (ctypes.c_void_p * max(1, len(accs)))(*[x.data_ptr() for x in accs])
                nat.check(L.gr_fit_param_step(p.numel(), act, nat.ptr(p), nat.ptr(gr), ptrs, len(accs), ctypes.c_float(reg),
                                              1, nat.ptr(m), nat.ptr(v), ctypes.c_float(ns), ctypes.c_float(bc),
                                              ctypes.c_double(b1), ctypes.c_double(b2), ctypes.c_float(eps), stream),
                          "gr_fit_param_step")
        torch.cuda.synchronize()
        runs.append([(p, gr, m, v) for p, gr, _, m, v, *_ in state])
    for a, b in zip(*runs):
        for x, y in zip(a, b):
            assert torch.equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("n,rgb", [(1, True), (1000, True), (300_001, False), (2_000_000, True)])
def test_fit_activations_match_torch(pkg, cuda, n, rgb):
    """gr_fit_activations (the fused step's activations, one launch) gives torch's softplus + 1e-3 and sigmoid bit for
    bit, across softplus's threshold (x > 20) and both tails of the sigmoid; its regulariser (reg_opacity * mean(o) +
    reg_scale * mean(s), the means in double) is torch's float32 value within 1e-6; the workspace counter is left
    zero (a second call, same results)."""
    fm = importlib.import_module("3dgaussian_amd.fit_multiview")
    gg = torch.Generator(device=cuda).manual_seed(n)
    params = {"means": torch.randn((n, 3), generator=gg, device=cuda),
              "scales_raw": torch.randn((n, 3), generator=gg, device=cuda) * 12.0,
              "opacities_raw": torch.randn((n,), generator=gg, device=cuda) * 40.0}
    if rgb:
        params["colors_raw"] = torch.randn((n, 3), generator=gg, device=cuda) * 30.0
    else:
        params["sh_raw"] = torch.randn((n, 16, 3), generator=gg, device=cuda)
    if n >= 4:  # the thresholds and tails exactly
        params["scales_raw"].view(-1)[:4] = torch.tensor([20.0, 20.000002, -104.0, 88.0], device=cuda)
        params["opacities_raw"][:4] = torch.tensor([-88.0, 104.0, 0.0, -1e-8], device=cuda)
    ws = torch.zeros(int(pkg._native.lib().gr_fit_activations_ws_bytes(n)), dtype=torch.uint8, device=cuda)
    w_o, w_s = 1e-3, 2.5e-4
    ref = fm.activations(params)
    ref_reg = float(w_o * ref[3].mean() + w_s * ref[1].mean())
    for _ in range(2):
        m, s, c, o, reg = fm.activations_native(params, (w_o, w_s), ws)
        torch.cuda.synchronize()
        assert m.data_ptr() == params["means"].data_ptr()
        assert torch.equal(s, ref[1]) and torch.equal(o, ref[3]) and torch.equal(c, ref[2])
        assert abs(float(reg) - ref_reg) <= 1e-6 * abs(ref_reg), (float(reg), ref_reg)
    _, s2, _, o2, none = fm.activations_native(params)  # no regulariser, no workspace
    assert none is None and torch.equal(s2, ref[1]) and torch.equal(o2, ref[3])
