"""Diagnostic: dense-reference error of the fused fit path's footprint as a function of its cutoff (sigma),
on the C4 bench scene (fresh and after 8 fit steps): relL2 of out/alpha at 1000 pixels and of the four
gradients of 1000 Gaussians against the float64 dense oracle, plus the view's pair count."""
import importlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import oracle as orc  # noqa: E402

tr = importlib.import_module("3dgaussian_amd.torch_renderer")
fm = importlib.import_module("3dgaussian_amd.fit_multiview")
bench = importlib.import_module("bench")
cuda = torch.device("cuda:0")
GRADS = ("d_means", "d_scales", "d_colors", "d_opac")
n, W, H, V = 1_000_000, 800, 800, 50
cuts = [float(c) for c in (sys.argv[1:] or ["5.0", "4.5", "4.0"])]


def run(acts, view, proj, sc, seed):
    rng = np.random.default_rng(seed)
    g_rgb = rng.standard_normal((H, W, 3)).astype(np.float32)
    g_a = rng.standard_normal((H, W)).astype(np.float32)
    pix = rng.choice(W * H, 1000, replace=False).astype(np.int32)
    sel = np.sort(rng.choice(n, 1000, replace=False)).astype(np.int32)
    v = orc.make_view(view, proj, W, H, None, cutoff=5.0, core_cutoff=5.0)
    d_out, d_a, _ = orc.dense_pixels(v, sc, pix)
    dense_g = orc.dense_grads_sel(v, sc, sel, g_rgb, g_a, None)
    for c in cuts:
        gv = tr.make_view(view, proj, W, H, None, cutoff=c, core_cutoff=c, depth_grad=False)
        out, alpha, depth, st = tr.forward_native(*acts, gv, want_depth=False)
        grads = tr.backward_native(*acts, st, torch.from_numpy(g_rgb).to(cuda), torch.from_numpy(g_a).to(cuda), None)
        errs = {"out": orc.rel_l2(out.cpu().numpy().reshape(-1, 3)[pix], d_out),
                "alpha": orc.rel_l2(alpha.cpu().numpy().reshape(-1)[pix], d_a)}
        for k, x, gd in zip(GRADS, grads, dense_g):
            errs[k] = orc.rel_l2(x.cpu().numpy()[sel], gd)
        print(f"  cutoff {c}: pairs {st.num_pairs}", {k: f"{e:.2e}" for k, e in errs.items()}, flush=True)


sc = orc.synthetic_scene(n, seed=0)
perm = fm.morton_order(torch.from_numpy(sc.means)).numpy()
sc = orc.Scene(sc.means[perm].copy(), sc.scales[perm].copy(), sc.colors[perm].copy(), sc.opacities[perm].copy())
view, proj = orc.orbit_cameras(V, W, H)[0]
print("fresh C4 scene, view 0", flush=True)
run([torch.from_numpy(a).to(cuda) for a in sc.arrays()], view, proj, sc, 7)

params = bench.synthetic_params(n, cuda)
cams = fm.orbit_cameras(V, W, H, cuda)
g = torch.Generator(device=cuda).manual_seed(1)
targets = [torch.rand((H, W, 3), generator=g, device=cuda) for _ in range(V)]
masks = [(t.mean(dim=2) > 0.5).float() for t in targets]
fit = fm.ViewShardedFitter(params, cams, targets, W, H, lr=0.02, masks=masks)
for _ in range(8):
    fit.step()
with torch.no_grad():
    acts = [a.detach().contiguous() for a in fm.activations(fit.params)]
sc = orc.Scene(*(a.cpu().numpy() for a in acts))
view, proj = orc.orbit_cameras(V, W, H)[3]
print("fitted C4 state (8 steps, lr 0.02), view 3", flush=True)
run(acts, view, proj, sc, 9)
