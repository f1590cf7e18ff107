"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself (container only).

Run once in the build container (the reference is absent on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Sources of truth (nothing from the reference is copied into the repo; only input/output vectors):
  * F1/F2 float goldens: /root/reference/python/torch_renderer.py imported as-is (torch 2.10 CPU,
    float32), outputs of render_gaussians_torch(..., return_aux=True) and autograd gradients of
    L = sum(out*g_rgb) + sum(alpha*g_alpha) + sum(depth*g_depth) for seeded random upstream grads.
  * F3 uint8 goldens: /root/reference/src/renderer_cpu.cpp compiled from source by
    oracle/build_ref.sh (oracle/_ref/libref.so), OIT and depth-sorted modes.
  * F4 fit curve: /root/reference/python/fit_multiview_stub.py run on CPU with
    torch.manual_seed(1234) on the tiny synthetic targets in tests/golden/fit_targets/.
  * F5 camera gradients (``make_golden.py camera`` writes only these): the same imported
    torch_renderer.py with camera.view / camera.proj requiring grad; autograd's d view / d proj of the F1
    loss with and without its depth term.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("GR_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(REF, "python"))
sys.path.insert(0, REPO)

import torch_renderer as ref  # noqa: E402  (the reference module, imported read-only)

from oracle import oracle as orc  # noqa: E402


def ref_cam(view, proj):
    return ref.Camera(view=torch.from_numpy(np.asarray(view, np.float32)), proj=torch.from_numpy(np.asarray(proj, np.float32)))


def run_ref(scene: orc.Scene, view, proj, W, H, bg, seed):
    """Reference forward + autograd backward in float32."""
    m = torch.from_numpy(scene.means.copy()).requires_grad_(True)
    s = torch.from_numpy(scene.scales.copy()).requires_grad_(True)
    c = torch.from_numpy(scene.colors.copy()).requires_grad_(True)
    o = torch.from_numpy(scene.opacities.copy()).requires_grad_(True)
    n = m.shape[0]
    res = ref.render_gaussians_torch(m, s, c, o, ref_cam(view, proj), W, H, background=torch.from_numpy(bg),
                                     max_gaussians=max(10000, n), return_aux=True)
    g = np.random.default_rng(seed + 7)
    g_rgb = g.standard_normal((H, W, 3)).astype(np.float32)
    g_a = g.standard_normal((H, W)).astype(np.float32)
    g_d = g.standard_normal((H, W)).astype(np.float32)
    out = {"g_rgb": g_rgb, "g_alpha": g_a, "g_depth": g_d}
    if n == 0:
        out.update(out_rgb=res.detach().numpy(), out_alpha=np.zeros((H, W), np.float32), out_depth=np.zeros((H, W), np.float32))
        for k, a in (("d_means", m), ("d_scales", s), ("d_colors", c), ("d_opacities", o)):
            out[k] = np.zeros(a.shape, np.float32)
        return out
    rgb, alpha, depth = res
    loss = (rgb * torch.from_numpy(g_rgb)).sum() + (alpha * torch.from_numpy(g_a)).sum() + (depth * torch.from_numpy(g_d)).sum()
    loss.backward()
    out.update(out_rgb=rgb.detach().numpy(), out_alpha=alpha.detach().numpy(), out_depth=depth.detach().numpy())
    for k, a in (("d_means", m), ("d_scales", s), ("d_colors", c), ("d_opacities", o)):
        out[k] = (a.grad if a.grad is not None else torch.zeros_like(a)).numpy().astype(np.float32)
    return out


def edge_scene(n, seed, sh=False) -> orc.Scene:
    """Random scene with every edge case the reference math has."""
    rng = np.random.default_rng(seed)
    means = rng.uniform(-0.9, 0.9, (n, 3)).astype(np.float32)
    scales = rng.uniform(0.01, 0.2, (n, 3)).astype(np.float32)
    opac = rng.uniform(0.05, 0.9, (n,)).astype(np.float32)
    if sh:
        colors = (rng.standard_normal((n, 4, 3)) * 0.3).astype(np.float32)
        colors[:, 0, :] += 0.5
    else:
        colors = rng.uniform(-0.2, 1.2, (n, 3)).astype(np.float32)  # some outside [0,1]
    if n >= 7:
        means[0] = [0.0, 0.5, 3.5]  # behind the camera (eye at z=2.5 looking at origin)
        means[1] = [6.0, 0.0, 0.0]  # far off-screen to the side
        means[2] = [0.0, 0.49, 2.48]  # right at the near plane
        scales[3] = [-0.1, -0.05, 0.3]  # negative scales (abs in torch)
        opac[4] = -0.3  # negative opacity (clamp_min 0)
        opac[5] = 0.0  # exactly zero opacity (gradient still flows)
        scales[6] = [1e-4, 1e-4, 1e-4]  # sub-pixel sigma (clamped to 1)
    return orc.Scene(means, scales, colors, opac)


def main():
    torch.set_num_threads(8)
    cams = {}
    fixtures = {}

    # ---- F1: edge cases ------------------------------------------------------------------
    cases = [(0, 17, 13, False), (1, 17, 13, False), (7, 32, 32, False), (64, 64, 48, False), (300, 64, 48, False),
             (64, 32, 32, True), (300, 64, 48, True)]
    for idx, (n, W, H, sh) in enumerate(cases):
        view = orc.look_at([0.0, 0.5, 2.5], [0, 0, 0], [0, 1, 0])
        proj = orc.perspective(60.0, W / H, 0.01, 100.0)
        bg = np.array([0.1, 0.2, 0.3], np.float32) if idx % 2 else np.zeros(3, np.float32)
        scene = edge_scene(n, seed=100 + idx, sh=sh)
        if n == 1:
            scene.means[0] = [0.05, -0.02, 0.1]
        res = run_ref(scene, view, proj, W, H, bg, seed=100 + idx)
        name = f"f1_n{n}_{W}x{H}{'_sh' if sh else ''}"
        fixtures[name] = dict(width=np.int32(W), height=np.int32(H), view=view, proj=proj, background=bg,
                              means=scene.means, scales=scene.scales, colors=scene.colors, opacities=scene.opacities, **res)

    # ---- F2: the C1 scene (1200 G, 128^2, 4 orbit views of fit_multiview_stub.py:70-90) ------
    scene = orc.synthetic_scene(1200, seed=0, scale=0.1061)
    for vi, (view, proj) in enumerate(orc.orbit_cameras(4, 128, 128)):
        res = run_ref(scene, view, proj, 128, 128, np.zeros(3, np.float32), seed=200 + vi)
        fixtures[f"f2_c1_view{vi}"] = dict(width=np.int32(128), height=np.int32(128), view=view, proj=proj,
                                           background=np.zeros(3, np.float32), means=scene.means, scales=scene.scales,
                                           colors=scene.colors, opacities=scene.opacities, **res)

    for name, d in fixtures.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name)

    # ---- F3: uint8 surface from the compiled reference CPU renderer ---------------------------
    so = os.path.join(REPO, "oracle", "_ref", "libref.so")
    if not os.path.exists(so):
        subprocess.run([os.path.join(REPO, "oracle", "build_ref.sh")], check=True)
    lib = ctypes.CDLL(so)
    P = ctypes.c_void_p

    def ref_u8(W, H, view, proj, bg, sort, sc: orc.Scene):
        out = np.zeros((H, W, 4), np.uint8)
        m, s, c, o = sc.arrays()
        lib.ref_render_u8(ctypes.c_int(W), ctypes.c_int(H), P(np.ascontiguousarray(view, np.float32).ctypes.data),
                          P(np.ascontiguousarray(proj, np.float32).ctypes.data), P(np.ascontiguousarray(bg, np.float32).ctypes.data),
                          ctypes.c_int(sort), ctypes.c_int(m.shape[0]), P(m.ctypes.data), P(s.ctypes.data), P(c.ctypes.data),
                          P(o.ctypes.data), P(out.ctypes.data))
        return out

    u8 = {}
    for (n, W, H, seed) in [(0, 17, 13, 1), (7, 32, 32, 2), (300, 64, 48, 3), (1200, 128, 128, 4)]:
        sc = edge_scene(n, seed) if n != 1200 else orc.synthetic_scene(1200, seed=0, scale=0.1061)
        if n != 1200:
            sc.colors = np.clip(sc.colors, 0, 1)  # reference surface has no colour clamp
        view = orc.look_at([0.3, 0.6, 2.4], [0, 0, 0], [0, 1, 0])
        proj = orc.perspective(55.0, W / H, 0.01, 100.0)
        bg = np.array([0.05, 0.1, 0.15], np.float32)
        for sort in (0, 1):
            key = f"u8_n{n}_{W}x{H}_sort{sort}"
            u8[key] = dict(width=np.int32(W), height=np.int32(H), view=view, proj=proj, background=bg, sort=np.int32(sort),
                           means=sc.means, scales=sc.scales, colors=sc.colors, opacities=sc.opacities,
                           rgba=ref_u8(W, H, view, proj, bg, sort, sc))
    for name, d in u8.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name)

    # ---- F4: fit-loop loss curve of the unchanged stub --------------------------------------
    tdir = os.path.join(HERE, "fit_targets")
    os.makedirs(tdir, exist_ok=True)
    from PIL import Image

    rng = np.random.default_rng(42)
    yy, xx = np.mgrid[0:48, 0:48].astype(np.float32) / 47.0
    for vi in range(3):
        img = np.zeros((48, 48, 3), np.float32)
        for _ in range(4):
            cx, cy, r = rng.uniform(0.2, 0.8), rng.uniform(0.2, 0.8), rng.uniform(0.08, 0.25)
            col = rng.uniform(0.2, 1.0, 3)
            mask = ((xx - cx) ** 2 + (yy - cy) ** 2) < r * r
            img[mask] = col
        Image.fromarray((img * 255).astype(np.uint8)).save(os.path.join(tdir, f"v{vi}.png"))
    with tempfile.TemporaryDirectory() as td:
        code = (
            "import sys, torch; sys.path.insert(0, %r); torch.manual_seed(1234); sys.argv=['fit', '--targets_dir', %r, "
            "'--out_dir', %r, '--iters', '6', '--width', '48', '--height', '48', '--num_gaussians', '300', "
            "'--max_gaussians', '400', '--densify_interval', '3', '--prune_interval', '3']; "
            "import fit_multiview_stub as f; f.main()"
        ) % (os.path.join(REF, "python"), tdir, td)
        env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
        subprocess.run([sys.executable, "-c", code], check=True, cwd=td, env=env)
        losses = np.array([float(x) for x in open(os.path.join(td, "loss.txt")).read().split()], np.float64)
    np.savez_compressed(os.path.join(HERE, "f4_fit_curve.npz"), losses=losses, iters=np.int32(6), width=np.int32(48),
                        num_gaussians=np.int32(300), max_gaussians=np.int32(400), densify_interval=np.int32(3), seed=np.int32(1234))
    print("F4 losses", losses)


def camera_main():
    """F5: camera-gradient fixtures (view / proj requiring grad in the reference's autograd)."""
    torch.set_num_threads(8)
    cases = [("f5_cam_n64_64x48", edge_scene(64, seed=501), 64, 48, orc.look_at([0.3, 0.5, 2.4], [0, 0, 0], [0, 1, 0])),
             ("f5_cam_n300_64x48_sh", edge_scene(300, seed=502, sh=True), 64, 48,
              orc.look_at([-0.4, 0.6, 2.3], [0, 0, 0], [0, 1, 0])),
             ("f5_cam_c1_view1", orc.synthetic_scene(1200, seed=0, scale=0.1061), 128, 128, orc.orbit_cameras(4, 128, 128)[1][0])]
    for ci, (name, scene, W, H, view) in enumerate(cases):
        proj = orc.perspective(60.0, W / H, 0.01, 100.0)
        bg = np.array([0.1, 0.2, 0.3], np.float32)
        g = np.random.default_rng(600 + ci)
        g_rgb = g.standard_normal((H, W, 3)).astype(np.float32)
        g_a = g.standard_normal((H, W)).astype(np.float32)
        g_d = g.standard_normal((H, W)).astype(np.float32)
        d = dict(width=np.int32(W), height=np.int32(H), view=np.asarray(view, np.float32), proj=np.asarray(proj, np.float32),
                 background=bg, means=scene.means, scales=scene.scales, colors=scene.colors, opacities=scene.opacities,
                 g_rgb=g_rgb, g_alpha=g_a, g_depth=g_d)
        for tag, with_depth in (("", True), ("_nodepth", False)):
            vt = torch.from_numpy(np.asarray(view, np.float32).copy()).requires_grad_(True)
            pt = torch.from_numpy(np.asarray(proj, np.float32).copy()).requires_grad_(True)
            m, s, c, o = (torch.from_numpy(a.copy()) for a in scene.arrays())
            rgb, alpha, depth = ref.render_gaussians_torch(m, s, c, o, ref.Camera(view=vt, proj=pt), W, H,
                                                           background=torch.from_numpy(bg), max_gaussians=10000,
                                                           return_aux=True)
            loss = (rgb * torch.from_numpy(g_rgb)).sum() + (alpha * torch.from_numpy(g_a)).sum()
            if with_depth:
                loss = loss + (depth * torch.from_numpy(g_d)).sum()
            loss.backward()
            d["d_view" + tag] = vt.grad.numpy().astype(np.float32)
            d["d_proj" + tag] = pt.grad.numpy().astype(np.float32)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name, float(np.abs(d["d_view"]).max()), float(np.abs(d["d_proj"]).max()))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "camera":
        camera_main()
    else:
        main()
