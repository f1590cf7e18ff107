"""Container-only check (the reference does not exist on the GPU box): run the UNCHANGED reference fit
loop /root/reference/python/fit_multiview_stub.py with this build's modules standing in for the
reference's ``torch_renderer`` and ``device_utils`` (the two modules the stub imports,
fit_multiview_stub.py:12-13), on the golden F4 setup (torch.manual_seed(1234), 300 Gaussians, 48x48,
3 targets, 6 iterations, densify/prune every 3), and compare its loss.txt with the reference's own
curve (tests/golden/f4_fit_curve.npz, made by tests/golden/make_golden.py from the reference modules).

The stub picks its device with get_default_device(): with no GPU (this container) that is ``cpu`` and
the drop-in runs its host op (cpu_renderer.py); on a HIP box it would be the HIP kernels.

Usage: python tools/run_reference_stub.py [--stub PATH]   (exit status 0 = curve matches at rtol 1e-4)
"""
import argparse, importlib, os, runpy, sys, tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stub", default="/root/reference/python/fit_multiview_stub.py")
    args = ap.parse_args()
    if not os.path.exists(args.stub):
        print(f"reference stub not found at {args.stub} (container-only check)")
        return 2
    import torch

    pkg = importlib.import_module("3dgaussian_amd")
    # the stub's `from torch_renderer import ...` / `from device_utils import ...` resolve to the drop-in
    sys.modules["torch_renderer"] = pkg.torch_renderer
    sys.modules["device_utils"] = pkg.device_utils
    g = np.load(os.path.join(REPO, "tests", "golden", "f4_fit_curve.npz"))
    sys.dont_write_bytecode = True
    with tempfile.TemporaryDirectory() as td:
        torch.manual_seed(int(g["seed"]))
        sys.argv = ["fit_multiview_stub.py", "--targets_dir", os.path.join(REPO, "tests", "golden", "fit_targets"),
                    "--out_dir", td, "--iters", str(int(g["iters"])), "--width", str(int(g["width"])),
                    "--height", str(int(g["width"])), "--num_gaussians", str(int(g["num_gaussians"])),
                    "--max_gaussians", str(int(g["max_gaussians"])), "--densify_interval", str(int(g["densify_interval"])),
                    "--prune_interval", str(int(g["densify_interval"]))]
        runpy.run_path(args.stub, run_name="__main__")
        losses = np.array([float(x) for x in open(os.path.join(td, "loss.txt")).read().split()])
    rel = np.abs(losses - g["losses"]) / np.abs(g["losses"])
    print("reference stub on the drop-in modules, device", pkg.device_utils.get_default_device())
    print("losses   ", " ".join(f"{x:.8f}" for x in losses))
    print("reference", " ".join(f"{x:.8f}" for x in g["losses"]))
    print(f"max relative difference {rel.max():.2e} (bar 1e-4)")
    return 0 if rel.max() <= 1e-4 else 1


if __name__ == "__main__":
    sys.exit(main())
