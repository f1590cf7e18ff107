"""3dgaussian_amd — MI355X-native differentiable Gaussian rasterizer (drop-in for Kirkice/3DGaussian's
render op).  Import as ``importlib.import_module("3dgaussian_amd")`` (the name starts with a digit), or
put this directory on ``sys.path`` and ``import torch_renderer`` exactly like the reference's python/."""
from . import _native, device_utils, gaussian_renderer, losses, torch_renderer  # noqa: F401
from .torch_renderer import Camera, get_default_device, look_at, perspective, rasterize, render_gaussians_torch  # noqa: F401

__all__ = ["Camera", "get_default_device", "look_at", "perspective", "rasterize", "render_gaussians_torch",
           "gaussian_renderer", "torch_renderer", "device_utils", "losses"]
