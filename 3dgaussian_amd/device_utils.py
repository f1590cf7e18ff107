"""Device policy (replaces python/device_utils.py:1-13).

The reference returns ``cuda`` only on Windows and otherwise ``mps``/``cpu`` (device_utils.py:9-13),
which on Linux/ROCm would put the fit loop on the CPU.  Here a visible HIP device is always chosen.
"""
from __future__ import annotations

import torch


def get_default_device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda")
    if getattr(torch.backends, "mps", None) is not None and torch.backends.mps.is_available():
        return torch.device("mps")
    return torch.device("cpu")
