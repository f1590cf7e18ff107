"""The drop-in op as the unchanged reference loop calls it (bench.dropin_op), alone, for profiling:
    python tools/dropin_run.py [steps] [warmup]"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

bench = importlib.import_module("bench")
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 1
print(json.dumps(bench.dropin_op(1_000_000, 50, 800, steps, warmup, torch.device("cuda", 0))))
