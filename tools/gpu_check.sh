#!/bin/bash
# GPU pass: gpu tests, smoke, the driver's bench command, optional extra configs.
# Usage: bash tools/gpu_check.sh <tag> [bench_configs names...]
set -e
TAG=${1:-r02}; shift || true
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/$TAG
mkdir -p $R/$O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1
if [ $# -gt 0 ]; then timeout -k 10 400 python tools/bench_configs.py "$@" --steps 4 > $O/configs.jsonl 2>&1; fi
