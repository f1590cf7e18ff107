#!/bin/bash
# One GPU-box pass: gpu tests, smoke, the driver's bench command.  Usage: bash tools/gpu_round3.sh <tag> [pytest -k expr]
set -e
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/$TAG
mkdir -p $R/$O
cd $R
K=${2:+-k "$2"}
timeout -k 10 840 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -s $K > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
