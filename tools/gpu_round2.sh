#!/bin/bash
# One GPU-box pass for the round record: gpu tests, smoke, the driver's bench command, rocprofv3 kernel
# stats (single stream and as run), PMC HBM traffic, the other configs.  Usage: bash tools/gpu_round2.sh <tag>
set -e
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/$TAG
mkdir -p $R/$O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_20.log 2>&1
bash tools/prof_r02.sh $TAG/prof 20 5
bash tools/pmc_bench.sh $O/pmc
timeout -k 10 400 python tools/bench_configs.py C2 C3 C5 C5d --steps 6 > $O/configs.jsonl 2>&1
