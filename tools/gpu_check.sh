#!/bin/bash
# The driver's round-end commands on the committed tree: GPU tests, smoke, bench.   bash tools/gpu_check.sh <tag>
set -e
TAG=${1:-check}
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra-modes --no-dropin --no-psnr > $O/bench20.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/dropin_copies -o run --output-format csv -- python3 $R/tools/dropin_run.py 2 1 > $O/dropin_copies.log 2>&1
cd $R && python tools/copy_summary.py $O/dropin_copies 150 > $O/dropin_copies.txt
