#!/bin/bash
# GPU tests (errors printed) with the working tree, then the depth-loss step: tree vs ab/<base> (same box).
#   bash tools/gpu_ab_depth.sh <tag> [base]
set -e
TAG=${1:-abd}; BASE=${2:-base}
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for i in 1 2; do
  echo -n "tree: " >> $O/depth.txt; timeout -k 10 200 python tools/depth_mode_run.py 3 50 2>/dev/null >> $O/depth.txt
  echo -n "$BASE: " >> $O/depth.txt; (cd ab/$BASE && timeout -k 10 200 python tools/depth_mode_run.py 3 50 2>/dev/null >> $O/depth.txt)
done
