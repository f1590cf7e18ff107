#!/bin/bash
# GPU tests (errors printed) with the working tree, then the depth-loss step for the tree and ab/tail3.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/tail2; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for i in 1 2; do
  echo -n "tree: " >> $O/depth.txt; timeout -k 10 200 python tools/depth_mode_run.py 3 50 >> $O/depth.txt 2>&1
  echo -n "tail3: " >> $O/depth.txt; (cd ab/tail3 && timeout -k 10 200 python tools/depth_mode_run.py 3 50 >> $O/depth.txt 2>&1)
done
