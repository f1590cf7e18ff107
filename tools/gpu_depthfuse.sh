#!/bin/bash
# Fused-depth-loss tests, then C3 / C2 configs for the tree and ab/base (same box).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/dfuse; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_c3_fit_gpu.py tests/test_fit_exec_gpu.py tests/test_fit_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
for i in 1 2; do
  echo "tree" >> $O/configs.txt; timeout -k 10 200 python tools/bench_configs.py C3 --steps 10 >> $O/configs.txt 2>/dev/null
  echo "base" >> $O/configs.txt; (cd ab/base && timeout -k 10 200 python tools/bench_configs.py C3 --steps 10 >> ../../gpurun_out/dfuse/configs.txt 2>/dev/null)
done
echo -n "tree: " >> $O/depth.txt; timeout -k 10 200 python tools/depth_mode_run.py 3 50 2>/dev/null >> $O/depth.txt
echo -n "base: " >> $O/depth.txt; (cd ab/base && timeout -k 10 200 python tools/depth_mode_run.py 3 50 2>/dev/null >> ../../gpurun_out/dfuse/depth.txt)
