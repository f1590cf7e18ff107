#!/bin/bash
# Determinism check of the native executor at C4 size, alternating tree copies, each run under its own limit:
#   bash tools/exec_det.sh <tag> <rounds> <dir>...
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for d in "$@"; do
    name=$(basename $(cd $R/$d && pwd))
    (cd $R/$d && timeout -k 10 200 python -u -m pytest tests/test_fit_exec_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread -k c4_size > $O/${name}_$r.log 2>&1)
    rc=$?
    echo "$name round $r: rc=$rc $(tail -1 $O/${name}_$r.log)" >> $O/det.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
