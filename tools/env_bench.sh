#!/bin/bash
# Same-box A/B of environment settings of this tree's bench step: bash tools/env_bench.sh <tag> <rounds> "<env>"...
# ("-" = no extra environment)
set -eo pipefail
TAG=$1
ROUNDS=$2
shift 2
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    [ "$e" = "-" ] && e=""
    (cd $R && env $e timeout -k 10 240 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-psnr --no-dropin \
      --no-extra-modes > $O/env${i}_$r.log 2>&1)
    echo "[$e] round $r: $(grep -o '"value": [0-9.]*' $O/env${i}_$r.log | head -1)"
  done
done
