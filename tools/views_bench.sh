#!/bin/bash
# The bench step at fewer views per rank (the 8-GPU run's per-rank share: 7 views of 50), both schedules.
#   [VIEWS="7 13"] [ENVS="- GR_NATIVE_EXEC=1"] bash tools/views_bench.sh <tag>
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$1
mkdir -p $O
for v in ${VIEWS:-7 13}; do
  for e in ${ENVS:-- GR_NATIVE_EXEC=1}; do  # "-": no extra environment
    [ "$e" = "-" ] && e=""
    (cd $R && env $e timeout -k 10 200 python bench.py --views $v --steps 20 --warmup 3 --no-cpu-baseline --no-psnr \
      --no-dropin --no-extra-modes > $O/views_${v}_${e:-py}.log 2>&1)
    echo "views $v ${e:-python schedule}: $(grep -o '"ms_per_step": [0-9.]*' $O/views_${v}_${e:-py}.log)"
  done
done
