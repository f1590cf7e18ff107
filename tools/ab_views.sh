#!/bin/bash
# Per-rank throughput at the view counts one rank renders when the driver scales C4 over N GPUs
# (50 views: 25 at N=2, 13 at N=4, 7 at N=8), over environment settings, same box:
#   bash tools/ab_views.sh "7 13" "GR_STREAMS=4 GR_STREAMS=3" [reps]
set -e
VIEWS=$1; SETS=$2; REPS=${3:-1}
R=${GRAFT_REPO_ROOT:-$PWD}
for i in $(seq $REPS); do
  for v in $VIEWS; do
    for e in $SETS; do
      echo -n "views=$v $e: "; env ${e//,/ } timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-extra-modes --no-dropin --no-psnr --views $v --steps 20 --warmup 3 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
    done
  done
done
