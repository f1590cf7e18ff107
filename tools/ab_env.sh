#!/bin/bash
# Same-box A/B of bench.py over environment settings, round-robin:
#   bash tools/ab_env.sh "GR_REDUCE_BATCH=1 GR_REDUCE_BATCH=4" [reps] [extra bench args]
set -e
SETS=$1; REPS=${2:-2}; shift 2 || true
R=${GRAFT_REPO_ROOT:-$PWD}
for i in $(seq $REPS); do
  for e in $SETS; do
    echo -n "$e: "; env ${e//,/ } timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-extra-modes --no-dropin --no-psnr "$@" 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); sp=d['splats']; print(d['value'], d['ms_per_step'], 'fwd_us', sp['fwd']['avg_launch_us'], 'bwd_us', sp['bwd']['avg_launch_us'])"
  done
done
