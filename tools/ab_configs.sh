#!/bin/bash
# Same-box A/B of tools/bench_configs.py over environment settings, round-robin:
#   bash tools/ab_configs.sh "C3 C5" "GR_STREAMS=4 GR_HIP_LIB=abl/libgr_prev.so,GR_PREP_FIRST=4" [reps]
set -e
CONFIGS=$1; SETS=$2; REPS=${3:-2}
R=${GRAFT_REPO_ROOT:-$PWD}
for i in $(seq $REPS); do
  for e in $SETS; do
    echo "== $e"; env ${e//,/ } timeout -k 10 400 python $R/tools/bench_configs.py $CONFIGS --steps 6 2>/dev/null | grep '^{' | python -c "import json,sys; [print(d['config'], d['mpx_per_s'], d['ms_per_step']) for d in map(json.loads, sys.stdin)]"
  done
done
