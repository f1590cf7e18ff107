#!/bin/bash
# Same-box comparison of bench.py over the working tree and ab/<name> variants, round-robin.
#   bash tools/ab_multi.sh "<name1> <name2> ..." [reps]
set -e
NAMES=$1; REPS=${2:-2}
R=${GRAFT_REPO_ROOT:-$PWD}
summ() { grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); sp=d['splats']; print(d['value'], 'fwd_us', sp['fwd']['avg_launch_us'], 'bwd_us', sp['bwd']['avg_launch_us'])"; }
for i in $(seq $REPS); do
  echo -n "tree: "; timeout -k 10 300 python $R/bench.py --no-cpu-baseline 2>/dev/null | summ
  for n in $NAMES; do
    echo -n "$n: "; (cd $R/ab/$n && timeout -k 10 300 python bench.py --no-cpu-baseline 2>/dev/null | summ)
  done
done
