#!/bin/bash
# Same-box A/B of bench.py: the working tree against ab/<name> trees (tools/ab_rev.sh), round-robin.
#   bash tools/ab_trees.sh "<name1> <name2>" [reps] [extra bench args]
set -e
NAMES=$1; REPS=${2:-2}; shift 2 || true
R=${GRAFT_REPO_ROOT:-$PWD}
summ() { grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); sp=d['splats']; print(d['value'], d['ms_per_step'], 'fwd_us', sp['fwd']['avg_launch_us'], 'bwd_us', sp['bwd']['avg_launch_us'], 'red_us', d.get('reduce_us_per_view'), 'bin_us', d.get('binning_us_per_view'))"; }
for i in $(seq $REPS); do
  echo -n "tree: "; timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-extra-modes "$@" 2>/dev/null | summ
  for n in $NAMES; do
    echo -n "$n: "; (cd $R/ab/$n && timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra-modes "$@" 2>/dev/null | summ)
  done
done
