#!/bin/bash
# Same-box A/B of bench.py: the working tree against ab/<name> (tools/ab_snapshot.sh), alternating.
#   bash tools/ab_bench.sh <name> [reps] [extra bench args]
set -e
NAME=${1:-base}; REPS=${2:-2}; shift 2 || true
R=${GRAFT_REPO_ROOT:-$PWD}
summ() { grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], 'bwd_us', r['avg_launch_us'], 'fwd_us', r['fwd_kernel_avg_us'])"; }
for i in $(seq $REPS); do
  echo -n "tree: "; timeout -k 10 300 python $R/bench.py --no-cpu-baseline "$@" 2>/dev/null | summ
  echo -n "$NAME: "; (cd $R/ab/$NAME && timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | summ)
done
