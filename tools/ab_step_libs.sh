#!/bin/bash
# Same-box step-level A/B of abl/libgr_<name>.so variants (tools/ab_lib.sh) against the tree's library:
# bench.py's C4 step, round-robin.  Usage: bash tools/ab_step_libs.sh "<n1> <n2>" [reps] [bench args]
set -e
NAMES=$1; REPS=${2:-2}; shift 2 || true
R=${GRAFT_REPO_ROOT:-$PWD}
val() { grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for i in $(seq $REPS); do
  echo -n "tree: "; timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-extra-modes "$@" 2>/dev/null | val
  for n in $NAMES; do
    echo -n "$n: "; GR_HIP_LIB=$R/abl/libgr_$n.so timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-extra-modes "$@" 2>/dev/null | val
  done
done
