#!/bin/bash
# Same-box per-kernel A/B (tools/ab_raster.py: fixed Gaussians, 10 views, HIP-event kernel times) over
# the working tree and ab/<name> variants:  bash tools/ab_raster_multi.sh "<n1> <n2>" [reps]
set -e
NAMES=$1; REPS=${2:-2}
R=${GRAFT_REPO_ROOT:-$PWD}
for i in $(seq $REPS); do
  echo -n "tree: "; timeout -k 10 200 python $R/tools/ab_raster.py 1000000 800 10 2>/dev/null | tail -1
  for n in $NAMES; do
    echo -n "$n: "; (cd $R/ab/$n && timeout -k 10 200 python tools/ab_raster.py 1000000 800 10 2>/dev/null | tail -1)
  done
done
