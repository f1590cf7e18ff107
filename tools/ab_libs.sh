#!/bin/bash
# Same-box per-kernel A/B over the tree's libgr_hip.so and abl/libgr_<name>.so variants
# (tools/ab_raster.py: fixed C4 Gaussians, 10 views, HIP-event kernel times):
#   bash tools/ab_libs.sh "<n1> <n2>" [reps]
set -e
NAMES=$1; REPS=${2:-2}
R=${GRAFT_REPO_ROOT:-$PWD}
for i in $(seq $REPS); do
  echo -n "tree: "; timeout -k 10 200 python $R/tools/ab_raster.py 1000000 800 10 2>/dev/null | tail -1
  for n in $NAMES; do
    echo -n "$n: "; GR_HIP_LIB=$R/abl/libgr_$n.so timeout -k 10 200 python $R/tools/ab_raster.py 1000000 800 10 2>/dev/null | tail -1
  done
done
