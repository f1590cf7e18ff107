#!/bin/bash
# Same-box per-kernel A/B of compile variants in abl/ (tools/ab_lib.sh): the fit path's kernels and the
# default precision mode's (depth loss: forward MODE 1, backward <true,3>).  Usage: bash tools/ab_r02o.sh "<n1> <n2>" [reps]
set -e
NAMES=$1; REPS=${2:-2}
R=${GRAFT_REPO_ROOT:-$PWD}
run() {  # <lib name or tree> <env...>
  local n=$1; shift
  if [ "$n" = tree ]; then env "$@" timeout -k 10 200 python $R/tools/ab_raster.py 1000000 800 10 2>/dev/null | tail -1
  else env "$@" GR_HIP_LIB=$R/abl/libgr_$n.so timeout -k 10 200 python $R/tools/ab_raster.py 1000000 800 10 2>/dev/null | tail -1; fi
}
for i in $(seq $REPS); do
  for n in tree $NAMES; do run $n AB_FIT=1; done
  for n in tree $NAMES; do run $n AB_FIT=0 AB_DEPTH=1; done
done
