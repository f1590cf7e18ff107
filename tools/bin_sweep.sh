#!/bin/bash
# Placement variants of the binning (tools/bin_bench.py under rocprofv3, one run per "waves:target" pair).
#   bash tools/bin_sweep.sh <tag> 8:0 4:0 4:6144 ...
set -eo pipefail
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for cfg in "$@"; do
  W=${cfg%%:*}
  T=${cfg##*:}
  echo "== $cfg $(date +%T)"
  (cd /tmp && GR_TUNE_PLACE_WAVES=$W GR_TUNE_COL_TARGET=$T timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/bin_${W}_${T} \
    -o run --output-format csv -- python3 $R/tools/bin_bench.py 30 > $O/bin_${W}_${T}.log 2>&1)
  grep us_per_binning $O/bin_${W}_${T}.log
  (cd $R && python tools/kstats.py $O/bin_${W}_${T} > $O/bin_${W}_${T}.txt && sed -n 2,6p $O/bin_${W}_${T}.txt)
done
