#!/bin/bash
# Same-box A/B of the bench step at a few views per rank between tree copies (ab/<name>, "." = this tree).
#   bash tools/ab_views.sh <tag> <rounds> <views> <dir>...
set -eo pipefail
TAG=$1
ROUNDS=$2
V=$3
shift 3
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for d in "$@"; do
    name=$(basename $(cd $R/$d && pwd))
    (cd $R/$d && timeout -k 10 200 python bench.py --views $V --steps 20 --warmup 3 --no-cpu-baseline --no-psnr --no-dropin \
      --no-extra-modes > $O/v${V}_${name}_$r.log 2>&1)
    echo "$name round $r views $V: $(grep -o '"ms_per_step": [0-9.]*' $O/v${V}_${name}_$r.log)"
  done
done
