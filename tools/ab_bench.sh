#!/bin/bash
# Same-box A/B of the bench step between tree copies (tools/ab_variant.sh, or `git archive` into ab/<name>):
# alternates the trees' benches, each under its own time limit.   bash tools/ab_bench.sh <tag> <rounds> <dir>...
# (a dir of "." is this tree)
set -eo pipefail
TAG=$1
ROUNDS=$2
shift 2
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for d in "$@"; do
    name=$(basename $(cd $R/$d && pwd))
    (cd $R/$d && timeout -k 10 240 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-psnr --no-dropin \
      --no-extra-modes > $O/ab_${name}_$r.log 2>&1)
    echo "$name round $r: $(python3 -c "
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); s=d.get('splats',{})
        print(d['value'], 'fwd_us', s.get('fwd',{}).get('avg_launch_us'), 'bwd_us', s.get('bwd',{}).get('avg_launch_us'),
              'red_us', d.get('reduce_us_per_view'), 'bin_us', d.get('binning_us_per_view'))
" $O/ab_${name}_$r.log)"
  done
done
