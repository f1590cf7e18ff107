#!/bin/bash
# Same-box A/B of tools/bench_configs.py configs between tree copies (tools/ab_variant.sh), alternating:
#   bash tools/ab_configs.sh <tag> <rounds> <steps> "<configs>" <dir>...      (a dir of "." is this tree)
set -eo pipefail
TAG=$1; ROUNDS=$2; STEPS=$3; CONFIGS=$4
shift 4
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for d in "$@"; do
    name=$(basename $(cd $R/$d && pwd))
    (cd $R/$d && timeout -k 10 240 python tools/bench_configs.py $CONFIGS --steps $STEPS > $O/cfg_${name}_$r.log 2>&1)
    echo "$name round $r: $(python3 -c "
import json,sys
print(' '.join('%s %.1f' % (d['config'], d['mpx_per_s']) for d in (json.loads(l) for l in open(sys.argv[1]) if l.startswith('{'))))
" $O/cfg_${name}_$r.log)"
  done
done
