#!/bin/bash
# Same-box A/B of tools/bench_configs.py between tree copies (ab/<name>, "." = this tree), alternating.
#   bash tools/ab_configs.sh <tag> <rounds> "<configs>" <dir>...
set -eo pipefail
TAG=$1
ROUNDS=$2
CFG=$3
shift 3
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for d in "$@"; do
    name=$(basename $(cd $R/$d && pwd))
    (cd $R/$d && timeout -k 10 300 python tools/bench_configs.py $CFG --steps 20 > $O/cfg_${name}_$r.txt 2> $O/cfg_${name}_$r.err)
    echo "$name round $r: $(python3 -c "import json,sys; print([(d['config'], d['mpx_per_s']) for d in map(json.loads, open(sys.argv[1]))])" $O/cfg_${name}_$r.txt)"
  done
done
