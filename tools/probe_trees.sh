#!/bin/bash
# tools/splat_probe.py in each tree copy, each under its own time limit:  bash tools/probe_trees.sh <tag> <dir>...
set -eo pipefail
TAG=$1; shift; ARGS=${PROBE_ARGS:---views 4 --reps 10 --steps 0}
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
for d in "$@"; do
  (cd $R/$d && timeout -k 10 200 python tools/splat_probe.py $ARGS >> $O/probe.txt 2>> $O/probe.err)
done
