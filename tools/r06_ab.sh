#!/bin/bash
# Round-6 consolidated same-box A/B on the GPU box: kernel probe + micro + bench, each step under its own limit.
#   bash tools/r06_ab.sh <tag> <base dir> [bench rounds]
set -eo pipefail
TAG=$1; BASE=$2; ROUNDS=${3:-2}
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
echo "== probe $(date +%T)"
bash tools/probe_trees.sh $TAG $BASE . $BASE .
if [ -x tools/microbin/mfma32_valu ]; then
  echo "== micro $(date +%T)"
  timeout -k 10 120 ./tools/microbin/mfma32_valu > $O/micro.txt 2>&1
fi
echo "== bench $(date +%T)"
bash tools/ab_bench.sh $TAG $ROUNDS $BASE . > $O/ab.txt 2>&1
echo "== done $(date +%T)"
