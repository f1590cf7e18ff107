#!/bin/bash
# GPU tests of a variant tree ab/<name> (goldens linked from the working tree), errors printed.
#   bash tools/gpu_variant_tests.sh <name> <tag> [pytest args...]
set -e
NAME=$1; TAG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R/ab/$NAME && ln -sfn $R/tests/golden tests/golden
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread "$@" > $O/pytest_$NAME.log 2>&1 || echo "pytest rc=$?" >> $O/pytest_$NAME.log
