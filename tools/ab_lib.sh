#!/bin/bash
# Build a variant of libgr_hip.so with extra compiler flags into abl/libgr_<name>.so (travels to the GPU
# box; git-ignored), for same-box A/B with tools/ab_libs.sh:  tools/ab_lib.sh <name> "-DGR_X=1 ..."
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/abl"
make -s -B -C "$ROOT/3dgaussian_amd/csrc" EXTRA="$FLAGS" OUT="$ROOT/abl/libgr_$NAME.so" >/dev/null
echo "built abl/libgr_$NAME.so ($FLAGS)"
