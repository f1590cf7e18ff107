#!/bin/bash
# Copy the working tree into ab/<name>/ and build its HIP library with extra compiler flags, for
# same-box A/B of compile-time knobs:  tools/ab_variant.sh <name> "-DGR_CH=2048 ..."
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
DST=$ROOT/ab/$NAME
rm -rf "$DST" && mkdir -p "$DST"
tar -C "$ROOT" --exclude=./ab --exclude=./.git --exclude=./gpurun_out --exclude=./tests/golden -cf - . | tar -x -C "$DST"
rm -f "$DST/3dgaussian_amd/libgr_hip.so"  # the copied library is newer than its source: force the rebuild
make -s -B -C "$DST/3dgaussian_amd/csrc" EXTRA="$FLAGS" >/dev/null
echo "built $DST ($FLAGS)"
