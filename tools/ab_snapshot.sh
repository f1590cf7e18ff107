#!/bin/bash
# Export a committed revision into ab/<name>/ (git-ignored, travels to the GPU box) and build its HIP
# library there, for same-box A/B runs of bench.py / tools/ab_raster.py:  tools/ab_snapshot.sh <rev> <name>
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
DST=$ROOT/ab/$NAME
rm -rf "$DST" && mkdir -p "$DST"
git -C "$ROOT" archive "$REV" | tar -x -C "$DST"
rm -rf "$DST/tests/golden"
make -s -C "$DST/3dgaussian_amd/csrc" >/dev/null
make -s -C "$DST/oracle" >/dev/null
echo "built $DST"
