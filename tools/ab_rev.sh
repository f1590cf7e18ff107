#!/bin/bash
# Export a git revision into ab/<name>/ and build its HIP library, for same-box A/B against the working
# tree (tools/ab_trees.sh):  tools/ab_rev.sh <name> <rev> [extra compiler flags]
set -e
NAME=$1; REV=$2; FLAGS=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
DST=$ROOT/ab/$NAME
rm -rf "$DST" && mkdir -p "$DST"
git -C "$ROOT" archive "$REV" | tar -x -C "$DST" --exclude=tests/golden
make -s -B -C "$DST/3dgaussian_amd/csrc" EXTRA="$FLAGS" >/dev/null
echo "built $DST from $(git -C "$ROOT" rev-parse --short "$REV") ($FLAGS)"
