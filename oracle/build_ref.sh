#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.  Compiles the reference's CPU renderer from its sources where they lie
# (/root/reference/src/renderer_cpu.cpp, renderer_dispatch.cpp) plus our ref_shim.cpp into
# oracle/_ref/libref.so.  No reference source is copied; outputs stay in oracle/_ref/ (git-ignored).
# The reference's CUDA path (src/renderer.cu) is not buildable here (no nvcc) and is not needed.
set -euo pipefail
REF=${GR_REFERENCE:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
if [ ! -f "$REF/src/renderer_cpu.cpp" ]; then
  echo "reference not present at $REF; skipping oracle/_ref build" >&2
  exit 0
fi
mkdir -p "$HERE/_ref"
g++ -O3 -std=c++17 -shared -fPIC -DGR_CUDA_ENABLED=0 -I"$REF/include" \
  "$REF/src/renderer_cpu.cpp" "$REF/src/renderer_dispatch.cpp" "$HERE/ref_shim.cpp" \
  -o "$HERE/_ref/libref.so"
echo "built $HERE/_ref/libref.so"
