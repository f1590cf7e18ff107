#!/bin/bash
# HBM traffic of the bench's kernels: separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over one
# bench step, summarised into profiles/pmc_traffic.json by tools/pmc_traffic.py (MI355X_MICROARCH.md
# HBM/rocprofv3 section: KiB units, gfx950 wide-read halving).  Run on the GPU box.
set -e
OUT=${1:-gpurun_out/pmc_bench}
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/$OUT/fetch -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $R/$OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/$OUT/write -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $R/$OUT/write.log 2>&1
cd $R && python tools/pmc_traffic.py $OUT/fetch $OUT/write $OUT/pmc_traffic.json > /dev/null  # copy into profiles/
