#!/bin/bash
# rocprofv3 kernel statistics of the bench at the driver's step count: single stream (each launch's own
# duration, comparable to the bench's roofline timing) and as run (3 streams), plus the kernel trace of
# the 3-stream run for tools/busy.py.  Usage: bash tools/prof_r02.sh <tag> [steps] [warmup]
set -e
TAG=${1:-r02}; STEPS=${2:-20}; WARM=${3:-5}
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
GR_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats1 -o run --output-format csv -- python3 $R/bench.py --steps $STEPS --warmup $WARM --no-cpu-baseline --no-extra-modes > $O/bench_prof1.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats4 -o run --output-format csv -- python3 $R/bench.py --steps $STEPS --warmup $WARM --no-cpu-baseline --no-extra-modes > $O/bench_prof3.log 2>&1
cd $R && python tools/kstats.py $O/stats1 > $O/kernel_stats_1stream.txt && python tools/kstats.py $O/stats4 > $O/kernel_stats_4streams.txt
