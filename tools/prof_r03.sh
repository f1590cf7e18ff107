#!/bin/bash
# Profiling pass on the GPU box (round 3): same-box A/B of environment settings, rocprofv3 kernel stats of
# the bench (single stream and as run, with the kernel trace of the 4-stream run for tools/busy.py), and
# the stamped PMC passes (tools/pmc_profile.sh).  Usage: bash tools/prof_r03.sh <tag> "<env sets>" [steps]
set -e
TAG=${1:-r03}; SETS=${2:-"GR_GATHER=1"}; STEPS=${3:-20}
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/ab_env.sh "$SETS" 2 --steps $STEPS --warmup 3 --no-dropin --no-psnr > $O/ab_env.txt 2>&1
cd /tmp && export TMPDIR=/tmp
GR_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats1 -o run --output-format csv -- python3 $R/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-extra-modes --no-dropin --no-psnr > $O/bench_prof1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats4 -o run --output-format csv -- python3 $R/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-extra-modes --no-dropin --no-psnr > $O/bench_prof4.log 2>&1
cd $R && python tools/kstats.py $O/stats1 > $O/kernel_stats_1stream.txt && python tools/kstats.py $O/stats4 > $O/kernel_stats_4streams.txt

cd $R && python tools/overlap.py $O/stats4 > $O/overlap_4streams.txt
bash tools/pmc_profile.sh gpurun_out/$TAG/pmc
