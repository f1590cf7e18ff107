#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench, rocprofv3 kernel stats, PMC HBM traffic.  Usage: bash tools/gpu_round.sh <tag>
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/$TAG
mkdir -p $R/$O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
# single-stream run: kernel durations are each launch's own and agree with the bench's roofline fields
GR_STREAMS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/stats -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/$O/bench_prof.log 2>&1
# the bench as run (3 streams): the same kernels, with other views' kernels beside them
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/stats_streams -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/$O/bench_prof_streams.log 2>&1
cd $R && bash tools/pmc_bench.sh $O/pmc
