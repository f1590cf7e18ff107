#!/bin/bash
# rocprofv3 kernel statistics + kernel trace of (a) the drop-in op as the reference loop calls it
# (tools/dropin_run.py) and (b) the bench including its default-precision (depth-loss) and f32-grade steps.
#   bash tools/prof_modes.sh <tag>
set -e
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dropin -o run --output-format csv -- python3 $R/tools/dropin_run.py 2 1 > $O/dropin.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/modes -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dropin --no-psnr > $O/modes.log 2>&1
cd $R && python tools/kstats.py $O/dropin > $O/kernel_stats_dropin.txt && python tools/busy.py $O/dropin >> $O/kernel_stats_dropin.txt
python tools/kstats.py $O/modes > $O/kernel_stats_modes.txt
