#!/bin/bash
# Round-3 closing pass on the GPU box: stamped PMC passes (copied to profiles/pmc_traffic.json so the
# bench reads them), rocprofv3 kernel stats of the bench (1 and 4 streams), the GPU tests, smoke, the
# driver's bench command, and the other configs (Python schedule vs native executor).
#   bash tools/gpu_final_r03.sh <tag>
set -e
TAG=${1:-r03f}
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/pmc_profile.sh gpurun_out/$TAG/pmc
cp $O/pmc/pmc.json $R/profiles/pmc_traffic.json
cd /tmp && export TMPDIR=/tmp
GR_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats1 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra-modes --no-dropin --no-psnr > $O/bench_prof1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats4 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra-modes --no-dropin --no-psnr > $O/bench_prof4.log 2>&1
cd $R && python tools/kstats.py $O/stats1 > $O/kernel_stats_1stream.txt && python tools/kstats.py $O/stats4 > $O/kernel_stats_4streams.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
for e in "GR_NATIVE_EXEC=0" "GR_NATIVE_EXEC=1"; do
  echo "$e" >> $O/configs.txt
  env $e timeout -k 10 300 python tools/bench_configs.py C2 C3 >> $O/configs.txt 2>/dev/null
done
