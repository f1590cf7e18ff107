set -e
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/r03s1; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
GR_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/depth1 -o run --output-format csv -- python3 $R/tools/depth_mode_run.py 2 50 > $O/depth1.log 2>&1
cd $R && python tools/kstats.py $O/depth1 > $O/kstats_depth1.txt
