#!/bin/bash
TAG=${1:-ab}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
grep '^{' $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['roofline']['avg_launch_us'], d['roofline']['fwd_kernel_avg_us'])"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/stats -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/bench_prof.log 2>&1
cd $R && python tools/kstats.py $O/stats | head -24
