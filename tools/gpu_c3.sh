set -e
R=${GRAFT_REPO_ROOT:-$PWD}; O=$R/gpurun_out/c3b; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_fit_exec_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_exec.log 2>&1
timeout -k 10 300 python tools/bench_configs.py C2 C3 --steps 10 > $O/configs_auto.txt 2>/dev/null
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c3trace -o run --output-format csv -- python3 $R/tools/bench_configs.py C3 --steps 8 > $O/c3trace.log 2>&1
cd $R && python tools/step_timeline.py $O/c3trace > $O/c3_timeline.txt
