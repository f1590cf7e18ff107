#!/bin/bash
# Round-5 GPU passes on the box (each step under its own time limit; the first failure ends the call).
#   bash tools/gpu_r05.sh <tag> <step>...
# steps: bench (20-step driver command), stats1 / stats4 (rocprofv3 kernel stats of the bench, 1 / 4 streams),
#        dropin (rocprofv3 kernel stats of the drop-in loop), tests (pytest -m gpu), smoke, configs (C2 C3),
#        pmc (stamped PMC passes -> profiles/pmc_traffic.json)
set -eo pipefail
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    bench)
      (cd $R && timeout -k 10 500 python bench.py > $O/bench.log 2>&1) ;;
    benchq)
      (cd $R && timeout -k 10 300 python bench.py --no-cpu-baseline --no-psnr > $O/benchq.log 2>&1) ;;
    stats1)
      (cd /tmp && GR_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats1 -o run --output-format csv -- \
        python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extra-modes --no-dropin --no-psnr > $O/bench_prof1.log 2>&1)
      (cd $R && python tools/kstats.py $O/stats1 > $O/kernel_stats_1stream.txt) ;;
    stats4)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats4 -o run --output-format csv -- \
        python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extra-modes --no-dropin --no-psnr > $O/bench_prof4.log 2>&1)
      (cd $R && python tools/kstats.py $O/stats4 > $O/kernel_stats_4streams.txt) ;;
    dropin)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dropin -o run --output-format csv -- \
        python3 $R/tools/dropin_run.py > $O/dropin.log 2>&1)
      (cd $R && python tools/kstats.py $O/dropin > $O/kernel_stats_dropin.txt) ;;
    tests)
      (cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1) ;;
    smoke)
      (cd $R && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1) ;;
    configs)
      (cd $R && timeout -k 10 300 python tools/bench_configs.py C2 C3 --steps 20 > $O/configs.txt 2>$O/configs.err) ;;
    configs5)
      (cd $R && timeout -k 10 400 python tools/bench_configs.py C5 C5d --steps 6 > $O/configs5.txt 2>$O/configs5.err) ;;
    c3prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3 -o run --output-format csv -- \
        python3 $R/tools/bench_configs.py C3 > $O/c3prof.log 2>&1)
      (cd $R && python tools/kstats.py $O/c3 > $O/kernel_stats_c3.txt) ;;
    c4dprof)
      (cd /tmp && GR_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4d -o run --output-format csv -- \
        python3 $R/tools/bench_configs.py C4d --steps 2 --warmup 1 > $O/c4dprof.log 2>&1)
      (cd $R && python tools/kstats.py $O/c4d > $O/kernel_stats_c4d.txt) ;;
    c4dstreams)  # the depth-loss mode at 1, 2 and 4 HIP streams
      for ns in 1 2 4; do
        (cd $R && GR_STREAMS=$ns timeout -k 10 300 python tools/bench_configs.py C4d --steps 4 --warmup 2 >> $O/c4d_streams.txt 2>>$O/c4d_streams.err)
      done ;;
    pmc)
      (cd $R && bash tools/pmc_profile.sh gpurun_out/$TAG/pmc && cp $O/pmc/pmc.json $R/profiles/pmc_traffic.json) ;;
    ab:*)  # ab:<rounds>:<dir>,<dir>... same-box bench A/B of tree copies (tools/ab_bench.sh)
      IFS=: read -r _ n dirs <<< "$step"
      (cd $R && bash tools/ab_bench.sh $TAG $n ${dirs//,/ } > $O/ab.txt 2>&1) ;;
    abdrop:*)  # abdrop:<rounds>:<dir>,<dir>... same-box A/B of the drop-in loop (tools/dropin_run.py) between tree copies
      IFS=: read -r _ n dirs <<< "$step"
      for r in $(seq 1 $n); do
        for d in ${dirs//,/ }; do
          (cd $R/$d && timeout -k 10 240 python tools/dropin_run.py 3 1 > $O/abdrop_$(basename $(cd $R/$d && pwd))_$r.log 2>&1)
          echo "$(basename $(cd $R/$d && pwd)) round $r: $(grep '^{' $O/abdrop_$(basename $(cd $R/$d && pwd))_$r.log)" >> $O/abdrop.txt
        done
      done ;;
    testk:*)  # testk:<pytest -k expression> a subset of the GPU tests
      (cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s -k "${step#testk:}" > $O/pytest_gpu_k.log 2>&1) ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
