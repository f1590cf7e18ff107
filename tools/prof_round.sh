set -e
R=$PWD
mkdir -p gpurun_out/r01f
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r01f/stats -o run --output-format csv rocpd -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/r01f/bench_prof.log 2>&1
cd $R && timeout -k 10 300 python bench.py > gpurun_out/r01f/bench.log 2>&1
bash tools/pmc_bench.sh gpurun_out/r01f/pmc
