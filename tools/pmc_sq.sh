set -e
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/pmcq
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $R/gpurun_out/pmcq/p1 -o run --output-format csv -- python3 $R/tools/ab_raster.py 1000000 800 4 > $R/gpurun_out/pmcq/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_MFMA -d $R/gpurun_out/pmcq/p2 -o run --output-format csv -- python3 $R/tools/ab_raster.py 1000000 800 4 > $R/gpurun_out/pmcq/p2.log 2>&1
