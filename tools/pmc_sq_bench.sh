#!/bin/bash
# SQ counter passes over one bench step (one rocprofv3 run per counter group, kernel-trace only), for
# the per-kernel wave/VALU/LDS/VMEM picture:  bash tools/pmc_sq_bench.sh <outdir>   (GPU box)
set -e
OUT=${1:-gpurun_out/pmc_sq}
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d $R/$OUT/p$i -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra-modes > $R/$OUT/p$i.log 2>&1
  i=$((i+1))
done
