#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, kernel-trace only) over tools/probe_view.py:
#   bash tools/pmc_passes.sh <outdir> [probe args]      (run on the GPU box; see profiles/README)
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/$OUT
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C -d $R/$OUT/p$i -o run --output-format csv -- python3 $R/tools/probe_view.py "$@" > $R/$OUT/p$i.log 2>&1
  i=$((i+1))
done
