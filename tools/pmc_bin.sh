#!/bin/bash
# PMC passes over tools/bin_bench.py (the binning alone), one rocprofv3 run per counter group, --kernel-trace only;
# summarised per kernel by tools/pmc_summarize.py.   bash tools/pmc_bin.sh <outdir> [tree (default: this one)]
set -e
OUT=${1:-gpurun_out/pmc_bin}
R=${GRAFT_REPO_ROOT:-$PWD}
TREE=$(cd ${2:-$R} && pwd)
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --pmc $C -d $R/$OUT/p$i -o run --output-format csv -- python3 $TREE/tools/bin_bench.py 10 > $R/$OUT/p$i.log 2>&1
  i=$((i+1))
done
cd $R && python tools/pmc_summarize.py $OUT > $OUT/pmc_summary.txt
