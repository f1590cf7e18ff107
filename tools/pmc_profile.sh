#!/bin/bash
# PMC passes over one bench step on the GPU box (one rocprofv3 run per counter group, --kernel-trace
# only, MI355X_MICROARCH.md §rocprofv3 PMC slots): HBM traffic (FETCH_SIZE, WRITE_SIZE) and the SQ
# counters behind valu_frac / mfma_frac, summarised by tools/pmc_summarize.py into <outdir>/pmc.json,
# stamped with the sha256 of 3dgaussian_amd/csrc/gr_hip.hip (bench.py reads profiles/pmc_traffic.json
# only when the stamp matches the tree).   bash tools/pmc_profile.sh <outdir> [extra bench args]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc $C -d $R/$OUT/p$i -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-extra-modes --no-dropin --no-psnr "$@" > $R/$OUT/p$i.log 2>&1
  i=$((i+1))
done
cd $R && python tools/pmc_summarize.py $OUT > $OUT/pmc_summary.txt
