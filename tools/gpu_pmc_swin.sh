#!/bin/bash
# SQ counter passes over the fused Swin stage-1/2 kernels (tools/mlp_bench.py: swin_mlp_res C=96,
# swin_mlp C=192) — where their time goes (VALU / MFMA busy, waits).  One rocprofv3 --pmc run per pass.
# usage (via gpurun): bash tools/gpu_pmc_swin.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o p -- python3 ${PMC_PY:-tools/mlp_bench.py} > $OUT/p$i.log 2>&1 || { echo "FAIL pass $i"; tail -5 $OUT/p$i.log; exit 1; }
  f=$(find $OUT/p$i -name "*counter_collection.csv" | head -1)
  for k in ${PMC_KERNELS:-swin_mlp_res<96 swin_mlp<192}; do echo "== pass $i $k"; python3 tools/pmc_summary.py $f "$k"; done
done
