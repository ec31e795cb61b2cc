# PMC passes (one rocprofv3 --pmc run each) over one GEMM shape under a pinned variant.
# usage: bash tools/gpu_pmc_gemm.sh <tag> M N K act variant
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o p -- python tools/pmc_gemm.py "$@" 5 > $OUT/p$i.log 2>&1 || { echo "FAIL pass $i"; tail -5 $OUT/p$i.log; exit 1; }
  f=$(find $OUT/p$i -name "*counter_collection.csv" | head -1)
  echo "== pass $i"; python tools/pmc_summary.py $f gemm_bf16_tn
done
