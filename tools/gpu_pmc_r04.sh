# Round-4 PMC passes (each counter group in its own rocprofv3 run): HBM traffic (FETCH_SIZE,
# WRITE_SIZE) and SQ busy counters for the kernels the timed steps run — the kNN search at Q=256 (p8
# KNN scan + select), the LayerNorm-folded bf16 FFN1 (cfg2) and the fused MX-fp8 FFN1 (cfg5).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_r04; mkdir -p $OUT
run() {  # tag counters cmd...
  local tag=$1 cnt=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $cnt --output-format csv -d $OUT/$tag -o p -- "$@" > $OUT/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 $OUT/$tag.log; exit 1; }
  find $OUT/$tag -name "*counter_collection.csv" | head -1
}
KF=$(run knn_f FETCH_SIZE python3 tools/knn_sweep.py --qs 256 --rounds 1 --reps 5 --variants f16) || exit 1
KW=$(run knn_w WRITE_SIZE python3 tools/knn_sweep.py --qs 256 --rounds 1 --reps 5 --variants f16) || exit 1
FF=$(run fold_f FETCH_SIZE python3 tools/pmc_ffn1.py fold) || exit 1
FW=$(run fold_w WRITE_SIZE python3 tools/pmc_ffn1.py fold) || exit 1
XF=$(run mx8_f FETCH_SIZE python3 tools/pmc_ffn1.py mx8) || exit 1
XW=$(run mx8_w WRITE_SIZE python3 tools/pmc_ffn1.py mx8) || exit 1
python3 tools/pmc_traffic.py $OUT/r04_pmc_traffic.json "r04: tools/gpu_pmc_r04.sh" \
  knn_scan_p8=$KF,$KW,gemm_bf16_tn_p8 knn_select_f16=$KF,$KW,knn_select_t knn_prep=$KF,$KW,knn_prep_queries \
  "bert_ffn1_ln_fold=$FF,$FW,gemm_bf16_tn_p8<4, 1, true, false, false, false, 0, 1" "bert_ffn1_mx8=$XF,$XW,gemm_bf16_tn_p8<4, 1, true, false, true, true" || exit 1
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
for m in fold mx8; do
  f=$(run sq_$m "$SQ" python3 tools/pmc_ffn1.py $m) || exit 1
  k=$([ $m = fold ] && echo "gemm_bf16_tn_p8<4, 1, true, false, false, false, 0, 1" || echo "gemm_bf16_tn_p8<4, 1, true, false, true, true")
  echo "== SQ $m"; python3 tools/pmc_summary.py $f "$k"
done
G="GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU"
for m in fold mx8; do
  f=$(run g_$m "$G" python3 tools/pmc_ffn1.py $m) || exit 1
  k=$([ $m = fold ] && echo "gemm_bf16_tn_p8<4, 1, true, false, false, false, 0, 1" || echo "gemm_bf16_tn_p8<4, 1, true, false, true, true")
  echo "== GRBM $m"; python3 tools/pmc_summary.py $f "$k"
done
cat $OUT/r04_pmc_traffic.json
