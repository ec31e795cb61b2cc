# PMC traffic passes (each counter in its own rocprofv3 run): HBM bytes (FETCH_SIZE x2 gfx950, WRITE_SIZE)
# of the kNN search at Q = 256 (p8 KNN scan + select) and Q = 16 (the lq scan + the RAW select: the
# cold-latency path), the LayerNorm-folded bf16 FFN1 (cfg2, the bench's roofline kernel: bench.py reads the
# latest profiles/rNN_pmc_traffic.json) and the fused MX-fp8 FFN1 (cfg5).
# usage (via gpurun): bash tools/gpu_pmc_traffic.sh <rNN>   -> gpurun_out/pmc_<rNN>/<rNN>_pmc_traffic.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=${1:-r06}
OUT=gpurun_out/pmc_$R; mkdir -p $OUT
run() {  # tag counters cmd...
  local tag=$1 cnt=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $cnt --output-format csv -d $OUT/$tag -o p -- "$@" > $OUT/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 $OUT/$tag.log; exit 1; }
  find $OUT/$tag -name "*counter_collection.csv" | head -1
}
KF=$(run knn_f FETCH_SIZE python3 tools/knn_sweep.py --qs 256 --rounds 1 --reps 5 --variants f16) || exit 1
KW=$(run knn_w WRITE_SIZE python3 tools/knn_sweep.py --qs 256 --rounds 1 --reps 5 --variants f16) || exit 1
SF=$(run k16_f FETCH_SIZE python3 tools/knn_sweep.py --qs 16 --rounds 1 --reps 5 --variants f16) || exit 1
SW=$(run k16_w WRITE_SIZE python3 tools/knn_sweep.py --qs 16 --rounds 1 --reps 5 --variants f16) || exit 1
FF=$(run fold_f FETCH_SIZE python3 tools/pmc_ffn1.py fold) || exit 1
FW=$(run fold_w WRITE_SIZE python3 tools/pmc_ffn1.py fold) || exit 1
XF=$(run mx8_f FETCH_SIZE python3 tools/pmc_ffn1.py mx8) || exit 1
XW=$(run mx8_w WRITE_SIZE python3 tools/pmc_ffn1.py mx8) || exit 1
python3 tools/pmc_traffic.py $OUT/${R}_pmc_traffic.json "$R: tools/gpu_pmc_traffic.sh" \
  knn_scan_p8=$KF,$KW,gemm_bf16_tn_p8 knn_select_f16=$KF,$KW,knn_select_t knn_prep=$KF,$KW,knn_prep_queries \
  knn16_scan_lq=$SF,$SW,knn_scan_f16_lq knn16_select_raw=$SF,$SW,knn_select_t \
  "bert_ffn1_ln_fold=$FF,$FW,gemm_bf16_tn_p8<4, 1, true, false, false, false, 0, 1" "bert_ffn1_mx8=$XF,$XW,gemm_bf16_tn_p8<4, 1, true, false, true, true" || exit 1
cat $OUT/${R}_pmc_traffic.json
