# Fresh HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs) for the round-3 kernels:
# the kNN search at Q=256 (f16 tile scan + select) and the BERT FFN1 / QKV GEMMs under their tuned
# persistent 8-phase variants (9: 256x256, 10: 256x192).  Output: profiles-ready JSON.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_r03; mkdir -p $OUT
run() {  # tag counter cmd...
  local tag=$1 cnt=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $cnt --output-format csv -d $OUT/$tag -o p -- "$@" > $OUT/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 $OUT/$tag.log; exit 1; }
  find $OUT/$tag -name "*counter_collection.csv" | head -1
}
KF=$(run knn_f FETCH_SIZE python3 tools/knn_sweep.py --qs 256 --rounds 1 --reps 5 --variants f16) || exit 1
KW=$(run knn_w WRITE_SIZE python3 tools/knn_sweep.py --qs 256 --rounds 1 --reps 5 --variants f16) || exit 1
GF=$(run ffn1_f FETCH_SIZE python3 tools/pmc_gemm.py 32768 3072 768 1 9 5) || exit 1
GW=$(run ffn1_w WRITE_SIZE python3 tools/pmc_gemm.py 32768 3072 768 1 9 5) || exit 1
QF=$(run qkv_f FETCH_SIZE python3 tools/pmc_gemm.py 32768 2304 768 0 10 5) || exit 1
QW=$(run qkv_w WRITE_SIZE python3 tools/pmc_gemm.py 32768 2304 768 0 10 5) || exit 1
python3 tools/pmc_traffic.py $OUT/r03_pmc_traffic.json "r03: tools/gpu_pmc_traffic_r03.sh" \
  knn_scan_p8=$KF,$KW,gemm_bf16_tn_p8 knn_select_f16=$KF,$KW,knn_select_t knn_prep=$KF,$KW,knn_prep_queries \
  bert_ffn1_v9=$GF,$GW,gemm_bf16_tn_p8 bert_qkv_v10=$QF,$QW,gemm_bf16_tn_p8
cp $OUT/r03_pmc_traffic.json profiles/ 2>/dev/null; cat $OUT/r03_pmc_traffic.json
