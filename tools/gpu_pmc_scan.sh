# PMC (SQ) counters of the kNN scan kernels, one rocprofv3 --pmc pass per variant.
# usage: bash tools/gpu_pmc_scan.sh <tag> <Q> <variant...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pmc}; Q=${2:-256}; shift 2; mkdir -p $OUT
CNT="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
for v in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc $CNT --output-format csv -d $OUT/$v -o p -- python tools/knn_sweep.py --qs $Q --rounds 1 --reps 5 --variants $v > $OUT/$v.log 2>&1 || { echo "FAIL $v"; tail -5 $OUT/$v.log; exit 1; }
  f=$(find $OUT/$v -name "*counter_collection.csv" | head -1)
  echo "== $v"; python tools/pmc_summary.py $f knn_scan
done
