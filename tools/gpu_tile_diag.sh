# Tile-scan diagnostics: per-kernel times for the f16 tile scan with / without its gallery or query
# loads (MMR_KNN_F16_TILE_DBG), rocprofv3 kernel trace.  usage: bash tools/gpu_tile_diag.sh <tag> [Q]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-diag}; mkdir -p $OUT
Q=${2:-256}
for v in f16 f16_noB f16_noA f16_stream; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/$v -o p -- python tools/knn_sweep.py --qs $Q --rounds 1 --reps 10 --variants $v > $OUT/$v.log 2>&1 || { echo "FAIL $v"; tail -5 $OUT/$v.log; exit 1; }
  echo "== $v"; python tools/prof_summary.py $(find $OUT/$v -name "*.db" | head -1) | head -6
done
