# rocprofv3 kernel-trace + stats over a short bench run; writes the per-kernel table.
# usage: bash tools/gpu_prof_bench.sh <tag> [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/prof_$TAG; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o k -- python3 bench.py --no-cpu-baseline "$@" > $OUT/bench.log 2>&1 || { echo "FAIL"; tail -5 $OUT/bench.log; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 tools/prof_csv_summary.py $f $OUT/stats.txt > /dev/null && head -45 $OUT/stats.txt
