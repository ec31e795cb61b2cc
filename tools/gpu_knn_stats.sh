#!/bin/bash
# rocprofv3 kernel stats of kNN-only bench runs: bash tools/gpu_knn_stats.sh <tag> "<bench args>" ...
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$i -o k \
    -- python3 bench.py --mode knn --steps 10 --warmup 2 --no-cpu-baseline $a > $OUT/p$i.log 2>&1
  f=$(find $OUT/p$i -name "*kernel_stats.csv" | head -1)
  echo "== $a"; python3 tools/prof_csv_summary.py $f $OUT/stats$i.txt > /dev/null; head -12 $OUT/stats$i.txt
done
