#!/bin/bash
# Kernel-trace timeline (gaps + durations) of kNN-only bench runs at a few batch sizes.
# usage (via gpurun): bash tools/gpu_knn_timeline.sh <tag> [batches...]
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-tl}; shift || true
BATCHES=${@:-16 256}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for b in $BATCHES; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tl$b -o k \
    -- python3 bench.py --mode knn --batch $b --steps 10 --warmup 2 --no-cpu-baseline > $OUT/tl$b.log 2>&1
  f=$(find $OUT/tl$b -name "*kernel_trace.csv" | head -1)
  python3 tools/csv_timeline.py $f 24 > $OUT/timeline_q$b.txt
  cat $OUT/timeline_q$b.txt
done
