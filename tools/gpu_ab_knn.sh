#!/bin/bash
# kNN A/B: knn GPU tests, then the kNN-only bench per env setting (hbm_regime + Q=256 search time).
# usage (via gpurun): bash tools/gpu_ab_knn.sh <tag> "<ENV=..>" ["<ENV=..>" ...]
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py tests/test_sharded_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for e in "$@"; do
  env $e timeout -k 10 200 python -u bench.py --mode knn --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $OUT/b.json 2> $OUT/b.err
  python3 -c "
import json,sys; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']
h=r['hbm_regime']; print('$e', 'Q256 ms %.4f frac %.3f | Q16 ms %.4f frac %.3f | single %.4f' % (r['ms_per_launch'], r['frac'], h['ms_per_search'], h['frac'], h.get('latency_ms_single') or 0))"
done
