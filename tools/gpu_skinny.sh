set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-skinny}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for q in 1 8 16 32 64 128 256; do
  timeout -k 10 120 python -u bench.py --mode knn --batch $q --steps 50 --warmup 5 --no-cpu-baseline >> $OUT/qsweep.jsonl 2>>$OUT/qsweep.err
done
for q in ${OLDQ:-}; do
  MMR_KNN_SKINNY_MAX=0 timeout -k 10 120 python -u bench.py --mode knn --batch $q --steps 50 --warmup 5 --no-cpu-baseline >> $OUT/qsweep_old.jsonl 2>>$OUT/qsweep.err
done
python -c "
import json
import os
for f in [x for x in ['qsweep','qsweep_old'] if os.path.exists('$OUT/'+x+'.jsonl')]:
  for l in open('$OUT/'+f+'.jsonl'):
    d=json.loads(l); print(f, d['config']['global_batch'], round(d['ms_per_step']*1e3,1),'us', d['roofline'].get('achieved'), d['roofline'].get('unit'))
"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o q16 -- python bench.py --mode knn --batch 16 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o q1 -- python bench.py --mode knn --batch 1 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof1.log 2>&1
ls -R $OUT/prof | head
