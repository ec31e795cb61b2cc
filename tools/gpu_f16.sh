# fp16 scan mode: parity tests + Q sweep (both modes).  usage: bash tools/gpu_f16.sh <tag>
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-f16}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for m in f16 x3; do
  for q in ${QS:-1 16 64 256 1024}; do
    timeout -k 10 120 python -u bench.py --mode knn --knn-mode $m --batch $q --steps 50 --warmup 5 --no-cpu-baseline >> $OUT/qsweep_$m.jsonl 2>>$OUT/qsweep.err
  done
done
python - <<PY
import json
for m in ['f16','x3']:
    for l in open('$OUT/qsweep_%s.jsonl' % m):
        d = json.loads(l); print(m, d['config']['global_batch'], round(d['ms_per_step'] * 1e3, 1), 'us', round(d['value'] / 1e9, 1), 'Gpairs/s')
PY
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o f16q256 -- python bench.py --mode knn --knn-mode f16 --batch 256 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o f16q16 -- python bench.py --mode knn --knn-mode f16 --batch 16 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof2.log 2>&1
ls $OUT/prof
