# fp16 scan variants at Q=128/256 + parity.  usage: bash tools/gpu_f16b.sh <tag>
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-f16b}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for sp in 1 0; do
  for q in 128 256 1024; do
    MMR_KNN_F16_SPLIT=$sp timeout -k 10 120 python -u bench.py --mode knn --batch $q --steps 50 --warmup 5 --no-cpu-baseline > $OUT/b.json 2>>$OUT/err.log
    python -c "import json;d=json.load(open('$OUT/b.json'));print('split=$sp', $q, round(d['ms_per_step']*1e3,1),'us', round(d['value']/1e9,1),'Gpairs/s')"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o q256 -- python bench.py --mode knn --batch 256 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
