#!/bin/bash
# Session-5 A/B: attention occupancy bounds (this tree vs tools/ab/libmmr_prev.so), same box.
# usage (via gpurun): bash tools/gpu_s5_ab.sh <tag>
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-s5ab}; mkdir -p $OUT
OLD=$GRAFT_REPO_ROOT/tools/ab/libmmr_prev.so
timeout -k 10 400 python -u -m pytest tests/test_towers_gpu.py tests/test_fusion_gpu.py tests/test_mxfp8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pyt.log 2>&1 || { tail -30 $OUT/pyt.log; exit 1; }
tail -1 $OUT/pyt.log
for i in 1 2; do
  for q in 0 1; do
    SWA_Q8=$q timeout -k 10 120 python -u tools/swa_bench.py "new q8=$q" 2>/dev/null | grep -v amdgpu
    SWA_Q8=$q MMR_LIBMMR=$OLD timeout -k 10 120 python -u tools/swa_bench.py "old q8=$q" 2>/dev/null | grep -v amdgpu
  done
  echo "== mha dh128 new"; MHA_D=1024 MHA_B=512 timeout -k 10 120 python -u tools/mha_bench.py 2>/dev/null | grep -v "amdgpu\|bert"
  echo "== mha dh128 old"; MHA_D=1024 MHA_B=512 MMR_LIBMMR=$OLD timeout -k 10 120 python -u tools/mha_bench.py 2>/dev/null | grep -v "amdgpu\|bert"
done
for i in 1 2; do for L in new old; do
  if [ $L = new ]; then E=X=0; else E=MMR_LIBMMR=$OLD; fi
  env $E timeout -k 10 500 python -u bench.py --preset cfg5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/cfg5ab.json 2> $OUT/cfg5ab.err
  python -c "import json;d=json.load(open('$OUT/cfg5ab.json'));print('cfg5 $L', round(d['ms_per_step'],3), round(d['value']))"
  env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/cfg2ab.json 2> $OUT/cfg2ab.err
  python -c "import json;d=json.load(open('$OUT/cfg2ab.json'));print('cfg2 $L', round(d['ms_per_step'],3), round(d['value']))"
done; done
