set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/s5g; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_towers_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pyt.log 2>&1 || { tail -30 $OUT/pyt.log; exit 1; }
tail -1 $OUT/pyt.log
for i in 1 2; do
  for q in 0 1; do
    SWA_Q8=$q timeout -k 10 120 python -u tools/swa_bench.py "new q8=$q" 2>/dev/null | grep -v amdgpu
    SWA_Q8=$q MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/libmmr_s5.so timeout -k 10 120 python -u tools/swa_bench.py "old q8=$q" 2>/dev/null | grep -v amdgpu
  done
done
