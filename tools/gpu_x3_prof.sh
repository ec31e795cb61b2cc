# rocprofv3 kernel trace of the x3 (fp32-faithful) cfg2 step with towers in sequence: per-kernel step
# table + launch list of one steady-state step.  usage: bash tools/gpu_x3_prof.sh <tag> [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/x3prof_$TAG; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT -o k -- python3 bench.py --no-cpu-baseline --tower-dtype x3 --sequential-towers --steps 4 --warmup 2 "$@" > $OUT/bench.log 2>&1 || { echo "FAIL"; tail -5 $OUT/bench.log; exit 1; }
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 tools/step_kernels.py $f 3 > $OUT/step_kernels.txt && python3 tools/step_list.py $f 3 > $OUT/step_list.txt && head -40 $OUT/step_kernels.txt
rm -f $f
