#!/bin/bash
# Session-end GPU pass: GPU tests, smoke, bench lines (cfg2 full + kNN, cfg3, cfg5), rocprofv3 kernel
# stats of cfg2 (towers in sequence) and of the kNN leg, kNN PMC traffic; x3 counters / step table (pmcx3,
# x3prof) and the roofline kernels' traffic (pmct).  Each GPU step has its own
# time limit; the first failing step ends the script.
# usage (via gpurun): bash tools/gpu_final.sh <tag> [steps...]
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-final}; shift || true
STEPS=${@:-tests smoke bench presets prof pmck}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
      tail -2 $OUT/tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
      tail -1 $OUT/smoke.log ;;
    bench)
      timeout -k 10 300 python -u bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err
      timeout -k 10 300 python -u bench.py --mode knn > $OUT/bench_knn.json 2> $OUT/bench_knn.err
      echo bench ok ;;
    presets)
      timeout -k 10 900 python -u bench.py --preset cfg3 --steps 5 --warmup 2 > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err
      timeout -k 10 800 python -u bench.py --preset cfg5 --steps 5 --warmup 2 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err
      echo presets ok ;;
    cfg3)  # closing cfg3 record: cpu_baseline, recall_vs_cpu, p_at_10 and the x3 parity line filled in
      timeout -k 10 900 python -u bench.py --preset cfg3 --steps 5 --warmup 2 > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err
      echo cfg3 ok ;;
    cfg5)
      timeout -k 10 800 python -u bench.py --preset cfg5 --steps 5 --warmup 2 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err
      echo cfg5 ok ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o full \
        -- python3 bench.py --sequential-towers --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_full.log 2>&1
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o knn \
        -- python3 bench.py --sequential-towers --mode knn --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof_knn.log 2>&1
      echo prof ok ;;
    prof5)  # cfg5 kernel stats, towers / fusion in sequence
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o cfg5 \
        -- python3 bench.py --sequential-towers --preset cfg5 --steps 3 --warmup 2 --no-cpu-baseline > $OUT/prof_cfg5.log 2>&1
      echo prof5 ok ;;
    pmck)
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc -o kfetch \
        -- python3 bench.py --sequential-towers --mode knn --steps 5 --warmup 1 --no-cpu-baseline > $OUT/pmc_kfetch.log 2>&1
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc -o kwrite \
        -- python3 bench.py --sequential-towers --mode knn --steps 5 --warmup 1 --no-cpu-baseline > $OUT/pmc_kwrite.log 2>&1
      echo pmc ok ;;
    pmcx3)  # x3 kernels' counters (tools/pmc_x3.py) -> gpurun_out/pmc_<tag>/pmc_x3.json
      bash tools/gpu_pmc_x3.sh $TAG > $OUT/pmc_x3.log 2>&1 || { tail -5 $OUT/pmc_x3.log; exit 1; }
      echo pmcx3 ok ;;
    pmct)   # HBM traffic of the roofline kernels -> gpurun_out/pmc_r06/r06_pmc_traffic.json
      bash tools/gpu_pmc_traffic.sh r06 > $OUT/pmc_traffic.log 2>&1 || { tail -5 $OUT/pmc_traffic.log; exit 1; }
      echo pmct ok ;;
    x3prof) # one sequential x3 cfg2 step, per-kernel table
      bash tools/gpu_x3_prof.sh $TAG > $OUT/x3prof.log 2>&1 || { tail -5 $OUT/x3prof.log; exit 1; }
      echo x3prof ok ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
