#!/bin/bash
# One GPU-box pass: parity tests, benches, rocprofv3 kernel stats, PMC HBM-traffic pass.
# usage (from the repo root, via gpurun): bash tools/gpu_round.sh <tag> [tests|bench|prof|pmc ...]
# Each GPU step has its own time limit; the first failing step ends the script.
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}; shift || true
STEPS=${@:-tests bench prof pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
      tail -3 "$OUT/tests.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      tail -2 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 300 python -u bench.py > "$OUT/bench_full.json" 2> "$OUT/bench_full.err"
      cat "$OUT/bench_full.json"
      timeout -k 10 300 python -u bench.py --mode knn > "$OUT/bench_knn.json" 2> "$OUT/bench_knn.err"
      cat "$OUT/bench_knn.json" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o full \
        -- python bench.py --sequential-towers --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_full.log" 2>&1
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o knn \
        -- python bench.py --sequential-towers --mode knn --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/prof_knn.log" 2>&1
      ls -R "$OUT/prof" | head -20 ;;
    pmc)
      # HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes (TCC slot budget)
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o fetch \
        -- python bench.py --sequential-towers --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc" -o write \
        -- python bench.py --sequential-towers --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o kfetch \
        -- python bench.py --sequential-towers --mode knn --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_kfetch.log" 2>&1
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc" -o kwrite \
        -- python bench.py --sequential-towers --mode knn --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_kwrite.log" 2>&1
      ls -R "$OUT/pmc" | head -20 ;;
    pmck)
      # kNN-mode HBM traffic only (default scan mode), FETCH_SIZE and WRITE_SIZE in separate passes
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o kfetch \
        -- python bench.py --sequential-towers --mode knn --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_kfetch.log" 2>&1
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc" -o kwrite \
        -- python bench.py --sequential-towers --mode knn --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_kwrite.log" 2>&1
      ls -R "$OUT/pmc" | head -20 ;;
    pmcg)
      # FFN1 GEMM traffic per candidate launch variant (the tuner's pick varies by box)
      for v in 0 1 2 7; do
        for c in FETCH_SIZE WRITE_SIZE; do
          timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmcg" -o "v${v}_$c" \
            -- python tools/pmc_gemm.py 32768 3072 768 1 $v > "$OUT/pmcg_v${v}_$c.log" 2>&1
        done
      done
      ls "$OUT/pmcg" | head -20 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
