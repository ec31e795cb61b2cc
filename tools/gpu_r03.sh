#!/bin/bash
# Round-3 GPU pass.  usage (via gpurun): bash tools/gpu_r03.sh <tag> [steps...]
# Each GPU step has its own time limit; the first failing step ends the script.
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03}; shift || true
STEPS=${@:-tests smoke bench}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 1050 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
      tail -3 $OUT/tests.log ;;
    testsx)  # a subset: TESTS env = pytest node ids / -k expression file list
      timeout -k 10 1050 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread > $OUT/testsx.log 2>&1 || { tail -40 $OUT/testsx.log; exit 1; }
      tail -3 $OUT/testsx.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
      tail -1 $OUT/smoke.log ;;
    bench)
      timeout -k 10 400 python -u bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err
      cat $OUT/bench_full.json ;;
    benchknn)
      timeout -k 10 300 python -u bench.py --mode knn > $OUT/bench_knn.json 2> $OUT/bench_knn.err
      cat $OUT/bench_knn.json ;;
    presets)
      timeout -k 10 400 python -u bench.py --preset cfg3 --steps 5 --warmup 2 > $OUT/bench_cfg3.json 2> $OUT/bench_cfg3.err
      timeout -k 10 500 python -u bench.py --preset cfg5 --steps 5 --warmup 2 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err
      echo presets ok ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o full \
        -- python3 bench.py --sequential-towers --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_full.log 2>&1
      f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); python tools/prof_csv_summary.py "$f" > $OUT/prof_summary.txt 2>&1 || cp "$f" $OUT/prof_summary.txt
      head -45 $OUT/prof_summary.txt ;;
    abr02)  # same-box A/B of the cfg2 step: this tree's libmmr vs tools/ab/${ABLIB:-libmmr_r02.so} (round 2's)
      for i in 1 2; do
        for lib in new old; do
          if [ $lib = old ]; then export MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/${ABLIB:-libmmr_r02.so}; else unset MMR_LIBMMR; fi
          timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > $OUT/ab_${lib}_$i.json 2> $OUT/ab_${lib}_$i.err
          python -c "import json;d=json.load(open('$OUT/ab_${lib}_$i.json'));print('$lib',round(d['ms_per_step'],3),{k:round(v['ms_per_launch']*1e3,1) for k,v in d['roofline']['bert_gemms'].items()})"
        done
      done
      unset MMR_LIBMMR ;;
    prof5)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o cfg5 \
        -- python3 bench.py --sequential-towers --preset cfg5 --steps 4 --warmup 2 --no-cpu-baseline > $OUT/prof5.log 2>&1
      f=$(find $OUT/prof5 -name "*kernel_stats.csv" | head -1); python tools/prof_csv_summary.py "$f" > $OUT/prof5_summary.txt 2>&1 || cp "$f" $OUT/prof5_summary.txt
      head -45 $OUT/prof5_summary.txt ;;
    mxab)  # same-box A/B of the MX-fp8 / bf16 GEMMs: this tree's libmmr vs tools/ab/${ABLIB:-libmmr_head.so}
      for i in 1 2; do
        for lib in new old; do
          if [ $lib = old ]; then export MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/${ABLIB:-libmmr_head.so}; else unset MMR_LIBMMR; fi
          echo "== $lib $i" >> $OUT/mxab.txt
          timeout -k 10 300 python -u tools/gemm_mx.py >> $OUT/mxab.txt 2>&1
        done
      done
      unset MMR_LIBMMR; cat $OUT/mxab.txt ;;
    clk)  # effective clock per GEMM kernel (GRBM_GUI_ACTIVE / 8 / duration), bf16 vs MX-fp8
      timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/clk -o clk -- python3 tools/clock_probe.py > $OUT/clk.log 2>&1
      f=$(find $OUT/clk -name "*counter_collection.csv" | head -1); python tools/clock_summary.py "$f" > $OUT/clk.txt 2>&1; cat $OUT/clk.txt ;;
    ksweep)
      timeout -k 10 300 python -u tools/gemm_ksweep.py > $OUT/ksweep.txt 2>&1; cat $OUT/ksweep.txt ;;
    stamps)  # per-tile breakdown of the 8-phase GEMM (diagnostic stamp build)
      MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/libmmr_stamps.so timeout -k 10 300 python -u tools/p8_stamps.py > $OUT/stamps.txt 2>&1; cat $OUT/stamps.txt
      if [ -f tools/ab/libmmr_nostore.so ]; then echo "== no stores" >> $OUT/stamps.txt
        MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/libmmr_nostore.so timeout -k 10 300 python -u tools/p8_stamps.py >> $OUT/stamps.txt 2>&1; cat $OUT/stamps.txt; fi ;;
    attnab)  # fused Swin attention block: this tree vs tools/ab/${ABLIB:-libmmr_head.so}
      for i in 1 2; do
        timeout -k 10 120 python -u tools/attn_ab.py >> $OUT/attn_ab.txt 2>&1
        MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/${ABLIB:-libmmr_head.so} timeout -k 10 120 python -u tools/attn_ab.py >> $OUT/attn_ab.txt 2>&1
      done; grep -v amdgpu.ids $OUT/attn_ab.txt ;;
    knnprof)  # kNN search (bench --mode knn) kernel stats: this tree vs tools/ab/${ABLIB:-libmmr_nostore.so}
      for lib in new old; do
        if [ $lib = old ]; then export MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/${ABLIB:-libmmr_nostore.so}; else unset MMR_LIBMMR; fi
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/knn_$lib -o k -- python3 bench.py --sequential-towers --mode knn --no-cpu-baseline > $OUT/knn_$lib.log 2>&1 || true
        f=$(find $OUT/knn_$lib -name "*kernel_stats.csv" | head -1); echo "== $lib"; python tools/prof_csv_summary.py "$f" | head -8
      done; unset MMR_LIBMMR ;;
    libab)  # same-box A/B of the tuned bf16 GEMM on the cfg2 shapes: this tree vs tools/ab/${ABLIB:-libmmr_nostore.so}
      for i in 1 2; do
        timeout -k 10 200 python -u tools/lib_ab.py new >> $OUT/libab.txt 2>&1
        MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/${ABLIB:-libmmr_nostore.so} timeout -k 10 200 python -u tools/lib_ab.py ${ABLIB:-nostore} >> $OUT/libab.txt 2>&1
      done; grep -v amdgpu.ids $OUT/libab.txt | tr '|' '\n' ;;
    swa)  # Swin window attention: this tree vs tools/ab/${ABLIB:-libmmr_head.so}
      for i in 1 2; do
        timeout -k 10 120 python -u tools/swa_bench.py new >> $OUT/swa.txt 2>&1
        MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/${ABLIB:-libmmr_head.so} timeout -k 10 120 python -u tools/swa_bench.py old >> $OUT/swa.txt 2>&1
      done; grep -v amdgpu.ids $OUT/swa.txt ;;
    mlpab)  # fused Swin MLP: this tree vs tools/ab/${ABLIB}
      for i in 1 2; do
        timeout -k 10 120 python -u tools/mlp_bench.py >> $OUT/mlpab_new.txt 2>&1
        MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/${ABLIB} timeout -k 10 120 python -u tools/mlp_bench.py >> $OUT/mlpab_old.txt 2>&1
      done; echo new; grep -v amdgpu.ids $OUT/mlpab_new.txt; echo $ABLIB; grep -v amdgpu.ids $OUT/mlpab_old.txt ;;
    trace)  # kernel trace of sequential cfg2 steps; launch list of step 4 (TRACEFLT filters names)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o tr \
        -- python3 bench.py --sequential-towers --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace.log 2>&1
      f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1); python tools/step_list.py "$f" 4 "${TRACEFLT:-}" > $OUT/step_list.txt; cat $OUT/step_list.txt | tail -${TRACEN:-60} ;;
    attab)  # attention cores (tools/mha_bench.py + tools/attn_ab.py): this tree vs tools/ab/${ABLIB:-libmmr_prev.so}
      for i in 1 2; do
        echo "== new $i" >> $OUT/attab.txt; timeout -k 10 120 python -u tools/mha_bench.py >> $OUT/attab.txt 2>&1
        timeout -k 10 120 python -u tools/attn_ab.py >> $OUT/attab.txt 2>&1
        echo "== old $i" >> $OUT/attab.txt
        MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/${ABLIB:-libmmr_prev.so} timeout -k 10 120 python -u tools/mha_bench.py >> $OUT/attab.txt 2>&1
        MMR_LIBMMR=$GRAFT_REPO_ROOT/tools/ab/${ABLIB:-libmmr_prev.so} timeout -k 10 120 python -u tools/attn_ab.py >> $OUT/attab.txt 2>&1
      done; grep -v amdgpu.ids $OUT/attab.txt ;;
    cfg5ab)  # cfg5 step: this tree vs tools/ab/${ABLIB:-libmmr_prev.so}, same box
      for i in 1 2; do for L in new old; do
        if [ $L = new ]; then E=X=0; else E=MMR_LIBMMR=tools/ab/${ABLIB:-libmmr_prev.so}; fi
        env $E timeout -k 10 500 python -u bench.py --preset cfg5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/cfg5ab.json 2> $OUT/cfg5ab.err
        python -c "import json;d=json.load(open('$OUT/cfg5ab.json'));print('$L', round(d['ms_per_step'],3), round(d['value']))"
      done; done ;;
    cfg5env)  # cfg5 step, env A / B (ENVA / ENVB), same box
      for i in 1 2; do for e in "${ENVA:-X=0}" "${ENVB:-X=1}"; do
        env $e timeout -k 10 500 python -u bench.py --preset cfg5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/cfg5env.json 2> $OUT/cfg5env.err
        python -c "import json;d=json.load(open('$OUT/cfg5env.json'));print('$e', round(d['ms_per_step'],3), round(d['value']))"
      done; done ;;
    pyt)  # a subset of the GPU tests (PYT = pytest selection)
      timeout -k 10 400 python -u -m pytest ${PYT} -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pyt.log 2>&1 || { tail -30 $OUT/pyt.log; exit 1; }
      tail -2 $OUT/pyt.log ;;
    knnab)  # kNN leg alone at KNNARGS (default cfg5: Q 2048 over 1M x 1024), env A / B (ENVA / ENVB)
      for i in 1 2; do for e in "${ENVA:-X=0}" "${ENVB:-X=1}"; do
        env $e timeout -k 10 300 python -u bench.py --mode knn ${KNNARGS:---preset cfg5 --batch 2048} --steps 10 --warmup 2 --no-cpu-baseline > $OUT/knnab.json 2> $OUT/knnab.err
        python -c "import json;d=json.load(open('$OUT/knnab.json'));print('$e', round(d['ms_per_step'],3), d['value'])"
      done; done ;;
    rw)
      timeout -k 10 200 python -u tools/rw_bench.py > $OUT/rw.txt 2>&1; grep -v amdgpu.ids $OUT/rw.txt ;;
    breakdown)  # per-(op, shape) times of one sequential cfg2 step
      timeout -k 10 300 python -u tools/step_breakdown.py ${BDARGS:-} > $OUT/breakdown.txt 2>&1; grep -v amdgpu.ids $OUT/breakdown.txt | head -70 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
