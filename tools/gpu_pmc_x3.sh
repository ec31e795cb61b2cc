# PMC evidence for the parity-grade (x3) kernels at cfg2 shapes (tools/pmc_x3.py): a kernel-trace pass, then
# one --pmc pass per counter group (SQ buckets + MFMA busy; GRBM clock; FETCH_SIZE; WRITE_SIZE), summarised by
# tools/pmc_x3_summary.py.  usage (via gpurun): bash tools/gpu_pmc_x3.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-x3}
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o k -- python3 tools/pmc_x3.py > $OUT/kt.log 2>&1 || { echo "FAIL kt"; tail -5 $OUT/kt.log; exit 1; }
KT=$(find $OUT/kt -name "*kernel_trace.csv" | head -1)
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"
P2="GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
CS=""
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o p -- python3 tools/pmc_x3.py > $OUT/p$i.log 2>&1 || { echo "FAIL pass $i"; tail -5 $OUT/p$i.log; exit 1; }
  CS="$CS $(find $OUT/p$i -name "*counter_collection.csv" | head -1)"
done
python3 tools/pmc_x3_summary.py $OUT/pmc_x3.json "$TAG" $KT $CS
