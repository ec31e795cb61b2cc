# knn_select_t phase clock (tools/select_trace.hip, MMR_SELECT_TRACE build) on the GPU box: built there, run at
# Q = 16 and 256 in f16 mode over 100k x 768.  usage (via gpurun): bash tools/gpu_select_trace.sh
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -I include tools/select_trace.hip \
  multi-modal-retrieval-predict-project_amd/csrc/capi.cpp multi-modal-retrieval-predict-project_amd/csrc/gemm.hip \
  -o /tmp/select_trace.bin > gpurun_out/seltrace_build.log 2>&1
for q in 16 256; do timeout -k 10 120 /tmp/select_trace.bin $q 2 >> gpurun_out/seltrace.txt 2>&1; done
cat gpurun_out/seltrace.txt
