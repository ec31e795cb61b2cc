# A/B two builds of libmmr.so on one box: the tree's libmmr.so ("new") against a saved earlier build
# multi-modal-retrieval-predict-project_amd/libmmr_base.so ("base", copied there before the change), alternated
# new / base / new / base around one diagnostic tool, then the new build restored.  Delete libmmr_base.so after.
# usage (via gpurun): bash tools/ab_lib_swap.sh <tool.py> [tool args...]
set -o pipefail
P=multi-modal-retrieval-predict-project_amd
mkdir -p gpurun_out
[ -f $P/libmmr_base.so ] || { echo "no $P/libmmr_base.so"; exit 1; }
cp $P/libmmr.so $P/libmmr_new.so
for v in new base new base; do
  cp $P/libmmr_$v.so $P/libmmr.so
  echo "== $v"; timeout -k 10 300 python -u "$@" > gpurun_out/ab_$v.txt 2>&1 || { cp $P/libmmr_new.so $P/libmmr.so; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab_$v.txt
done
cp $P/libmmr_new.so $P/libmmr.so
