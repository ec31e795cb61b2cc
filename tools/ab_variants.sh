# A/B several builds of libmmr.so on one box: multi-modal-retrieval-predict-project_amd/libmmr_<v>.so for each
# variant v given, alternated over two rounds around one diagnostic tool; the tree's libmmr.so restored after.
# usage (via gpurun): bash tools/ab_variants.sh "v0 v1 ..." <tool.py> [tool args...]
set -o pipefail
P=multi-modal-retrieval-predict-project_amd
VS=$1; shift
mkdir -p gpurun_out
cp $P/libmmr.so $P/libmmr_tree.so
for rnd in 1 2; do
  for v in $VS; do
    [ -f $P/libmmr_$v.so ] || { echo "no $P/libmmr_$v.so"; cp $P/libmmr_tree.so $P/libmmr.so; exit 1; }
    cp $P/libmmr_$v.so $P/libmmr.so
    echo "== $v (round $rnd)"
    timeout -k 10 300 python -u "$@" > gpurun_out/abv_$v.txt 2>&1 || { cat gpurun_out/abv_$v.txt; cp $P/libmmr_tree.so $P/libmmr.so; exit 1; }
    grep -v amdgpu.ids gpurun_out/abv_$v.txt
  done
done
cp $P/libmmr_tree.so $P/libmmr.so
