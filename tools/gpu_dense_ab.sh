# The dense tail's kernel durations (tools/dense_probe.py under rocprofv3 --stats) for the in-tree
# library and gpar-at-scale_amd/ab_prev/.   bash tools/gpu_dense_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
for v in cur prev; do
  if [ $v = prev ]; then export GPAR_HIP_LIB=$PWD/gpar-at-scale_amd/ab_prev/libgparhip.so; else unset GPAR_HIP_LIB; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/d_$v -o run --output-format csv -- python3 tools/dense_probe.py --m 512 --batch 8 > $O/dense_$v.txt 2>&1 || exit 1
  find $O/d_$v -name '*kernel_stats.csv' -exec cp {} $O/dense_${v}_stats.csv \;
  rm -rf $O/d_$v
done
unset GPAR_HIP_LIB
