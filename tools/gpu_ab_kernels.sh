# Kernel-level A/B (rocprofv3 --kernel-trace --stats) of the tree library vs
# gpar-at-scale_amd/abl/libgparhip_$VAR.so on tools/gram_probe.py:
#   VAR=x N=100000 D=32 bash tools/gpu_ab_kernels.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in base $VAR; do
  if [ $lib = base ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$lib.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$lib -o run --output-format csv -- python3 tools/gram_probe.py --evals 10 --n ${N:-1000000} --d ${D:-32} > gpurun_out/ab_$lib.txt 2>&1 || { tail gpurun_out/ab_$lib.txt; exit 1; }
done
python3 tools/ab_compare.py gpurun_out/ab_base gpurun_out/ab_$VAR
