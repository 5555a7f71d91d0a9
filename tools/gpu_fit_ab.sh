# Fit-path A/B (whitening from the distance cache): tree library vs the variants in $VARS
# (gpar-at-scale_amd/abl/libgparhip_<var>.so), gram_probe --fit at N=1e6, M=512, D=$D (default 32)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/fit_ab.txt
for rep in 1 2; do
for lib in base $VARS; do
  if [ $lib = base ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$lib.so; fi
  echo -n "$lib " >> gpurun_out/fit_ab.txt
  timeout -k 10 200 python tools/gram_probe.py --fit --evals ${EVALS:-20} --d ${D:-32} 2>/dev/null >> gpurun_out/fit_ab.txt || exit 1
done
done
sed 's/dtc=.*gram/gram/; s/gains:.*//' gpurun_out/fit_ab.txt
