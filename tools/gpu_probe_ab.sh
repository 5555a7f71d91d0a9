# A/B of a library variant: tree library vs gpar-at-scale_amd/abl/libgparhip_$VAR.so, per D (N=1e6, M=512)
#   VAR=occ3 DS="24 32" bash tools/gpu_probe_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/probe_ab.txt
for d in ${DS:-16 32 48 63}; do
  for lib in base $VAR; do
    if [ $lib = base ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$lib.so; fi
    echo -n "$lib " >> gpurun_out/probe_ab.txt
    timeout -k 10 200 python tools/gram_probe.py --evals 10 --d $d 2>/dev/null >> gpurun_out/probe_ab.txt || exit 1
  done
done
sed 's/dtc=.*gram/gram/; s/gains:.*//' gpurun_out/probe_ab.txt
