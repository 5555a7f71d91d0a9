# A/B of the whitening: tree library vs gpar-at-scale_amd/abl/libgparhip_orig.so, per D (N=1e6, M=512)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/probe_ab.txt
for d in 16 24 32 40 48 56 63; do
  for lib in orig new; do
    if [ $lib = orig ]; then export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_orig.so; else unset GPAR_LIB_PATH; fi
    echo -n "$lib " >> gpurun_out/probe_ab.txt
    timeout -k 10 200 python tools/gram_probe.py --evals 10 --d $d 2>/dev/null >> gpurun_out/probe_ab.txt || exit 1
  done
done
cat gpurun_out/probe_ab.txt
