set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/mfma_valu_overlap > gpurun_out/ubench_overlap.txt 2>&1 || exit 1
cat gpurun_out/ubench_overlap.txt
rm -f gpurun_out/probe.txt
for d in 16 32 48 63; do
  timeout -k 10 200 python tools/gram_probe.py --evals 10 --d $d >> gpurun_out/probe.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/probe.txt
