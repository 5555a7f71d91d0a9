# whitening iteration: parity tests of the DTC path, then per-D timing probes (N=1e6, M=512)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dtc.py tests/test_gpu_edges.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_whiten.txt 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/pytest_whiten.txt; exit 1; }
tail -2 gpurun_out/pytest_whiten.txt
rm -f gpurun_out/probe.txt
for d in 16 32 48 63; do
  timeout -k 10 200 python tools/gram_probe.py --evals 10 --d $d >> gpurun_out/probe.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/probe.txt
