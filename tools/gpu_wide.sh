# config 5 at full width: tests + per-evaluation timing at D = 255 (N = 1e7, M = 1024)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_wide.txt 2>&1 || { echo PYTEST FAILED; tail -40 gpurun_out/pytest_wide.txt; exit 1; }
tail -15 gpurun_out/pytest_wide.txt
for d in 32 255; do
  timeout -k 10 300 python tools/gram_probe.py --n 10000000 --m 1024 --d $d --evals 3 >> gpurun_out/config5_probe.txt 2>&1 || { echo PROBE FAILED; tail -20 gpurun_out/config5_probe.txt; exit 1; }
done
cat gpurun_out/config5_probe.txt
