# All GPU tests on the tree library, then kernel-level and bench A/B against abl/libgparhip_prev.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
VAR=prev N=${N:-1000000} D=32 bash tools/gpu_ab_kernels.sh > gpurun_out/ab.txt || exit 1
grep -E "${KPAT:-whiten|gram|TOTAL}" gpurun_out/ab.txt
VAR=prev CFG=${CFG:-north} bash tools/gpu_bench_ab.sh || exit 1
