set -o pipefail
cd $GRAFT_REPO_ROOT
export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_gdiag.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_dtc.py tests/test_gpu_edges.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gdiag.txt 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/pytest_gdiag.txt; exit 1; }
tail -2 gpurun_out/pytest_gdiag.txt
unset GPAR_LIB_PATH
VAR=gdiag N=1000000 D=32 bash tools/gpu_ab_kernels.sh > gpurun_out/ab.txt || exit 1
grep -E "gram|TOTAL" gpurun_out/ab.txt
