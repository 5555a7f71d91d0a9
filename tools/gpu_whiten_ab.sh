# GPU tests, then whitening A/B per D bucket (rocprof kernel stats) and a north bench A/B of the
# tree library vs gpar-at-scale_amd/abl/libgparhip_prev.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
for d in ${DS:-16 32 48 63}; do
  VAR=prev N=1000000 D=$d bash tools/gpu_ab_kernels.sh > gpurun_out/ab_d$d.txt || exit 1
  echo "D=$d"; grep -E "whiten_kfu|TOTAL" gpurun_out/ab_d$d.txt
done
[ -n "$NOBENCH" ] || VAR=prev CFG=${CFG:-north} bash tools/gpu_bench_ab.sh
