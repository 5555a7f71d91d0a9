# v3 Gram check: full GPU suite on the tree library, then probe + bench A/B against the v2 build
# (gpar-at-scale_amd/abl/libgparhip_GRAM_V30.so from tools/build_abl.sh GRAM_V3 0)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_v3.txt 2>&1 || { tail -30 gpurun_out/pytest_v3.txt; exit 1; }
tail -3 gpurun_out/pytest_v3.txt
VAR=GRAM_V30 DS="3 32" bash tools/gpu_probe_ab.sh || exit 1
VAR=GRAM_V30 bash tools/gpu_bench_ab.sh
