# A subset of the GPU suite (test files as arguments), then smoke and the default bench line.
# Usage: bash tools/gpu_tests.sh tag [tests/test_x.py ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-sub}
shift
timeout -k 10 1000 python -u -m pytest "$@" -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu_$tag.txt 2>&1 || { echo PYTEST FAILED; tail -40 gpurun_out/pytest_gpu_$tag.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu_$tag.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.txt 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke_$tag.txt; exit 1; }
tail -1 gpurun_out/smoke_$tag.txt
timeout -k 10 700 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
