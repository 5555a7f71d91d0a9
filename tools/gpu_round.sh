# Round evidence: full pytest -m gpu suite, __graft_entry__.smoke(), the default bench line.
# Usage: bash tools/gpu_round.sh [tag]   (outputs gpurun_out/pytest_gpu_<tag>.txt, bench_<tag>.json)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-round}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/pytest_gpu_$tag.txt 2>&1 || { echo PYTEST FAILED; tail -40 gpurun_out/pytest_gpu_$tag.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu_$tag.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.txt 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke_$tag.txt; exit 1; }
tail -1 gpurun_out/smoke_$tag.txt
timeout -k 10 600 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
