#!/bin/bash
# Round-3 evidence (second session): full GPU suite, smoke, PMC passes over the Gram / whitening of a batched fit
# (-> profiles/pmc_gram_whiten_r03.json, which the bench line's `traffic` reads), rocprof kernel
# stats of the north bench, and the default bench line (with cpu_baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
bash tools/pmc_passes.sh > gpurun_out/pmc_summary.txt 2>&1 || { echo PMC FAILED; tail -20 gpurun_out/pmc_summary.txt; exit 1; }
cp gpurun_out/pmc/summary.json profiles/pmc_gram_whiten_r03.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_rocprof.json 2> gpurun_out/bench_rocprof.err || { echo ROCPROF BENCH FAILED; tail -20 gpurun_out/bench_rocprof.err; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
