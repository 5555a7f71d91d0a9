# Round profile: PMC passes (Gram + whitening traffic, SQ counters), then rocprofv3 kernel stats of
# the default north bench (1 warm-up + 1 timed step), then the plain bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_passes.sh > gpurun_out/pmc_summary.txt 2>&1 || { echo PMC FAILED; tail -20 gpurun_out/pmc_summary.txt; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_rocprof.json 2> gpurun_out/bench_rocprof.err || { echo ROCPROF BENCH FAILED; tail -20 gpurun_out/bench_rocprof.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
