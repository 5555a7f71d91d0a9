# bench modes beyond the default line: chained inference inputs and the MC estimator
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config small --inference chained --no-cpu-baseline > gpurun_out/bench_small_chained.json 2> gpurun_out/bench_small_chained.err || { echo SMALL CHAINED FAILED; tail -20 gpurun_out/bench_small_chained.err; exit 1; }
cat gpurun_out/bench_small_chained.json
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --predict mc --no-cpu-baseline > gpurun_out/bench_north_mc.json 2> gpurun_out/bench_north_mc.err || { echo MC FAILED; tail -20 gpurun_out/bench_north_mc.err; exit 1; }
cat gpurun_out/bench_north_mc.json
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --inference chained --no-cpu-baseline > gpurun_out/bench_north_chained.json 2> gpurun_out/bench_north_chained.err || { echo CHAINED FAILED; tail -20 gpurun_out/bench_north_chained.err; exit 1; }
cat gpurun_out/bench_north_chained.json
