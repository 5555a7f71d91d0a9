# Round evidence: full GPU suite, smoke, PMC passes, rocprof kernel stats of the north bench, and
# the default bench line (with cpu_baseline).  bash tools/gpu_final.sh <tag>, e.g. r04z: every
# summary lands under gpurun_out/final_<tag>/ named as profiles/ wants it.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
OUT=gpurun_out/final_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.txt 2>&1 || { echo PYTEST FAILED; tail -30 $OUT/pytest_gpu_$TAG.txt; exit 1; }
tail -1 $OUT/pytest_gpu_$TAG.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.txt 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke_$TAG.txt; exit 1; }
tail -1 $OUT/smoke_$TAG.txt
bash tools/pmc_passes.sh > $OUT/pmc_summary.txt 2>&1 || { echo PMC FAILED; tail -20 $OUT/pmc_summary.txt; exit 1; }
cp gpurun_out/pmc/summary.json $OUT/pmc_gram_whiten_$TAG.json
# the bench lines below read this round's traffic from profiles/ (bench.py PMC_FILE)
PMC=$(python3 -c "import re;print(re.search(r'PMC_FILE = \"(.*)\"', open('bench.py').read()).group(1))")
cp gpurun_out/pmc/summary.json profiles/$PMC
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/bench_${TAG}_north_rocprof_run.json 2> $OUT/bench_rocprof.err || { echo ROCPROF BENCH FAILED; tail -20 $OUT/bench_rocprof.err; exit 1; }
find gpurun_out/prof -name '*kernel_stats.csv' -exec cp {} $OUT/rocprof_bench_${TAG}_north_stats.csv \;
timeout -k 10 600 python bench.py > $OUT/bench_${TAG}_north.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench_${TAG}_north.json
