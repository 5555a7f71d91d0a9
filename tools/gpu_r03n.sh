#!/bin/bash
# r03n: the dense tail's G-independent half (Kuu, chol, inverse) issued ahead of the round's Grams
# on the Gram stream: parity subset of the split / headline / driver / cache tests, the north job
# (two steps) with GPAR_DENSE_EARLY=1 / 0 on the same box, and a kernel trace of one north step
# (round gaps: tools/trace_rounds.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_split.py tests/test_gpu_headline.py tests/test_gpu_driver.py tests/test_gpu_dist_cache.py tests/test_gpu_dtc.py \
  > gpurun_out/r03n_tests.log 2>&1 || { tail -60 gpurun_out/r03n_tests.log; exit 1; }
tail -1 gpurun_out/r03n_tests.log
for v in 1 0 1 0; do
  GPAR_DENSE_EARLY=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03n_north_d$v.json 2> gpurun_out/r03n_north_d$v.err || { echo BENCH FAILED; tail -20 gpurun_out/r03n_north_d$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03n_north_d$v.json')); print('dense_early $v', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), 'pred', d['roofline_predict'].get('wall_ms_per_step'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03n_trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03n_trace.json 2> gpurun_out/r03n_trace.err || { echo TRACE FAILED; tail -20 gpurun_out/r03n_trace.err; exit 1; }
python3 tools/trace_rounds.py gpurun_out/r03n_trace/run_kernel_trace.csv > gpurun_out/r03n_rounds.txt 2>&1 || { tail gpurun_out/r03n_rounds.txt; exit 1; }
cat gpurun_out/r03n_rounds.txt
rm -f gpurun_out/r03n_trace/run_kernel_trace.csv
