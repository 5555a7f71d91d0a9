#!/bin/bash
# r03r: a batched round's uploads / results through a pinned arena (eval_dtc): parity subset, north
# A/B GPAR_ROUND_STAGING=1 / 0 on the same box, trace of one north step (round gaps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_split.py tests/test_gpu_headline.py tests/test_gpu_driver.py tests/test_gpu_dist_cache.py tests/test_gpu_dtc.py tests/test_gpu_multirank.py \
  > gpurun_out/r03r_tests.log 2>&1 || { tail -60 gpurun_out/r03r_tests.log; exit 1; }
tail -1 gpurun_out/r03r_tests.log
for v in 1 0 1 0; do
  GPAR_ROUND_STAGING=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03r_north_s$v.json 2> gpurun_out/r03r_north_s$v.err || { echo BENCH FAILED; tail -20 gpurun_out/r03r_north_s$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03r_north_s$v.json')); print('round_staging $v', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), 'pred', d['roofline_predict'].get('wall_ms_per_step'), d['self_check']['max_rel'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03r_trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03r_trace.json 2> gpurun_out/r03r_trace.err || { echo TRACE FAILED; tail -20 gpurun_out/r03r_trace.err; exit 1; }
python3 tools/trace_rounds.py gpurun_out/r03r_trace/run_kernel_trace.csv > gpurun_out/r03r_rounds.txt 2>&1 || { tail gpurun_out/r03r_rounds.txt; exit 1; }
sed -n 1,4p gpurun_out/r03r_rounds.txt
gzip gpurun_out/r03r_trace/run_kernel_trace.csv
