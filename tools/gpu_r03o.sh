#!/bin/bash
# r03o: split round head (first output's gains alone, its whitening + chain on the whole chip, the
# other outputs' gains on the Gram CUs) + the early dense prefix: parity subset, north A/B with
# GPAR_SPLIT_HEAD=1 / 0 on the same box, a kernel trace of one north step (round gaps).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_split.py tests/test_gpu_headline.py tests/test_gpu_driver.py tests/test_gpu_dist_cache.py tests/test_gpu_dtc.py tests/test_gpu_predict.py \
  > gpurun_out/r03o_tests.log 2>&1 || { tail -60 gpurun_out/r03o_tests.log; exit 1; }
tail -1 gpurun_out/r03o_tests.log
for v in 1 0 1 0; do
  GPAR_SPLIT_HEAD=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03o_north_h$v.json 2> gpurun_out/r03o_north_h$v.err || { echo BENCH FAILED; tail -20 gpurun_out/r03o_north_h$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03o_north_h$v.json')); print('split_head $v', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), 'pred', d['roofline_predict'].get('wall_ms_per_step'), d['self_check']['max_rel'], d['roofline_predict'].get('one_lane_probe'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03o_trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03o_trace.json 2> gpurun_out/r03o_trace.err || { echo TRACE FAILED; tail -20 gpurun_out/r03o_trace.err; exit 1; }
python3 tools/trace_rounds.py gpurun_out/r03o_trace/run_kernel_trace.csv > gpurun_out/r03o_rounds.txt 2>&1 || { tail gpurun_out/r03o_rounds.txt; exit 1; }
head -40 gpurun_out/r03o_rounds.txt
gzip gpurun_out/r03o_trace/run_kernel_trace.csv
