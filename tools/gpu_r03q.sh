#!/bin/bash
# r03q: parity subset (split / headline / driver / cache / dtc / predict / path) with the split
# round head, the early dense prefix and the y* column out of the wide adjoint; north A/B
# GPAR_SPLIT_HEAD=1 / 0; predict_var timing ablations (tools/gpu_r03p.sh); a kernel trace of one
# north step (tools/trace_rounds.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_split.py tests/test_gpu_headline.py tests/test_gpu_driver.py tests/test_gpu_dist_cache.py tests/test_gpu_dtc.py tests/test_gpu_predict.py tests/test_gpu_path.py \
  > gpurun_out/r03q_tests.log 2>&1 || { tail -60 gpurun_out/r03q_tests.log; exit 1; }
tail -1 gpurun_out/r03q_tests.log
for v in 1 0 1 0; do
  GPAR_SPLIT_HEAD=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03q_north_h$v.json 2> gpurun_out/r03q_north_h$v.err || { echo BENCH FAILED; tail -20 gpurun_out/r03q_north_h$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03q_north_h$v.json')); print('split_head $v', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), 'pred', d['roofline_predict'].get('wall_ms_per_step'), d['self_check']['max_rel'], d['roofline_predict'].get('one_lane_probe'))"
done
bash tools/gpu_r03p.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r03q_trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03q_trace.json 2> gpurun_out/r03q_trace.err || { echo TRACE FAILED; tail -20 gpurun_out/r03q_trace.err; exit 1; }
python3 tools/trace_rounds.py gpurun_out/r03q_trace/run_kernel_trace.csv > gpurun_out/r03q_rounds.txt 2>&1 || { tail gpurun_out/r03q_rounds.txt; exit 1; }
head -30 gpurun_out/r03q_rounds.txt
gzip gpurun_out/r03q_trace/run_kernel_trace.csv
