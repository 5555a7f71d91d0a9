#!/bin/bash
# r03s (dense prefix queued after the round's gains launches): host side of a Nelder-Mead round boundary: kernel + HIP API trace of one north step,
# the HIP calls inside the median round gap (tools/trace_rounds.py --hip).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/r03s_trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03s_trace.json 2> gpurun_out/r03s_trace.err || { echo TRACE FAILED; tail -20 gpurun_out/r03s_trace.err; exit 1; }
ls -la gpurun_out/r03s_trace
python3 tools/trace_rounds.py gpurun_out/r03s_trace/run_kernel_trace.csv --hip gpurun_out/r03s_trace/run_hip_api_trace.csv > gpurun_out/r03s_rounds.txt 2>&1 || { tail gpurun_out/r03s_rounds.txt; exit 1; }
grep -A60 "HIP API calls" gpurun_out/r03s_rounds.txt | head -90
gzip gpurun_out/r03s_trace/*.csv
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03s_north.json 2> gpurun_out/r03s_north.err || { echo BENCH FAILED; tail -20 gpurun_out/r03s_north.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03s_north.json')); print('north', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), 'pred', d['roofline_predict'].get('wall_ms_per_step'), d['self_check']['max_rel'])"
