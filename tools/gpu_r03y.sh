#!/bin/bash
# r03y: the committed tree at the end of round 3: full GPU suite, smoke, default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('north', round(d['ms_per_step'],1), d['value'], 'gram frac', round(d['roofline']['frac'],3), 'pred', d['roofline_predict'].get('wall_ms_per_step'), d['memory']['dist_cache'], d['cpu_baseline']['value'])"
