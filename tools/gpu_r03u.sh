#!/bin/bash
# r03u: the dense prefix queued after the round's gains launches (GPAR_DENSE_EARLY=1) vs before
# them (2, the r03n order), north, same box, no profiler (rocprof's per-dispatch bookkeeping made
# a launch behind running work cost ~90 us instead of ~2.5 us: tools/ubench/launch_cost).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_headline.py > gpurun_out/r03u_tests.log 2>&1 || { tail -40 gpurun_out/r03u_tests.log; exit 1; }
tail -1 gpurun_out/r03u_tests.log
for v in 1 2 1 2; do
  GPAR_DENSE_EARLY=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03u_north_d$v.json 2> gpurun_out/r03u_north_d$v.err || { echo BENCH FAILED; tail -20 gpurun_out/r03u_north_d$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03u_north_d$v.json')); print('dense_early $v', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), 'pred', d['roofline_predict'].get('wall_ms_per_step'), d['self_check']['max_rel'])"
done
# one rank's shard of the 8-GPU job (rank 1 of 8, the slowest in r03d/e) with the current code
for r in 1 0; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --shard $r/8 > gpurun_out/r03u_shard$r.json 2> gpurun_out/r03u_shard$r.err || { echo SHARD FAILED; tail -20 gpurun_out/r03u_shard$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03u_shard$r.json')); print('shard $r/8', d['config'].get('shard_outputs'), round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3))"
done
