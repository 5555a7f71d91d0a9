#!/bin/bash
# r03x: the prediction workspace estimate without Q rows on the fused path (so the distance cache
# budget holds every north output): cache / headline / driver tests, north job twice.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dist_cache.py tests/test_gpu_headline.py tests/test_gpu_driver.py > gpurun_out/r03x_tests.log 2>&1 || { tail -40 gpurun_out/r03x_tests.log; exit 1; }
tail -1 gpurun_out/r03x_tests.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03x_north$r.json 2> gpurun_out/r03x_north$r.err || { echo BENCH FAILED; tail -20 gpurun_out/r03x_north$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03x_north$r.json')); print('north', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), 'pred', d['roofline_predict'].get('wall_ms_per_step'), d['memory']['dist_cache'], round(d['memory']['device_free_gb'],1))"
done
