#!/bin/bash
# r03a: new parity tests (headline schedule, all-D cache, distances, memory pressure), then the
# north job with the cache released per fit call (new default) vs kept.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_dist_cache.py tests/test_gpu_split.py \
  > gpurun_out/r03a_tests.log 2>&1 || { tail -40 gpurun_out/r03a_tests.log; exit 1; }
tail -5 gpurun_out/r03a_tests.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r03a_bench_release.json 2> gpurun_out/r03a_bench_release.err || exit 1
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --dist-cache-keep \
  > gpurun_out/r03a_bench_keep.json 2> gpurun_out/r03a_bench_keep.err || exit 1
python - <<'PY'
import json
for f in ("release", "keep"):
    d = json.load(open(f"gpurun_out/r03a_bench_{f}.json"))
    print(f, d["ms_per_step"], d["value"], d.get("self_check"), d["memory"].get("dist_cache"))
PY
