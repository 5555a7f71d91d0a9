#!/bin/bash
# r03b: round-overlapping fit -- parity (split tests incl. overlap on/off bit-identity, headline
# schedule), then the north job overlap on vs off (same box).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_split.py tests/test_gpu_headline.py tests/test_gpu_driver.py tests/test_gpu_predict.py \
  > gpurun_out/r03b_tests.log 2>&1 || { tail -60 gpurun_out/r03b_tests.log; exit 1; }
tail -3 gpurun_out/r03b_tests.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r03b_bench_overlap.json 2> gpurun_out/r03b_bench_overlap.err || exit 1
GPAR_OVERLAP=0 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r03b_bench_nooverlap.json 2> gpurun_out/r03b_bench_nooverlap.err || exit 1
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --shard 1/8 \
  > gpurun_out/r03b_bench_shard1of8.json 2> gpurun_out/r03b_bench_shard1of8.err || exit 1
GPAR_OVERLAP=0 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --shard 1/8 \
  > gpurun_out/r03b_bench_shard1of8_nooverlap.json 2> gpurun_out/r03b_bench_shard1of8_nooverlap.err || exit 1
python - <<'PY'
import json
for f in ("overlap", "nooverlap", "shard1of8", "shard1of8_nooverlap"):
    d = json.load(open(f"gpurun_out/r03b_bench_{f}.json"))
    print(f, round(d["ms_per_step"], 1), d["value"], d.get("self_check", {}).get("max_rel"),
          d["roofline"]["avg_ms"], d.get("roofline_whiten", {}).get("avg_ms"))
PY
