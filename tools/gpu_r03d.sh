#!/bin/bash
# r03d: overlapped fit with its gains + dense tails beside the whitening (s_d); path sampling
# (posterior_rand, PATH mode) parity; north / shard overlap A/B; north PATH-mode cost.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_path.py tests/test_gpu_split.py tests/test_gpu_predict.py tests/test_gpu_driver.py \
  > gpurun_out/r03d_tests.log 2>&1 || { tail -60 gpurun_out/r03d_tests.log; exit 1; }
tail -2 gpurun_out/r03d_tests.log
for v in 1 0; do
  GPAR_OVERLAP=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r03d_north_ov$v.json 2> gpurun_out/r03d_north_ov$v.err || exit 1
  GPAR_OVERLAP=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --shard 1/8 \
    > gpurun_out/r03d_shard_ov$v.json 2> gpurun_out/r03d_shard_ov$v.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --predict path \
  > gpurun_out/r03d_north_path.json 2> gpurun_out/r03d_north_path.err || exit 1
python - <<'PY'
import json
for f in ("north_ov1", "north_ov0", "shard_ov1", "shard_ov0", "north_path"):
    d = json.load(open(f"gpurun_out/r03d_{f}.json"))
    print(f, round(d["ms_per_step"], 1), d["value"], d["roofline"]["avg_ms"], d.get("roofline_whiten", {}).get("avg_ms"),
          {k: round(v["ms_per_step"], 1) for k, v in d.get("roofline_predict", {}).items() if isinstance(v, dict)})
PY
