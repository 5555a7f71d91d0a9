#!/bin/bash
# r03c: overlapped fit with the dense tails on the whitening CUs: overlap bit-identity, then the
# north job and the 1/8 shard, overlap on vs off (same box).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_split.py > gpurun_out/r03c_tests.log 2>&1 || { tail -60 gpurun_out/r03c_tests.log; exit 1; }
tail -2 gpurun_out/r03c_tests.log
for v in 1 0; do
  GPAR_OVERLAP=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r03c_north_ov$v.json 2> gpurun_out/r03c_north_ov$v.err || exit 1
  GPAR_OVERLAP=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --shard 1/8 \
    > gpurun_out/r03c_shard_ov$v.json 2> gpurun_out/r03c_shard_ov$v.err || exit 1
done
python - <<'PY'
import json
for f in ("north_ov1", "north_ov0", "shard_ov1", "shard_ov0"):
    d = json.load(open(f"gpurun_out/r03c_{f}.json"))
    print(f, round(d["ms_per_step"], 1), d["value"], d["roofline"]["avg_ms"], d.get("roofline_whiten", {}).get("avg_ms"))
PY
