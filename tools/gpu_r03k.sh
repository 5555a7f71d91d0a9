#!/bin/bash
# r03k: q(u) batched over a gpar_fit_predict call's outputs (run_q_u_batch) -- parity subset, then
# the north job with GPAR_QU_BATCH=1 / 0 (same box, predictions' wall span).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_predict.py tests/test_gpu_driver.py tests/test_gpu_path.py tests/test_gpu_split.py \
  tests/test_gpu_headline.py tests/test_gpu_dist_cache.py \
  > gpurun_out/r03k_tests.log 2>&1 || { tail -60 gpurun_out/r03k_tests.log; exit 1; }
tail -2 gpurun_out/r03k_tests.log
for v in 1 0; do
  GPAR_QU_BATCH=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r03k_north_qb$v.json 2> gpurun_out/r03k_north_qb$v.err || exit 1
done
python3 - <<'PY'
import json
for v in (1, 0):
    d = json.load(open(f"gpurun_out/r03k_north_qb{v}.json"))
    rp = d.get("roofline_predict", {})
    print("qu_batch", v, round(d["ms_per_step"], 1), d["value"], "pred wall", rp.get("wall_ms_per_step"),
          {k: round(x["ms_per_step"], 1) for k, x in rp.items() if isinstance(x, dict)})
PY
