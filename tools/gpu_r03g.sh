#!/bin/bash
# r03g: predict_var v3 (row-split waves, LDS-DMA V slabs) + adjoint prefetch -- parity subset,
# probe A/B fused vs unfused under rocprofv3 --stats, north bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_predict.py tests/test_gpu_driver.py tests/test_gpu_headline.py tests/test_gpu_path.py \
  > gpurun_out/r03g_tests.log 2>&1 || { tail -60 gpurun_out/r03g_tests.log; exit 1; }
tail -2 gpurun_out/r03g_tests.log
for v in 1 0; do
  GPAR_PREDICT_FUSED=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03g_prof_f$v -o run --output-format csv -- \
    python3 tools/predict_probe.py --outputs 8 --dmin 30 --reps 3 > gpurun_out/r03g_prof_f$v.log 2>&1 || { tail -20 gpurun_out/r03g_prof_f$v.log; exit 1; }
  echo "fused $v"; grep rep gpurun_out/r03g_prof_f$v.log
done
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r03g_north.json 2> gpurun_out/r03g_north.err || exit 1
python - <<'PY'
import json, csv
for v in (1, 0):
    rows = list(csv.DictReader(open(f"gpurun_out/r03g_prof_f{v}/run_kernel_stats.csv")))
    print("fused", v, [(r["Name"][:28], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3)) for r in rows[:10]])
d = json.load(open("gpurun_out/r03g_north.json"))
rp = d.get("roofline_predict", {})
print("north", round(d["ms_per_step"], 1), d["value"], d["roofline"]["avg_ms"], rp.get("wall_ms_per_step"),
      {k: round(v["ms_per_step"], 1) for k, v in rp.items() if isinstance(v, dict)})
PY
