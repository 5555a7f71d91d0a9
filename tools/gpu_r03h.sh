#!/bin/bash
# r03h: predict_var v4 (single stage, w in LDS, one DMA base) + the predictions-span check;
# isolated (one lane) A/B fused vs unfused under rocprofv3 --stats; parity subset.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_predict.py tests/test_gpu_driver.py tests/test_gpu_path.py \
  > gpurun_out/r03h_tests.log 2>&1 || { tail -60 gpurun_out/r03h_tests.log; exit 1; }
tail -2 gpurun_out/r03h_tests.log
timeout -k 10 200 python -u tools/pred_timer_check.py > gpurun_out/r03h_timer.log 2>&1 || { tail -20 gpurun_out/r03h_timer.log; exit 1; }
cat gpurun_out/r03h_timer.log | grep rep
for v in 1 0; do
  GPAR_PREDICT_LANES=1 GPAR_PREDICT_FUSED=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03h_prof_f$v -o run --output-format csv -- \
    python3 tools/predict_probe.py --outputs 8 --dmin 30 --reps 3 > gpurun_out/r03h_prof_f$v.log 2>&1 || { tail -20 gpurun_out/r03h_prof_f$v.log; exit 1; }
  echo "fused $v"; grep rep gpurun_out/r03h_prof_f$v.log
done
python - <<'PY'
import csv
for v in (1, 0):
    rows = list(csv.DictReader(open(f"gpurun_out/r03h_prof_f{v}/run_kernel_stats.csv")))
    print("fused", v, [(r["Name"][:28], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3)) for r in rows[:12]])
PY
