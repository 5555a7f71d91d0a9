#!/bin/bash
# r03j: adjoint_local_wide through a buffer descriptor (8 rows in flight, dropped stores at train
# rows) -- parity subset, one-lane probe under rocprofv3 --stats; then the r03i bench modes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_predict.py tests/test_gpu_driver.py tests/test_gpu_path.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py \
  > gpurun_out/r03j_tests.log 2>&1 || { tail -60 gpurun_out/r03j_tests.log; exit 1; }
tail -2 gpurun_out/r03j_tests.log
GPAR_PREDICT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03j_prof -o run --output-format csv -- \
  python3 tools/predict_probe.py --outputs 8 --dmin 30 --reps 3 > gpurun_out/r03j_prof.log 2>&1 || { tail -20 gpurun_out/r03j_prof.log; exit 1; }
grep rep gpurun_out/r03j_prof.log
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r03j_prof/run_kernel_stats.csv")))
print([(r["Name"][:28], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3)) for r in rows[:10]])
PY
bash tools/gpu_r03i.sh
