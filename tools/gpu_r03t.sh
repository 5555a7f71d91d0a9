#!/bin/bash
# r03t: host cost of a kernel launch on this pool (tools/ubench/launch_cost), plain and under
# rocprofv3 --kernel-trace (whose per-dispatch bookkeeping may inflate it); adjoint pass A/B with
# 576-column vs 256-column workgroups on the one-lane predict probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
env | grep -E "^(HIP|AMD|GPU|HSA|ROC)" | sort > gpurun_out/r03t_env.txt
timeout -k 10 120 ./tools/ubench/launch_cost > gpurun_out/r03t_launch.txt 2>&1 || { cat gpurun_out/r03t_launch.txt; exit 1; }
cat gpurun_out/r03t_launch.txt
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/r03t_prof -o run --output-format csv -- ./tools/ubench/launch_cost > gpurun_out/r03t_launch_prof.txt 2>&1 || { tail gpurun_out/r03t_launch_prof.txt; exit 1; }
grep "per launch" gpurun_out/r03t_launch_prof.txt
rm -rf gpurun_out/r03t_prof
for cw in 576 256; do
  GPAR_ADJ_CW=$cw GPAR_PREDICT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03t_adj$cw -o run --output-format csv -- \
    python3 tools/predict_probe.py --outputs 8 --dmin 30 --reps 2 > gpurun_out/r03t_adj$cw.log 2>&1 || { tail -20 gpurun_out/r03t_adj$cw.log; exit 1; }
  python3 - "$cw" <<'PY'
import csv, sys
cw = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/r03t_adj{cw}/run_kernel_stats.csv")))
for r in rows:
    if "adjoint_local" in r["Name"]:
        print("cw", cw, r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
  rm -f gpurun_out/r03t_adj$cw/run_kernel_trace.csv
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_predict.py tests/test_gpu_driver.py > gpurun_out/r03t_tests.log 2>&1 || { tail -40 gpurun_out/r03t_tests.log; exit 1; }
tail -1 gpurun_out/r03t_tests.log
