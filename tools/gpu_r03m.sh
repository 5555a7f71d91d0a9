#!/bin/bash
# r03m: predict_var with the carry term after the k-loop (C_j = chat_j V^T, one triangular GEMM per
# prediction) vs per k-step: full GPU suite, smoke, one-lane rocprof A/B on the predict probe, and
# the north job (two steps) with GPAR_PREDICT_VAR_EPI=1 / 0 on the same box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; tail -40 gpurun_out/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
for v in 1 0; do
  GPAR_PREDICT_LANES=1 GPAR_PREDICT_VAR_EPI=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03m_prof_e$v -o run --output-format csv -- \
    python3 tools/predict_probe.py --outputs 8 --dmin 30 --reps 3 > gpurun_out/r03m_prof_e$v.log 2>&1 || { tail -20 gpurun_out/r03m_prof_e$v.log; exit 1; }
  echo "epi $v"; grep rep gpurun_out/r03m_prof_e$v.log
done
python3 - <<'PY'
import csv
for v in (1, 0):
    rows = list(csv.DictReader(open(f"gpurun_out/r03m_prof_e{v}/run_kernel_stats.csv")))
    print("epi", v, [(r["Name"][:28], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3)) for r in rows[:14]])
PY
for v in 1 0; do
  GPAR_PREDICT_VAR_EPI=$v timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03m_north_e$v.json 2> gpurun_out/r03m_north_e$v.err || { echo BENCH FAILED; tail -20 gpurun_out/r03m_north_e$v.err; exit 1; }
done
python3 - <<'PY'
import json
for v in (1, 0):
    d = json.load(open(f"gpurun_out/r03m_north_e{v}.json"))
    rp = d.get("roofline_predict", {})
    print("epi", v, round(d["ms_per_step"], 1), d["value"], "gram", round(d["roofline"]["avg_ms"], 3), "pred wall", rp.get("wall_ms_per_step"),
          {k: round(x["avg_ms"], 2) for k, x in rp.items() if isinstance(x, dict) and "avg_ms" in x})
PY
