#!/bin/bash
# r03l: re-created container, HEAD rebuilt: full GPU suite, smoke, a two-step north bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; tail -40 gpurun_out/pytest_gpu.txt; exit 1; }
tail -1 gpurun_out/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { echo SMOKE FAILED; tail -20 gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03l_north.json 2> gpurun_out/r03l_north.err || { echo BENCH FAILED; tail -20 gpurun_out/r03l_north.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r03l_north.json"))
rp = d.get("roofline_predict", {})
print(round(d["ms_per_step"], 1), d["value"], "gram", round(d["roofline"]["avg_ms"], 3), "pred wall", rp.get("wall_ms_per_step"),
      {k: round(x["ms_per_step"], 1) for k, x in rp.items() if isinstance(x, dict) and "ms_per_step" in x})
PY
