#!/bin/bash
# r03e: prediction tail -- PMC passes over the merged-grid kernels, lanes A/B on the probe (8
# outputs, D 30..37), north with the predictions' wall-time span, shard 1/8 with the overlap gate.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 2; do
  GPAR_PREDICT_LANES=$v timeout -k 10 200 python -u tools/predict_probe.py --outputs 8 --dmin 30 --reps 3 \
    > gpurun_out/r03e_probe_l$v.log 2>&1 || { tail -20 gpurun_out/r03e_probe_l$v.log; exit 1; }
  echo "lanes $v"; cat gpurun_out/r03e_probe_l$v.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03e_prof -o run --output-format csv -- \
  python3 tools/predict_probe.py --outputs 8 --dmin 30 --reps 2 > gpurun_out/r03e_prof.log 2>&1 || { tail -20 gpurun_out/r03e_prof.log; exit 1; }
for v in 2 1; do
  GPAR_PREDICT_LANES=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r03e_north_l$v.json 2> gpurun_out/r03e_north_l$v.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --shard 1/8 \
  > gpurun_out/r03e_shard.json 2> gpurun_out/r03e_shard.err || exit 1
python - <<'PY'
import json
for f in ("north_l2", "north_l1", "shard"):
    d = json.load(open(f"gpurun_out/r03e_{f}.json"))
    rp = d.get("roofline_predict", {})
    print(f, round(d["ms_per_step"], 1), d["value"], d["roofline"]["avg_ms"], rp.get("wall_ms_per_step"),
          {k: round(v["ms_per_step"], 1) for k, v in rp.items() if isinstance(v, dict)})
PY
bash tools/pmc_predict.sh > gpurun_out/r03e_pmc.log 2>&1 || { tail -20 gpurun_out/r03e_pmc.log; exit 1; }
tail -3 gpurun_out/r03e_pmc.log
