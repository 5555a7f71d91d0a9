#!/bin/bash
# r03p: predict_var timing ablations (PV_ABL, tools/build_abl.sh): which part of the k-loop sets
# its time -- the A-operand loads (1), the V slab DMA (2), the per-step wait + barrier (3), the
# MFMAs (4) -- on the one-lane predict probe (8 outputs, N = N* = 1e6).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in base PV_ABL1 PV_ABL2 PV_ABL3 PV_ABL4; do
  if [ $lib = base ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$lib.so; fi
  GPAR_PREDICT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03p_$lib -o run --output-format csv -- \
    python3 tools/predict_probe.py --outputs 8 --dmin 30 --reps 2 > gpurun_out/r03p_$lib.log 2>&1 || { tail -20 gpurun_out/r03p_$lib.log; exit 1; }
  python3 - "$lib" <<'PY'
import csv, sys
lib = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/r03p_{lib}/run_kernel_stats.csv")))
for r in rows:
    if "predict_var" in r["Name"]:
        print(lib, r["Name"][:30], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
done
