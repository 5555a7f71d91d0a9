#!/bin/bash
# r03v: predict_var's prefetching path (operands by LDS-DMA two k-steps ahead, DMA and operand reads
# by inline asm, bare s_barrier) -- prediction parity tests, then the one-lane predict probe
# against the PV_PF2=0 build (tools/build_abl.sh), then the north job.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_predict.py tests/test_gpu_driver.py tests/test_gpu_path.py > gpurun_out/r03v_tests.log 2>&1 || { tail -40 gpurun_out/r03v_tests.log; exit 1; }
tail -1 gpurun_out/r03v_tests.log
for lib in base PV_PF20; do
  if [ $lib = base ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$lib.so; fi
  GPAR_PREDICT_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03v_$lib -o run --output-format csv -- \
    python3 tools/predict_probe.py --outputs 8 --dmin 30 --reps 2 > gpurun_out/r03v_$lib.log 2>&1 || { tail -20 gpurun_out/r03v_$lib.log; exit 1; }
  python3 - "$lib" <<'PY'
import csv, sys
lib = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/r03v_{lib}/run_kernel_stats.csv")))
for r in rows:
    if "predict_var" in r["Name"]:
        print(lib, r["Name"][:30], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
  rm -f gpurun_out/r03v_$lib/run_kernel_trace.csv
done
unset GPAR_LIB_PATH
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03v_north.json 2> gpurun_out/r03v_north.err || { echo BENCH FAILED; tail -20 gpurun_out/r03v_north.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03v_north.json')); rp=d['roofline_predict']; print('north', round(d['ms_per_step'],1), 'pred', rp.get('wall_ms_per_step'), rp.get('one_lane_probe',{}).get('pred_var'), d['self_check']['max_rel'])"
