# predict_var A/B: the library in gpar-at-scale_amd/ab_old/ (the previous build) against the
# current one: prediction parity tests, rocprof kernel stats of tools/predict_probe.py and one
# north bench line each.  bash tools/gpu_pvar_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_predict.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for v in old new; do
  if [ $v = old ]; then export GPAR_HIP_LIB=$PWD/gpar-at-scale_amd/ab_old/libgparhip.so; else unset GPAR_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- python3 tools/predict_probe.py --outputs 2 --dmin 62 --reps 2 > $OUT/probe_$v.log 2>&1 || { echo PROBE $v FAILED; tail -20 $OUT/probe_$v.log; exit 1; }
  f=$(find $OUT/prof_$v -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if any(k in n for k in ('predict_var','whiten_kfu_mfma','adjoint_local')): print('$v', n[:40], r['Calls'], round(float(r['AverageNs'])/1e6,4))"
done
for v in old new old new; do
  if [ $v = old ]; then export GPAR_HIP_LIB=$PWD/gpar-at-scale_amd/ab_old/libgparhip.so; else unset GPAR_HIP_LIB; fi
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --h2h-steps 0 > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { echo BENCH $v FAILED; tail -20 $OUT/bench_$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$OUT/bench_$v.json'));r=d['roofline_predict']
print('$v', round(d['ms_per_step'],1), {k:round(r[k]['avg_ms'],3) for k in ('pred_whiten','pred_adjoint','pred_var')}, round(r.get('wall_ms_per_step',0),1))"
  cp $OUT/bench_$v.json $OUT/bench_${v}_$RANDOM.json
done
