# Library A/B at the north config: a variant build in gpar-at-scale_amd/ab_var/ (GPAR_HIP_LIB)
# against the current one, alternating, one bench line each (one timed step after one warm-up),
# then the schedule test on the variant.  bash tools/gpu_lib_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
VAR=$PWD/gpar-at-scale_amd/ab_var/libgparhip.so
i=0
for v in cur var cur var; do
  if [ $v = var ]; then export GPAR_HIP_LIB=$VAR; else unset GPAR_HIP_LIB; fi
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --h2h-steps 0 > $OUT/b${i}_$v.json 2> $OUT/b${i}_$v.err || { echo BENCH $v FAILED; tail -20 $OUT/b${i}_$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$OUT/b${i}_$v.json'))
print('$v', round(d['ms_per_step'],1), round(d['roofline']['avg_ms'],4), round(d['roofline_whiten']['avg_ms'],4), json.dumps({k:round(x,1) for k,x in d['fit_rounds']['marks_ms_per_step'].items()}), round(d['roofline_predict'].get('wall_ms_per_step',0),1))"
  i=$((i+1))
done
export GPAR_HIP_LIB=$VAR
timeout -k 10 400 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_var.txt 2>&1 || { echo PYTEST FAILED; tail -30 $OUT/pytest_var.txt; exit 1; }
tail -1 $OUT/pytest_var.txt
