# One bench line per (config, schedule string), same box, after a GPU test subset:
#   TAG=x bash tools/gpu_sched_cfg_ab.sh "tests ..." "cfg:k=v,k=v" "cfg:" ...
# (an empty schedule after the colon = the defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sab}
mkdir -p $OUT
if [ -n "$1" ]; then
  timeout -k 10 1200 python -u -m pytest $1 -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.txt; exit 1; }
  tail -2 $OUT/pytest.txt
fi
shift
i=0
for cs in "$@"; do
  cfg=${cs%%:*}; sch=${cs#*:}
  timeout -k 10 700 python bench.py --config $cfg --no-cpu-baseline --h2h-steps 0 ${sch:+--schedule $sch} > $OUT/b$i.json 2> $OUT/b$i.err || { echo "bench $cs failed"; tail -20 $OUT/b$i.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$OUT/b$i.json'))
fr=d.get('fit_rounds') or {}; r=d.get('roofline') or {}
print('$cs', round(d['ms_per_step'],2), 'gram', round(r.get('avg_ms') or 0,4), 'frac', round(r.get('frac') or 0,3), 'launches', r.get('launches'), 'head', round(fr.get('head_ms_per_step') or 0,1), 'pred', round((d.get('roofline_predict') or {}).get('wall_ms_per_step',0),1))"
  i=$((i+1))
done
