# The staggered chained schedule measured one rank at a time (bench.py --shard R/W --inference
# chained: that rank's fits + posteriors, then the whole ordered sweep) for ranks covering every
# block size, then the W-GPU projection (tools/chained_projection.py), and a 2-rank rehearsal of the
# staggered sweep on one GPU over gloo.   TAG=x W=8 RANKS="0 3 7" bash tools/gpu_chained.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-chained}
W=${W:-8}
mkdir -p $OUT
lines=""
for r in ${RANKS:-0 3 7}; do
  timeout -k 10 900 python bench.py --shard $r/$W --inference chained --no-cpu-baseline --h2h-steps 0 > $OUT/shard$r.json 2> $OUT/shard$r.err || { echo "shard $r failed"; tail -20 $OUT/shard$r.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$OUT/shard$r.json'));c=d['chained_sweep']
print('shard $r/$W', round(d['ms_per_step'],1), 'fit', round(c['fit_ms_per_step'],1), 'sweep', round(c['ms_per_step'],1), 'per', round(c['sweep_ms_per_output'],2), 'proj', round(c['projected_step_ms'],1))"
  lines="$lines $OUT/shard$r.json"
done
python3 tools/chained_projection.py $W $lines > $OUT/projection.json && cat $OUT/projection.json
timeout -k 10 600 python bench.py --rehearse --gpus 2 --config small --inference chained > $OUT/rehearse2.json 2> $OUT/rehearse2.err || { echo "rehearsal failed"; tail -20 $OUT/rehearse2.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/rehearse2.json')); print('rehearsal', round(d['ms_per_step'],1), [ (r.get('rank'), r.get('fit_ms'), r.get('sweep_ms')) for r in d['ranks']])"
