# One rank's shard (--shard R/W) under schedule strings, one bench line each (one timed step after
# one warm-up).  bash tools/gpu_shard_ab.sh <tag> <R/W> "<k=v,...>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:?tag}
SH=${2:?R/W}
shift 2
i=0
for s in "$@"; do
  timeout -k 10 300 python bench.py --shard $SH --steps 1 --warmup 1 --no-cpu-baseline --h2h-steps 0 --schedule "$s" > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$i.json'));print('shard $SH [$s]', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],4), 'whiten', round(d['roofline_whiten']['avg_ms'],4), 'fit_call', round(d['fit_calls']['ms_per_step'],1))"
  i=$((i+1))
done
