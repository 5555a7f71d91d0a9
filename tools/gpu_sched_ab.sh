# Schedule A/B at the north config on one box: one bench line (one timed step after one warm-up) per
# schedule string.  bash tools/gpu_sched_ab.sh <tag> "<k=v,k=v>" "<k=v>" ...   ("" = the defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:?tag}
shift
i=0
for s in "$@"; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --h2h-steps 0 --schedule "$s" > gpurun_out/${TAG}_$i.json 2> gpurun_out/${TAG}_$i.err || { tail -20 gpurun_out/${TAG}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$i.json'));print('[$s]', round(d['ms_per_step'],1), round(d['roofline']['avg_ms'],4), round(d['roofline_whiten']['avg_ms'],4), json.dumps({k:round(v,1) for k,v in d['fit_rounds']['marks_ms_per_step'].items()}), round(d['fit_rounds']['not_gram_ms_per_step'],1))"
  i=$((i+1))
done
