# Round-overlap groups at the north config: round by round (auto at 63 outputs) vs K groups of
# g outputs (overlap_group = g), one timed step each after one warm-up, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ov}
shift
for g in "$@"; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --h2h-steps 0 --schedule overlap_group=$g > gpurun_out/${tag}_g$g.json 2> gpurun_out/${tag}_g$g.err || { echo BENCH g=$g FAILED; tail -20 gpurun_out/${tag}_g$g.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${tag}_g$g.json'));print('g=$g', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), d.get('fit_rounds'))"
done
