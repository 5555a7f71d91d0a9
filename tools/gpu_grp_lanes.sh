# A/B: the grouped Gram's whitenings over 2 or 3 streams (GPAR_GRP_LANES) at the 1-GPU eeg, the eeg
# shard and dtc, alternating.   bash tools/gpu_grp_lanes.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:?tag}
mkdir -p $O
one() {  # lanes, name, bench args...
  local l=$1 name=$2; shift 2
  GPAR_GRP_LANES=$l timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > $O/${name}_$l.json 2>> $O/ab.err || { echo BENCH FAILED; tail -5 $O/ab.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/${name}_$l.json'));print('$name lanes $l', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), 'not_gram', round(d['fit_calls']['not_gram_ms_per_step'],1))"
}
for r in 1 2; do
  for l in 3 2; do one $l eeg --config eeg --steps 2 --warmup 1; done
done
for l in 3 2 3 2; do one $l dtc --config dtc --steps 3 --warmup 1; done
for l in 3 2; do one $l eeg_s0 --config eeg --shard 0/8 --steps 3 --warmup 1 --schedule overlap=0; done
