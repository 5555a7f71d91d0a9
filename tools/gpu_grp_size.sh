# Grouped Gram group size A/B (schedule gram_group) on the 1-GPU eeg and the eeg shard.
#   bash tools/gpu_grp_size.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:?tag}
mkdir -p $O
one() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 200 python bench.py "$@" --no-cpu-baseline > $O/${name}.json 2>> $O/ab.err || exit 1
  python3 -c "
import json;d=json.load(open('$O/${name}.json'));print('$name', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), round(d['roofline']['frac'],3))"
}
for g in 4 6 8 12; do one eeg_g$g --config eeg --steps 2 --warmup 1 --schedule gram_group=$g; done
one eeg_s0_g4 --config eeg --shard 0/8 --steps 3 --warmup 1 --schedule gram_group=4
one eeg_g8b --config eeg --steps 2 --warmup 1 --schedule gram_group=8
