# Unsplit round overlap: group sizes (overlap_group) at the eeg shard and the 1-GPU eeg.
#   bash tools/gpu_overlap_groups.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
one() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > $O/${name}.json 2>> $O/ab.err || { echo BENCH $name FAILED; tail -5 $O/ab.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/${name}.json'));print('$name', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), round(d['roofline']['frac'],3))"
}
for g in 2 3 4; do one eeg_s0_g$g --config eeg --shard 0/8 --steps 3 --warmup 1 --schedule overlap_group=$g; done
one eeg_s0_rr --config eeg --shard 0/8 --steps 3 --warmup 1 --schedule overlap=0
for g in 8 16 32; do one eeg_g$g --config eeg --steps 2 --warmup 1 --schedule overlap_group=$g; done
one dtc_g2 --config dtc --steps 3 --warmup 1 --schedule overlap_group=2
