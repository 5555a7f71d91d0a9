# The grouped Gram's plan rule (kGrpMinRows) on the eeg shard, dtc and the 1-GPU eeg (groups of 16
# and of 8), then the schedule / dtc GPU tests.   bash tools/gpu_grp_rule.sh <tag>
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
one eeg_s0 --config eeg --shard 0/8 --steps 3 --warmup 1
one dtc --config dtc --steps 3 --warmup 1
one eeg --config eeg --steps 2 --warmup 1
one eeg_g8 --config eeg --steps 2 --warmup 1 --schedule gram_group=8
one eeg_s0b --config eeg --shard 0/8 --steps 3 --warmup 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_dtc.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
