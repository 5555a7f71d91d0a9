# The unsplit round overlap: its GPU tests (and the schedule / dtc ones), then the eeg shard, dtc
# and the 1-GPU eeg lines with overlap 1 / 0.   bash tools/gpu_overlap_unsplit.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap_unsplit.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
one() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > $O/${name}.json 2>> $O/ab.err || { echo BENCH $name FAILED; tail -5 $O/ab.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/${name}.json'));print('$name', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), round(d['roofline']['frac'],3))"
}
one eeg_s0_ov --config eeg --shard 0/8 --steps 3 --warmup 1
one eeg_s0_rr --config eeg --shard 0/8 --steps 3 --warmup 1 --schedule overlap=0
one dtc_ov --config dtc --steps 3 --warmup 1
one dtc_rr --config dtc --steps 3 --warmup 1 --schedule overlap=0
one eeg_ov --config eeg --steps 2 --warmup 1 --schedule overlap_group=32
one eeg_rr --config eeg --steps 2 --warmup 1 --schedule overlap=0
