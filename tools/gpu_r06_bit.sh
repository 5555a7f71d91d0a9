# Bit-identity of the in-tree library against gpar-at-scale_amd/ab_prev/ (tools/lib_bitcheck.py's
# workload), a GPU test subset, and the eeg-shard / eeg / dtc config lines.
#   bash tools/gpu_r06_bit.sh <tag> [tests ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
shift
mkdir -p $O
GPAR_HIP_LIB=$PWD/gpar-at-scale_amd/ab_prev/libgparhip.so timeout -k 10 300 python tools/lib_bitcheck.py run $O/old.npz > $O/bit_old.txt 2>&1 || exit 1
timeout -k 10 300 python tools/lib_bitcheck.py run $O/new.npz > $O/bit_new.txt 2>&1 || exit 1
python tools/lib_bitcheck.py compare $O/old.npz $O/new.npz > $O/bitcheck.txt; cat $O/bitcheck.txt | grep -v bit-identical
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest.txt; exit 1; }
  tail -1 $O/pytest.txt
fi
for i in 1 2; do
  timeout -k 10 200 python bench.py --config eeg --shard 0/8 --steps 3 --warmup 1 >> $O/eeg_s0.jsonl 2>> $O/eeg.err || exit 1
done
timeout -k 10 200 python bench.py --config eeg --steps 2 --warmup 1 --no-cpu-baseline > $O/eeg_1gpu.json 2> $O/eeg_1gpu.err || exit 1
timeout -k 10 200 python bench.py --config dtc --steps 3 --warmup 1 --no-cpu-baseline > $O/dtc.json 2> $O/dtc.err || exit 1
python3 -c "
import json
for l in open('$O/eeg_s0.jsonl'):
  d=json.loads(l); print('eeg s0', round(d['ms_per_step'],1), 'notgram', round(d['fit_calls']['not_gram_ms_per_step'],1), 'gram avg', round(d['roofline']['avg_ms'],3))
for f in ('eeg_1gpu.json','dtc.json'):
  d=json.load(open('$O/'+f)); print(f, round(d['ms_per_step'],1), 'notgram', round(d['fit_calls']['not_gram_ms_per_step'],1), 'gram avg', round(d['roofline']['avg_ms'],3))"
