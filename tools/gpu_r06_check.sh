# r06 check on one box: a GPU test subset, the ssm and eeg-shard lines, and the eeg shard's
# between-Gram trace.   bash tools/gpu_r06_check.sh <tag> [tests ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest.txt; exit 1; }
  tail -1 $O/pytest.txt
fi
timeout -k 10 200 python bench.py --config ssm --steps 5 --warmup 2 > $O/ssm.json 2> $O/ssm.err || exit 1
timeout -k 10 200 python bench.py --config eeg --shard 0/8 --steps 3 --warmup 1 > $O/eeg_s0.json 2> $O/eeg_s0.err || exit 1
EVALS=50 BENCH_ARGS="--config eeg --shard 0/8" bash tools/gpu_trace_head.sh $TAG/trace_eeg > $O/trace_eeg.txt 2>&1 || exit 1
python3 -c "
import json
d=json.load(open('$O/ssm.json')); print('ssm', round(d['ms_per_step'],2), 'logpdf', round(d['roofline']['avg_ms'],4), 'smooth', round(d['roofline_smooth']['avg_ms'],3), d.get('self_check',{}).get('ok'))
d=json.load(open('$O/eeg_s0.json')); print('eeg s0', round(d['ms_per_step'],1), round(d['fit_calls']['not_gram_ms_per_step'],1))"
head -20 $O/trace_eeg.txt
