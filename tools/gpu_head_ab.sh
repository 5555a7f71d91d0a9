# The round head with a cached output leading each round: the schedule tests, then the north line
# (its fit_rounds marks) twice.   bash tools/gpu_head_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_headline.py tests/test_gpu_driver.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --h2h-steps 0 > $O/north_$r.json 2> $O/north_$r.err || { echo BENCH FAILED; tail -5 $O/north_$r.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/north_$r.json'));f=d['fit_rounds'];print('north', round(d['ms_per_step'],1), 'head', round(f['head_ms_per_step'],1), json.dumps({k:round(v,1) for k,v in f['marks_ms_per_step'].items()}))"
done
