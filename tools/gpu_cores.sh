# r-cache: tests + one/two-lane A/B on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_dist_cache.py tests/test_gpu_driver.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_rc.txt 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/pytest_rc.txt; exit 1; }
tail -1 gpurun_out/pytest_rc.txt
run() { # tag, lanes
  timeout -k 10 400 python bench.py --steps 1 --no-cpu-baseline --lanes $2 > gpurun_out/b_$1.json 2> gpurun_out/b_$1.err || { echo BENCH $1 FAILED; tail -20 gpurun_out/b_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b_$1.json')); print('$1', round(d['ms_per_step']), {k: round(v) for k, v in d['kernels'].items()})"
}
run l1 1
run l2 2
run l1b 1
run l2b 2
