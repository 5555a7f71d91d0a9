# Full-size parity tests (tests/test_gpu_fullsize.py) and one bench line per SURVEY §8d config.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_fullsize.txt 2>&1 || { echo PYTEST FAILED; tail -40 gpurun_out/pytest_fullsize.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_fullsize.txt
for c in ${CONFIGS:-dtc eeg ssm}; do
  timeout -k 10 600 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo BENCH $c FAILED; tail -20 gpurun_out/bench_$c.err; exit 1; }
  cat gpurun_out/bench_$c.json
done
