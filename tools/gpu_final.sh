# Round-end evidence: GPU tests, smoke, the default bench line (with cpu_baseline), a rocprofv3
# kernel-trace profile of the north bench, and the other SURVEY configs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.txt 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/pytest_gpu_final.txt; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.txt 2>&1 || { cat gpurun_out/smoke.txt; exit 1; }
tail -1 gpurun_out/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_rocprof.json 2> gpurun_out/bench_rocprof.err || { tail gpurun_out/bench_rocprof.err; exit 1; }
for c in dtc eeg ssm; do
  timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail gpurun_out/bench_$c.err; exit 1; }
done
python3 -c "
import json
for c in ['rocprof','dtc','eeg','ssm']:
    d=json.load(open('gpurun_out/bench_%s.json'%c)); print(c, round(d['ms_per_step'],1), '%.4g'%d['value'])"
