set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
for v in "" "--separate-predict"; do
  timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline $v > gpurun_out/bfp.json 2> gpurun_out/bfp.err || { tail gpurun_out/bfp.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bfp.json'));print('$v', round(d['ms_per_step'],1), d['kernels'])"
done
