# Split-round head variants at the north config, same box: split_head = 1 (default), 2, 0; one
# timed step each after one warm-up.  bash tools/gpu_head_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:?tag}
timeout -k 10 600 python -u -m pytest tests/test_gpu_schedule.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/pytest_$TAG.txt 2>&1 || { tail -30 gpurun_out/pytest_$TAG.txt; exit 1; }
tail -1 gpurun_out/pytest_$TAG.txt
for h in 1 2 0; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --h2h-steps 0 --schedule split_head=$h > gpurun_out/${TAG}_h$h.json 2> gpurun_out/${TAG}_h$h.err || { tail -20 gpurun_out/${TAG}_h$h.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_h$h.json'));print('split_head=$h', round(d['ms_per_step'],1), round(d['roofline']['avg_ms'],4), round(d['roofline_whiten']['avg_ms'],4), json.dumps({k:round(v,1) for k,v in d['fit_rounds']['marks_ms_per_step'].items()}), round(d['fit_rounds']['not_gram_ms_per_step'],1))"
done
