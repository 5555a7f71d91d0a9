# Pipelined Gram stage A/B: full GPU suite (pipelined default), then the north bench with
# GPAR_PIPELINE=0 / 1 alternating, one step each, ${REPS:-2} pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pipe_tests.txt 2>&1 || { tail -30 gpurun_out/pipe_tests.txt; exit 1; }
tail -1 gpurun_out/pipe_tests.txt
for rep in $(seq ${REPS:-2}); do
  for pv in 0 1; do
    GPAR_PIPELINE=$pv timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --config ${CFG:-north} > gpurun_out/pipe_$pv.json 2> gpurun_out/pipe_$pv.err || { tail gpurun_out/pipe_$pv.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/pipe_$pv.json'));print('pipeline=$pv', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],4), 'whiten', round(d['roofline_whiten']['avg_ms'],4))"
  done
done
