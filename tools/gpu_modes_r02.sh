# The bench's other modes with the CU split default, one short step each (no warm-up): MC
# predictions, chained inference inputs, host-memory inputs, and a 2-rank rehearsal (eeg config:
# two north-size ranks on one GPU would each budget the whole HBM for their distance caches)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in "--predict mc" "--inference chained" "--inputs host" "--rehearse --gpus 2 --config eeg"; do
  tag=$(echo $m | tr -d '-' | tr ' ' '_')
  timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline $m > gpurun_out/mode_$tag.json 2> gpurun_out/mode_$tag.err || { echo "MODE $m FAILED"; tail -20 gpurun_out/mode_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/mode_$tag.json'));print('$m', round(d['ms_per_step'],1), d['n_gpus'], d['config'].get('cu_split'))"
done
