# Multi-rank rehearsal on one GPU (gloo, every rank on device 0): the bench launcher, output
# sharding, shared-input broadcasts, theta gathers and the chained predictions across ranks
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for args in "--config small --gpus 2" "--config small --gpus 2 --inference chained" "--config eeg --gpus 4 --steps 1 --warmup 1" "--config ssm --gpus 2 --steps 1 --warmup 1"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 400 python bench.py --rehearse --no-cpu-baseline $args > gpurun_out/reh_$tag.json 2> gpurun_out/reh_$tag.err || { echo REHEARSAL $tag FAILED; tail -30 gpurun_out/reh_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/reh_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['n_gpus'], round(d['ms_per_step'], 1), d['config']['outputs_per_rank'] if len(str(d['config']['outputs_per_rank'])) < 200 else '...')"
done
