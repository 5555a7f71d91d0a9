# lanes=2 A/B at the north config and one bench line per other SURVEY §8d config
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --lanes 2 --no-cpu-baseline > gpurun_out/bench_lanes2.json 2> gpurun_out/bench_lanes2.err || { echo LANES2 FAILED; tail -20 gpurun_out/bench_lanes2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_lanes2.json')); print('lanes2', d['ms_per_step'])"
for c in dtc eeg ssm; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo BENCH $c FAILED; tail -20 gpurun_out/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_$c.json')); print('$c', d['ms_per_step'], d['value'])"
done
