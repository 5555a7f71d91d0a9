# Round-6 config lines on one box (each BASELINE config; EEG per rank of the 8-GPU job).
#   bash tools/gpu_r06_configs.sh <tag>   -> gpurun_out/<tag>/*.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
run() {  # name, seconds, bench args...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -5 $O/$name.err; exit 1; }
}
run stress_shard0of8 600 --config stress --shard 0/8 --steps 2 --warmup 1
run stress_shard7of8 600 --config stress --shard 7/8 --steps 1 --warmup 1 --no-cpu-baseline
run ssm 200 --config ssm --steps 5 --warmup 2
run dtc 200 --config dtc --steps 3 --warmup 1
run eeg 300 --config eeg --steps 2 --warmup 1
for R in 0 3 7; do
  run eeg_shard${R}of8_given 200 --config eeg --shard $R/8 --steps 3 --warmup 1
  run eeg_shard${R}of8_chained 200 --config eeg --shard $R/8 --inference chained --steps 3 --warmup 1
done
python3 - <<PY
import glob, json, os
for f in sorted(glob.glob("$O/*.json")):
    d = json.load(open(f))
    r = d.get("roofline") or {}
    print(os.path.basename(f), round(d["ms_per_step"], 1), d["unit"], "%.3g" % d["value"],
          "frac", None if r.get("frac") is None else round(r["frac"], 3),
          "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
