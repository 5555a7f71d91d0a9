# Grouped-Gram configs after a plan change: the schedule / dtc / driver GPU tests, then the dtc,
# eeg and eeg-per-rank lines.   bash tools/gpu_r06_eeg.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_dtc.py tests/test_gpu_driver.py tests/test_gpu_golden.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
run() {  # name, seconds, bench args...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name FAILED"; tail -5 $O/$name.err; exit 1; }
}
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
