# Kernel trace of the ssm config (one step) and its round boundaries (tools/trace_ssm_rounds.py).
#   bash tools/gpu_trace_ssm.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 bench.py --config ssm --steps 1 --warmup 1 --no-cpu-baseline > $O/ssm.json 2> $O/ssm.err || { echo TRACE FAILED; tail -20 $O/ssm.err; exit 1; }
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
python tools/trace_ssm_rounds.py "$f" > $O/rounds.txt && cat $O/rounds.txt
rm -rf $O/tr
