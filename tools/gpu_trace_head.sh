# Kernel trace of a short north fit (8 evaluations, one step, no warm-up) and the round-boundary
# timeline (tools/trace_rounds.py), and the gains launches by grid size (tools/trace_kernels.py).
# BENCH_ARGS adds bench.py arguments (e.g. "--config eeg --shard 0/8"; its between-Gram gaps by
# tools/trace_gaps.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-trace}
rm -rf gpurun_out/$tag
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/$tag -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --evals ${EVALS:-8} --no-cpu-baseline --h2h-steps 0 ${BENCH_ARGS} > gpurun_out/${tag}.json 2> gpurun_out/${tag}.err || { echo TRACE FAILED; tail -20 gpurun_out/${tag}.err; exit 1; }
f=$(find gpurun_out/$tag -name "*kernel_trace.csv" | head -1)
echo "trace: $f"
python tools/trace_rounds.py "$f" --top 25 > gpurun_out/${tag}_rounds.txt
python tools/trace_gaps.py "$f" --top 25 > gpurun_out/${tag}_gaps.txt
cat gpurun_out/${tag}_gaps.txt
cat gpurun_out/${tag}_rounds.txt | head -120
python tools/trace_kernels.py "$f" --match gains --top 20 > gpurun_out/${tag}_gains.txt
cat gpurun_out/${tag}_gains.txt
rm -rf gpurun_out/$tag
