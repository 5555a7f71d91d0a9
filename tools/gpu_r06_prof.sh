# r06 profiles: rocprofv3 kernel stats of the ssm and stress lines, the stress Gram's PMC passes,
# and the eeg shard's between-Gram trace.   bash tools/gpu_r06_prof.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ssm -o run --output-format csv -- python3 bench.py --config ssm --steps 5 --warmup 2 --no-cpu-baseline > $O/ssm_prof.json 2> $O/ssm_prof.err || { echo SSM PROF FAILED; exit 1; }
find $O/prof_ssm -name '*kernel_stats.csv' -exec cp {} $O/rocprof_ssm_stats.csv \;
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_stress -o run --output-format csv -- python3 bench.py --config stress --shard 0/8 --evals 2 --steps 1 --warmup 0 --no-cpu-baseline > $O/stress_prof.json 2> $O/stress_prof.err || { echo STRESS PROF FAILED; exit 1; }
find $O/prof_stress -name '*kernel_stats.csv' -exec cp {} $O/rocprof_stress_stats.csv \;
rm -rf $O/prof_ssm $O/prof_stress
bash tools/pmc_stress.sh $TAG/pmc_stress > $O/pmc_stress.txt 2>&1 || { echo PMC FAILED; tail -5 $O/pmc_stress.txt; exit 1; }
EVALS=50 BENCH_ARGS="--config eeg --shard 0/8" bash tools/gpu_trace_head.sh $TAG/trace_eeg > $O/trace_eeg.txt 2>&1 || exit 1
head -24 $O/trace_eeg.txt
