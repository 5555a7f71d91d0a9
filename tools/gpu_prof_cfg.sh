# rocprofv3 kernel stats of one bench config: CFG=eeg bash tools/gpu_prof_cfg.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$CFG -o run --output-format csv -- python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_$CFG.json 2> gpurun_out/bench_prof_$CFG.err || { tail -20 gpurun_out/bench_prof_$CFG.err; exit 1; }
cat gpurun_out/bench_prof_$CFG.json
