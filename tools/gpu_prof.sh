set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 0 1 2 3 4; do
  if [ $k = 0 ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_WHITEN_ABL$k.so; fi
  echo "ABL=$k" >> gpurun_out/abl.txt
  timeout -k 10 200 python tools/gram_probe.py --evals 10 >> gpurun_out/abl.txt 2>&1 || exit 1
done
unset GPAR_LIB_PATH
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r01d -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_rocprof.json 2> gpurun_out/bench_rocprof.err || exit 1
cat gpurun_out/abl.txt; cat gpurun_out/bench_rocprof.json
