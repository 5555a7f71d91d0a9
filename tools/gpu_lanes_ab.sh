# North bench (1 step): lanes=1 and lanes=2 on the tree library, lanes=2 on each of $VARS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # tag lanes
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --lanes $2 > gpurun_out/lab_$1.json 2> gpurun_out/lab_$1.err || { tail gpurun_out/lab_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/lab_$1.json'));print('$1', round(d['ms_per_step'],1), {k: round(v) for k, v in d['kernels'].items()})"
}
run base_l1 1 || exit 1
run base_l2 2 || exit 1
for v in $VARS; do
  GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$v.so run ${v}_l2 2 || exit 1
done
