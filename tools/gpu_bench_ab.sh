# Bench A/B: tree library vs gpar-at-scale_amd/abl/libgparhip_$VAR.so (north, 1 step)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in $VAR base; do
  if [ $lib = base ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$lib.so; fi
  timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --config ${CFG:-north} > gpurun_out/bab_$lib.json 2> gpurun_out/bab_$lib.err || { tail gpurun_out/bab_$lib.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bab_$lib.json'));print('$lib', round(d['ms_per_step'],1), d['kernels'])"
done
