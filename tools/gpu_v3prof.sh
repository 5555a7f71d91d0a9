# Per-kernel times of the Gram from a short objective probe under rocprofv3, for the tree library
# and the variants in $VARS (gpar-at-scale_amd/abl/libgparhip_<var>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in base $VARS; do
  if [ $lib = base ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$lib.so; fi
  rm -rf gpurun_out/v3prof_$lib
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/v3prof_$lib -o run --output-format csv -- python3 tools/gram_probe.py --evals 10 --d ${D:-3} > gpurun_out/v3prof_$lib.txt 2>&1 || { tail -20 gpurun_out/v3prof_$lib.txt; exit 1; }
  f=$(find gpurun_out/v3prof_$lib -name '*kernel_stats.csv' | head -1)
  echo "== $lib"
  python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs'])):
    if 'gram' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
PY
done
