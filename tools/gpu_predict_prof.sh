# Prediction-kernel profile (tools/predict_probe.py under rocprofv3 --stats) for the tree library and
# the variants in $VARS (gpar-at-scale_amd/abl/libgparhip_<var>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in base $VARS; do
  if [ $lib = base ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$lib.so; fi
  rm -rf gpurun_out/pp_$lib
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pp_$lib -o run --output-format csv -- python3 tools/predict_probe.py > gpurun_out/pp_$lib.txt 2>&1 || { tail -20 gpurun_out/pp_$lib.txt; exit 1; }
  f=$(find gpurun_out/pp_$lib -name '*kernel_stats.csv' | head -1)
  echo "== $lib"
  python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:8]:
    print(r['Name'][:44].ljust(44), r['Calls'].rjust(5), round(float(r['AverageNs'])/1e3,1),'us')
PY
done
