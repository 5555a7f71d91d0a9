# Kernel timeline of a few Gram launches (rocprofv3 kernel trace) for the library $LIB
# (default: the tree's), objective probe at N=1e6, M=512, D=32
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$LIB" ] && export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$LIB.so
rm -rf gpurun_out/trace_gram
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace_gram -o run --output-format csv -- python3 tools/gram_probe.py --evals 4 --d 32 > gpurun_out/trace_gram.txt 2>&1 || { tail -20 gpurun_out/trace_gram.txt; exit 1; }
f=$(find gpurun_out/trace_gram -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=[r for r in csv.DictReader(open(sys.argv[1])) if 'gram' in r['Kernel_Name']]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
t0=None
for r in rows[-12:]:
    s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
    if t0 is None: t0=s
    print(r['Kernel_Name'][:34].ljust(34), 'start %8.1f us  end %8.1f us  dur %7.1f us' % ((s-t0)/1e3,(e-t0)/1e3,(e-s)/1e3))
PY
