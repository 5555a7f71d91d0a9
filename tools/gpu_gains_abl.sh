# gains-kernel durations per grid shape (rocprofv3 kernel trace of a 4-evaluation north run),
# tree library vs abl/libgparhip_$VAR.so
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in base $VAR; do
  if [ $lib = base ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$lib.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gab_$lib -o run --output-format csv -- python3 bench.py --config north --steps 1 --warmup 0 --evals 4 --no-cpu-baseline > /dev/null 2>gpurun_out/gab_$lib.err || { tail gpurun_out/gab_$lib.err; exit 1; }
done
python3 - <<'PY'
import csv,glob,collections,os
for lib in ("base", os.environ["VAR"]):
    f=glob.glob(f"gpurun_out/gab_{lib}/**/*kernel_trace.csv",recursive=True)[0]
    d=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'gains_phase' in r['Kernel_Name']:
            d[(r['Kernel_Name'].split('(')[0][-16:], r['Grid_Size_Y'])].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
    for k,v in sorted(d.items()): print(lib, k, len(v), f"avg {sum(v)/len(v):.1f} us")
PY
