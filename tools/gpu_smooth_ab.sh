# smooth_back / gains changes: the ssm A/B and trace (tools/gpu_device_nm.sh), then the north
# line under rocprof for the Matern-5/2 smoother of output 1 (smooth_back<3>).
#   bash tools/gpu_smooth_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
bash tools/gpu_device_nm.sh $1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --h2h-steps 0 > $O/north_prof.json 2> $O/north_prof.err || { echo ROCPROF FAILED; tail -5 $O/north_prof.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/north_stats.csv \;
rm -rf $O/prof
python3 -c "
import csv
for r in csv.DictReader(open('$O/north_stats.csv')):
    if any(k in r['Name'] for k in ('smooth_back','gains_phase1','gains_phase2','gains_phase3')):
        print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
