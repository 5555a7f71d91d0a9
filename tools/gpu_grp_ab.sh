# A/B of the grouped Gram's plan (GPAR_GRP_CUS_PCT) at the eeg shard 0/8 and the 1-GPU eeg, plus a
# rocprof kernel summary of the shard.   bash tools/gpu_grp_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config eeg --shard 0/8 --steps 2 --warmup 1 > $O/prof_eeg_s0.json 2> $O/prof.err || exit 1
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/rocprof_eeg_s0_stats.csv \;
rm -rf $O/prof
for pct in 100 200 50 100 200 50 400; do
  GPAR_GRP_CUS_PCT=$pct timeout -k 10 200 python bench.py --config eeg --shard 0/8 --steps 3 --warmup 1 > $O/eeg_s0_$pct.json 2>> $O/ab.err || exit 1
  python3 -c "
import json;d=json.load(open('$O/eeg_s0_$pct.json'));print('pct $pct', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), round(d['roofline']['frac'],3))"
done
