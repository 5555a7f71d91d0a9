# r06 library A/B (one box): the in-tree build against gpar-at-scale_amd/ab_var/ (a variant build)
# on the prediction kernels (tools/whiten_ab.py), alternating; then the bit-identity check against
# gpar-at-scale_amd/ab_prev/ (tools/gpu_bitcheck.sh's workload) and the eeg / dtc config lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06g}
mkdir -p $O
VAR=$PWD/gpar-at-scale_amd/ab_var/libgparhip.so
for v in cur var cur var; do
  if [ $v = var ]; then export GPAR_HIP_LIB=$VAR; else unset GPAR_HIP_LIB; fi
  timeout -k 10 200 python tools/whiten_ab.py --dims 32 63 --reps 3 >> $O/whiten_$v.txt 2>> $O/whiten.err || exit 1
done
unset GPAR_HIP_LIB
GPAR_HIP_LIB=$PWD/gpar-at-scale_amd/ab_prev/libgparhip.so timeout -k 10 300 python tools/lib_bitcheck.py run $O/old.npz > $O/bit_old.txt 2>&1 || exit 1
timeout -k 10 300 python tools/lib_bitcheck.py run $O/new.npz > $O/bit_new.txt 2>&1 || exit 1
python tools/lib_bitcheck.py compare $O/old.npz $O/new.npz > $O/bitcheck.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --config eeg --shard 0/8 --steps 3 --warmup 1 >> $O/eeg_s0.jsonl 2>> $O/eeg.err || exit 1
done
timeout -k 10 200 python bench.py --config eeg --steps 2 --warmup 1 > $O/eeg_1gpu.json 2> $O/eeg_1gpu.err || exit 1
timeout -k 10 200 python bench.py --config dtc --steps 3 --warmup 1 > $O/dtc.json 2> $O/dtc.err || exit 1
