#!/bin/bash
# BASELINE config 4 (EEG shape: N = 1e5, M = 512, P = 64) per rank of the 8-GPU job, on one GPU:
# the 1-GPU line, then ranks 0, 3 and 7 of the 8-way assignment with given and with chained
# inference inputs (bench.py --shard R/8).  Usage (on the GPU box):
#   bash tools/eeg_per_rank.sh <tag>      -> gpurun_out/<tag>/eeg_*.json
set -e
TAG=${1:-eeg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 240 python -u bench.py --config eeg --steps 2 --warmup 1 > "$OUT/eeg_1gpu.json" 2> "$OUT/eeg_1gpu.err"
for R in 0 3 7; do
  for INF in given chained; do
    timeout -k 10 240 python -u bench.py --config eeg --shard $R/8 --inference $INF --steps 3 --warmup 1 \
      > "$OUT/eeg_shard${R}of8_$INF.json" 2> "$OUT/eeg_shard${R}of8_$INF.err"
  done
done
