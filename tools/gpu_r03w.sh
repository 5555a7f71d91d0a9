#!/bin/bash
# r03w: the round-overlapping fit for the whole 63-output north call (GPAR_OVERLAP_MAX=64): equal
# halves vs a small second group (GPAR_OVERLAP_B = 8, 4) vs the round-by-round default; same box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03w_$tag.json 2> gpurun_out/r03w_$tag.err || { echo BENCH $tag FAILED; tail -20 gpurun_out/r03w_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03w_$tag.json')); print('$tag', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],3), 'pred', d['roofline_predict'].get('wall_ms_per_step'), d['self_check']['max_rel'])"
}
run base GPAR_OVERLAP_MAX=16 || exit 1
run ov_halves GPAR_OVERLAP_MAX=64 GPAR_OVERLAP_B=0 || exit 1
run ov_b8 GPAR_OVERLAP_MAX=64 GPAR_OVERLAP_B=8 || exit 1
run ov_b4 GPAR_OVERLAP_MAX=64 GPAR_OVERLAP_B=4 || exit 1
run base2 GPAR_OVERLAP_MAX=16 || exit 1
