#!/bin/bash
# r03i: the north job once each with the reference's noise-free q(u)
# (--qu-noise-free: NOT_PD or a time), the per-output API with host inputs (a reference caller's
# loop through the shim), and the two-rank rehearsal on one GPU (gloo; each rank's cache budget
# sees the other's allocations).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# (the --qu-noise-free run: profiles/bench_r03i_north_qu_noise_free.json, NOT_PD at q(u))
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --api per-output --inputs host \
  > gpurun_out/r03i_perout_host.json 2> gpurun_out/r03i_perout_host.err || { tail -20 gpurun_out/r03i_perout_host.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03i_perout_host.json')); print('per-output host', round(d['ms_per_step'],1), d['value'])"
timeout -k 10 700 python -u bench.py --rehearse --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r03i_reh2.json 2> gpurun_out/r03i_reh2.err || { tail -30 gpurun_out/r03i_reh2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r03i_reh2.json').read().strip().splitlines()[-1]); print('rehearse 2', d['n_gpus'], round(d['ms_per_step'],1), d.get('memory'))"
