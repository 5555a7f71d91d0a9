# The other SURVEY §8d configs with the CU split (default) and without (--cu-split 0), one line each,
# plus a 2-rank rehearsal (gloo, both ranks on the one GPU) of the small eeg-shaped config
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CONFIGS:-dtc eeg}; do
  for w in 8 0; do
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --cu-split $w > gpurun_out/cab_${c}_$w.json 2> gpurun_out/cab_${c}_$w.err || { echo BENCH $c $w FAILED; tail -20 gpurun_out/cab_${c}_$w.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/cab_${c}_$w.json'));print('$c split=$w', round(d['ms_per_step'],1), d['value'])"
  done
done
timeout -k 10 300 python bench.py --config eeg --rehearse --gpus 2 --no-cpu-baseline > gpurun_out/rehearse_eeg2.json 2> gpurun_out/rehearse_eeg2.err || { echo REHEARSE FAILED; tail -20 gpurun_out/rehearse_eeg2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/rehearse_eeg2.json'));print('rehearse eeg 2 ranks', round(d['ms_per_step'],1), d['n_gpus'], d['config']['cu_split'])"
