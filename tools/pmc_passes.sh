# PMC passes (one counter group per rocprofv3 run, MI355X_MICROARCH.md PMC slots) over the Gram
# and whitening kernels of a 4-evaluation batched gpar_fit of 3 outputs (tools/gram_probe.py --fit
# --batch 3: N=1e6, M=512, D=32, the CU-split Gram stage, so the whitening reads the fit's distance cache); summarised by tools/pmc_sq.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
KRE="gram|whiten_kfu"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -d gpurun_out/pmc/$name -o run --output-format csv -- python3 tools/gram_probe.py --fit --evals 4 --batch 3 > gpurun_out/pmc/$name.log 2>&1 || { echo "pass $name failed"; tail -5 gpurun_out/pmc/$name.log; exit 1; }
}
run sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
python3 tools/pmc_sq.py gpurun_out/pmc > gpurun_out/pmc/summary.json && cat gpurun_out/pmc/summary.json
