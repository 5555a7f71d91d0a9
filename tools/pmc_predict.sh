# PMC passes over the prediction kernels: tools/predict_probe.py, two outputs
# at D = 62, 63 (the fused whitening's DP = 64 bucket) at N = N* = 1e6, M = 512, one evaluation
# each, so the merged-grid (2e6-row) whitening whiten_kfu_mfma, the adjoint pass, the rows and the
# variance GEMM dominate; one counter group per rocprofv3 run; summarised by tools/pmc_predict.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcp
KRE="whiten_kfu_mfma|adjoint_local_wide|predict_rows|gemm_nt|predict_var"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -d gpurun_out/pmcp/$name -o run --output-format csv -- python3 tools/predict_probe.py --outputs 2 --dmin 62 --reps 1 > gpurun_out/pmcp/$name.log 2>&1 || { echo "pass $name failed"; tail -5 gpurun_out/pmcp/$name.log; exit 1; }
}
run sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
# LDS pass last and optional (the summary reads it when present)
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "$KRE" -d gpurun_out/pmcp/lds -o run --output-format csv -- python3 tools/predict_probe.py --outputs 2 --dmin 62 --reps 1 > gpurun_out/pmcp/lds.log 2>&1 || echo "lds pass failed (skipped)"
python3 tools/pmc_predict.py gpurun_out/pmcp > gpurun_out/pmcp/summary.json && cat gpurun_out/pmcp/summary.json
