# PMC passes over the Gram and whitening kernels at the stress config's shape (BASELINE config 5:
# N = 1e7, M = 1024; D = 8: the Gram does not depend on D), two objective evaluations of one output
# (tools/gram_probe.py), one counter group per rocprofv3 run; summarised by tools/pmc_sq.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_stress}
mkdir -p $OUT
KRE="gram|whiten_kfu"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -d $OUT/$name -o run --output-format csv -- python3 tools/gram_probe.py --n 10000000 --m 1024 --d 8 --evals 2 > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
}
run sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
PMC_SOURCE="tools/pmc_stress.sh: rocprofv3 --pmc passes over tools/gram_probe.py --n 10000000 --m 1024 --d 8 --evals 2 (two objective evaluations of one output at the stress config's N and M, whole chip; the whitening is the fused kernel at D = 8, its algorithmic bytes below assume the cached form); " PMC_N=10000000 PMC_M=1024 PMC_D=8 python3 tools/pmc_sq.py $OUT > $OUT/summary.json && cat $OUT/summary.json
