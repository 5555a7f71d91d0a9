# PMC passes over the gains kernels (gains_phase1/2/3) of a short bench run: wave-time split, VALU /
# memory counts, HBM bytes; per-kernel averages by tools/pmc_lds.py.
#   [CFG=north|ssm] [EVALS=2] [TAG=pmcg] bash tools/pmc_gains.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${CFG:-north}
EVALS=${EVALS:-2}
OUT=gpurun_out/${TAG:-pmcg}
mkdir -p $OUT
KRE="gains_phase|chain_carry_lml"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -d $OUT/$name -o run --output-format csv -- python3 bench.py --config $CFG --steps 1 --warmup 0 --evals $EVALS --no-cpu-baseline --h2h-steps 0 > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
  python3 tools/pmc_lds.py $OUT/$name > $OUT/$name.json && rm -rf $OUT/$name
}
run sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
