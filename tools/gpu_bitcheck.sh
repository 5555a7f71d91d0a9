# Bit-identity of the in-tree library against gpar-at-scale_amd/ab_old/ (a saved earlier build; AB_OLD=<dir> for another) on
# tools/lib_bitcheck.py's workload, then the GPU suite subset given as arguments and the default
# bench line.   bash tools/gpu_bitcheck.sh <tag> [tests ...]
# BITCHECK_TOLS="key_prefix=rtol ..." lets named outputs move within rounding (lib_bitcheck.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
GPAR_HIP_LIB=${AB_OLD:-$PWD/gpar-at-scale_amd/ab_old}/libgparhip.so timeout -k 10 300 python tools/lib_bitcheck.py run $OUT/old.npz > $OUT/bit_old.txt 2>&1 || { echo OLD RUN FAILED; tail -20 $OUT/bit_old.txt; exit 1; }
timeout -k 10 300 python tools/lib_bitcheck.py run $OUT/new.npz > $OUT/bit_new.txt 2>&1 || { echo NEW RUN FAILED; tail -20 $OUT/bit_new.txt; exit 1; }
python tools/lib_bitcheck.py compare $OUT/old.npz $OUT/new.npz $BITCHECK_TOLS | tee $OUT/bitcheck.txt
if [ $# -gt 0 ]; then
  timeout -k 10 1500 python -u -m pytest "$@" -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.txt; exit 1; }
  tail -3 $OUT/pytest.txt
fi
timeout -k 10 700 python bench.py --no-cpu-baseline --h2h-steps 0 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench.json'))
print('bench', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],4), json.dumps({k:round(x,1) for k,x in d['fit_rounds']['marks_ms_per_step'].items()}), 'pred', round(d['roofline_predict'].get('wall_ms_per_step',0),1))"
