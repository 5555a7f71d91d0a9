# CU-split variants, one north step each, in the order given by VARS (name:GPAR_SPLIT_CUS:GPAR_SPLIT_DGW)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARS:-base:0:0 dgw:8:1 nodgw:8:0}; do
  IFS=: read name w dgw <<< "$v"
  GPAR_SPLIT_CUS=$w GPAR_SPLIT_DGW=$dgw timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/sv_$name.json 2> gpurun_out/sv_$name.err || { tail gpurun_out/sv_$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sv_$name.json'));print('$name', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],4), 'whiten', round(d['roofline_whiten']['avg_ms'],4))"
done
if [ -n "$TESTS" ]; then
  GPAR_SPLIT_CUS=8 GPAR_SPLIT_DGW=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sv_tests.txt 2>&1 || { tail -30 gpurun_out/sv_tests.txt; exit 1; }
  tail -1 gpurun_out/sv_tests.txt
fi
