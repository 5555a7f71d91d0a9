# CU-split experiment: mask probe, then the north bench with GPAR_SPLIT_CUS = 0 (pipelined, whole
# chip) and the listed whitening widths (CUs per XCD), one step each; then a parity subset in the
# split mode (GPAR_SPLIT_CUS forces the width at any size)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 5 60 ./tools/ubench/cumask_probe > gpurun_out/cumask.txt 2>&1 || { cat gpurun_out/cumask.txt; exit 1; }
grep -A1 "bits 0..39\|bits 40" gpurun_out/cumask.txt | cut -c1-200
for w in ${WS:-0 4 6 8}; do
  GPAR_SPLIT_CUS=$w timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/split_$w.json 2> gpurun_out/split_$w.err || { tail gpurun_out/split_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/split_$w.json'));print('split=$w', round(d['ms_per_step'],1), 'gram', round(d['roofline']['avg_ms'],4), 'whiten', round(d['roofline_whiten']['avg_ms'],4))"
done
GPAR_SPLIT_CUS=${WT:-6} timeout -k 10 600 python -u -m pytest tests/test_gpu_driver.py tests/test_gpu_dtc.py tests/test_gpu_predict.py -x -q --timeout 300 --timeout-method thread > gpurun_out/split_tests.txt 2>&1 || { tail -30 gpurun_out/split_tests.txt; exit 1; }
tail -1 gpurun_out/split_tests.txt
