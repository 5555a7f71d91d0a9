# Device Nelder-Mead for the chains fit: its GPU tests, the ssm line with device_nm 1 / 0 (twice
# each, alternating) and the round-boundary trace.   bash tools/gpu_device_nm.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_nm.py tests/test_gpu_predict.py tests/test_gpu_schedule.py tests/test_gpu_edges.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for rep in 1 2; do
  for v in 1 0; do
    timeout -k 10 200 python bench.py --config ssm --steps 5 --warmup 2 --no-cpu-baseline --schedule device_nm=$v > $O/ssm_nm${v}_$rep.json 2>> $O/ab.err || { echo BENCH FAILED; tail -5 $O/ab.err; exit 1; }
    python3 -c "
import json;d=json.load(open('$O/ssm_nm${v}_$rep.json'));print('device_nm $v', round(d['ms_per_step'],2), 'logpdf', round(d['roofline']['ms_per_step'],2), 'smooth', round(d['roofline_smooth']['avg_ms'],2))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 bench.py --config ssm --steps 1 --warmup 1 --no-cpu-baseline > $O/ssm_trace.json 2> $O/ssm_trace.err || { echo TRACE FAILED; tail -20 $O/ssm_trace.err; exit 1; }
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
python tools/trace_ssm_rounds.py "$f" > $O/rounds.txt && cat $O/rounds.txt
rm -rf $O/tr
