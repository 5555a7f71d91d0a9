# Variant check: GPU parity tests that exercise the Gram on gpar-at-scale_amd/abl/libgparhip_$VAR.so,
# then the objective probe (N=1e6, M=512) on the tree library and the variant, twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$VAR.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dtc.py tests/test_gpu_golden.py tests/test_gpu_dist_cache.py tests/test_gpu_fullsize.py tests/test_gpu_driver.py -x -q --timeout 300 --timeout-method thread > gpurun_out/var_tests.txt 2>&1 || { tail -30 gpurun_out/var_tests.txt; exit 1; }
tail -1 gpurun_out/var_tests.txt
rm -f gpurun_out/var_probe.txt
for rep in 1 2; do
  for lib in base $VAR; do
    if [ $lib = base ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_$lib.so; fi
    echo -n "$lib " >> gpurun_out/var_probe.txt
    timeout -k 10 200 python tools/gram_probe.py --evals 10 --d ${D:-32} 2>/dev/null >> gpurun_out/var_probe.txt || exit 1
  done
done
sed 's/dtc=.*gram/gram/; s/gains:.*//' gpurun_out/var_probe.txt
