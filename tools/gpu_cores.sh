# A/B: non-temporal loads/stores in the cached whitening (D2_NT=1 library variant), one box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
NT=$PWD/gpar-at-scale_amd/abl/libgparhip_D2_NT1.so
for i in 1 2; do
  timeout -k 10 200 python tools/gram_probe.py --fit --evals 10 2>&1 | grep N= | sed 's/^/base /' | cut -c1-160
  GPAR_LIB_PATH=$NT timeout -k 10 200 python tools/gram_probe.py --fit --evals 10 2>&1 | grep N= | sed 's/^/nt   /' | cut -c1-160
done
