# Gram at one workgroup per CU (GPAR_GRAM_SLOTS=256): timing ablations 6 (no K-step barrier) and 7 (no LDS-DMA)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for k in 0 6 7; do
  if [ $k = 0 ]; then unset GPAR_LIB_PATH; else export GPAR_LIB_PATH=$PWD/gpar-at-scale_amd/abl/libgparhip_GRAM_ABL$k.so; fi
  for sl in 512 256; do
    GPAR_GRAM_SLOTS=$sl timeout -k 10 200 python tools/gram_probe.py --evals 10 2>&1 | grep N= | sed "s/^/ABL=$k slots=$sl /" | cut -c1-120
  done
done
