#!/bin/bash
# Timing-ablation variants of libgparhip.so (WHITEN_ABL / GRAM_ABL compile-time switches):
#   tools/build_abl.sh WHITEN_ABL 1 2 3 4  -> gpar-at-scale_amd/abl/libgparhip_WHITEN_ABL<k>.so
# Load one with GPAR_LIB_PATH=<path> (tools/gram_probe.py).  Not product code.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/gpar-at-scale_amd
make -C "$PKG" -j8 >/dev/null
sw=$1; shift
mkdir -p "$PKG/abl"
for k in "$@"; do
  case $sw in WHITEN_ABL) src=k_lgssm;; GRAM_ABL) src=k_gram;; *) src=$SRC;; esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -I"$ROOT/include" -I"$PKG/csrc" \
    -D$sw=$k -c "$PKG/csrc/$src.hip" -o "$PKG/abl/${src}_$sw$k.o" &
done
wait
for k in "$@"; do
  objs=$(ls "$PKG"/build/*.o | grep -v "/$src.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$PKG/abl/libgparhip_$sw$k.so" $objs "$PKG/abl/${src}_$sw$k.o"
done
ls "$PKG/abl"/*.so
