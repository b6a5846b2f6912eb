#!/bin/bash
# Ablation builds of the single-pass variable-rate encoder (gcow_amd/csrc/var1d.hip, V1_ABLATE bits) as whole
# libgcow.so variants in ab/ (V1_ABLATE builds time only: their streams are wrong by construction).
# usage: var1d_ablate.sh NAME=-DFLAG[,-DFLAG..] ...
set -e
cd "$(dirname "$0")/../.."
make -s -C gcow_amd/csrc
OUT=${ABL_DIR:-ab}; mkdir -p $OUT
B=gcow_amd/csrc/build
for a in "$@"; do  # NAME=-DFLAGS,... e.g. 8=-DV1_ABLATE=8 or poll1=-DV1_POLL=1
  name=${a%%=*}; flags=${a#*=}; flags=${flags//,/ }
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Igcow_amd/csrc $flags \
    -c gcow_amd/csrc/var1d.hip -o $OUT/var1d_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/v1ab_$name.so $B/gcow_kernels.o $B/gcow_blocks.o $OUT/var1d_$name.o $B/gcow_api.o
done
