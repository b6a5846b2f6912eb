#!/bin/bash
# A/B builds of libgcow.so: compile the listed sources with extra defines, link them with the in-tree objects of the
# other sources, into abv/libgcow_NAME.so (git-ignored; travels to the GPU box). Time them with
# tools/bench_configs.py --lib abv/libgcow_NAME.so (or tools/prof_cases.py --lib ...).
# usage: tools/build_variant.sh NAME "DEFS" src.hip [src.hip ...]
set -e
NAME=$1; DEFS=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/gcow_amd/csrc
OBJ=/tmp/gcow_variant_$NAME
mkdir -p $OBJ $ROOT/abv
make -s -C $CS >/dev/null
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Werror=pass-failed -I$ROOT/include -I$CS"
objs=""
for f in gcow_kernels gcow_blocks var1d gcow_api; do
  src=$CS/$f.hip; [ -f $src ] || src=$CS/$f.cpp
  if printf '%s\n' "$@" | grep -qx "$(basename $src)"; then
    /opt/rocm/bin/hipcc $FLAGS $DEFS -c $src -o $OBJ/$f.o &
    objs="$objs $OBJ/$f.o"
  else
    objs="$objs $CS/build/$f.o"
  fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/abv/libgcow_$NAME.so $objs
echo "abv/libgcow_$NAME.so"
