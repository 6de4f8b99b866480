#!/bin/bash
# Build tuning variants of libcbg: only cbg_local.hip is recompiled with the
# given -D overrides; the result goes to build/variants/<name>/libcbg.so and is
# selected at run time with CBG_LIB=<path>.
#   tools/variants.sh p16c4096 "-DCBG_PANEL_LOG_MAX=16 -DCBG_SLAB_CAP=4096 -DCBG_FINE_LOG=12 -DCBG_SLAB_LARGE_BS=512"
set -e
cd "$(dirname "$0")/../combblas-spmm-test_amd"
make -s libcbg.so
name=$1; shift
out=../build/variants/$name
mkdir -p $out
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../include -Wall -Wno-unused-function -Wno-unused-variable"
/opt/rocm/bin/hipcc $FLAGS $* -c ${SRC:-csrc/cbg_local.hip} -o $out/cbg_local.o
objs=$(ls build/*.o | grep -v cbg_local.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/libcbg.so $out/cbg_local.o $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo $out/libcbg.so
