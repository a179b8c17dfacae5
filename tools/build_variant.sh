#!/bin/bash
# An experiment build of the library with extra -D flags for the search sources:
# hsa_amd/libhsa_gpu_<name>.so, selected with HSA_GPU_LIB=libhsa_gpu_<name>.so for A/B
# runs.  Never the product.   usage: tools/build_variant.sh <name> "<-DFLAGS ...>"
set -e
N=$1; X=$2
D=$(mktemp -d)
S=$(cd "$(dirname "$0")/../hsa_amd/csrc" && pwd)
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result"
make -C $S -s
/opt/rocm/bin/hipcc $F $X -c $S/hsa_search.hip -o $D/s.o &
/opt/rocm/bin/hipcc $F $X -c $S/hsa_search64.hip -o $D/s64.o &
wait
/opt/rocm/bin/hipcc $F -shared $D/s.o $D/s64.o $S/hsa_index.o $S/hsa_bwt_build.o $S/hsa_sa.o $S/hsa_extend.o $S/bwtaln_gpu.o $S/bwtgap_gpu.o $S/bwtse_gpu.o $S/bwtext_gpu.o -lpthread -lm -o $S/../libhsa_gpu_$N.so
rm -rf $D
echo built hsa_amd/libhsa_gpu_$N.so
