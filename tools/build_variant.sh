#!/bin/bash
# Build an alternative in-tree variant of the library for A/B runs:
#   tools/build_variant.sh <name> <extra hipcc flags for hsa_search.hip...>
# -> hsa_amd/libhsa_gpu_<name>.so (select with HSA_GPU_LIB=libhsa_gpu_<name>.so)
set -e
N=$1; shift
D=$(mktemp -d)
S=$(cd "$(dirname "$0")/../hsa_amd/csrc" && pwd)
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result"
make -C $S -s
/opt/rocm/bin/hipcc $F "$@" -c $S/hsa_search.hip -o $D/s.o
/opt/rocm/bin/hipcc $F -shared $D/s.o $S/hsa_index.o $S/hsa_bwt_build.o $S/hsa_sa.o $S/bwtaln_gpu.o $S/bwtgap_gpu.o -lpthread -lm -o $S/../libhsa_gpu_$N.so
rm -rf $D
