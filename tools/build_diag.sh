#!/bin/bash
# Diagnostic build of the library (in-kernel clock stamps + event counters, -DHSA_DIAG):
# hsa_amd/libhsa_gpu_diag.so, selected with HSA_GPU_LIB=libhsa_gpu_diag.so.  Never the product.
set -e
D=$(mktemp -d)
S=$(cd "$(dirname "$0")/../hsa_amd/csrc" && pwd)
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result"
make -C $S -s
/opt/rocm/bin/hipcc $F -DHSA_DIAG -c $S/hsa_search.hip -o $D/s.o
/opt/rocm/bin/hipcc $F -DHSA_DIAG -c $S/hsa_search64.hip -o $D/s64.o
/opt/rocm/bin/hipcc $F -shared $D/s.o $D/s64.o $S/hsa_index.o $S/hsa_bwt_build.o $S/hsa_sa.o $S/hsa_extend.o $S/hsa_splice.o $S/bwtaln_gpu.o $S/bwtgap_gpu.o $S/bwtse_gpu.o $S/bwtsam_gpu.o $S/bwtext_gpu.o -lpthread -lm -o $S/../libhsa_gpu_diag.so
rm -rf $D
