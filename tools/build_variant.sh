#!/bin/bash
# A/B build of the library with extra -D flags:
#   tools/build_variant.sh NAME "-DHSA_X=0"  ->  hsa_amd/libhsa_gpu_NAME.so (HSA_GPU_LIB=libhsa_gpu_NAME.so).
# The flags apply to the search kernels (hsa_search.hip, hsa_search64.hip); VARIANT_SPLICE=1 applies them
# to the splice kernel (hsa_splice.hip) as well.  Never the product; list the output in .gpurunignore once
# its A/B run is done.
set -e
N=$1; X=$2
D=$(mktemp -d)
S=$(cd "$(dirname "$0")/../hsa_amd/csrc" && pwd)
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result"
make -C $S -s
/opt/rocm/bin/hipcc $F $X -c $S/hsa_search.hip -o $D/s.o &
/opt/rocm/bin/hipcc $F $X -c $S/hsa_search64.hip -o $D/s64.o &
SP=$S/hsa_splice.o
if [ "${VARIANT_SPLICE:-0}" = 1 ]; then /opt/rocm/bin/hipcc $F $X -c $S/hsa_splice.hip -o $D/sp.o & SP=$D/sp.o; fi
wait
/opt/rocm/bin/hipcc $F -shared $D/s.o $D/s64.o $S/hsa_index.o $S/hsa_bwt_build.o $S/hsa_sa.o $S/hsa_extend.o $SP $S/bwtaln_gpu.o $S/bwtgap_gpu.o $S/bwtse_gpu.o $S/bwtsam_gpu.o $S/bwtext_gpu.o -lpthread -lm -o $S/../libhsa_gpu_$N.so
rm -rf $D
echo built hsa_amd/libhsa_gpu_$N.so
