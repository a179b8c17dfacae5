#!/bin/bash
# Round 4: kernel time of one 100 000-read drop-in call (config 2) -- the product, the
# unique-interval walk build and the search-trie build.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python tools/dropin_time.py --reads 100000 > gpurun_out/r04_sb_$tag.log 2>&1
  echo "$tag $? $(grep -h 'call 3' gpurun_out/r04_sb_$tag.log)"
}
run prod HSA_VERBOSE=1 || exit 1
run walk HSA_GPU_LIB=libhsa_gpu_walk.so HSA_WALK=1 HSA_VERBOSE=1 || exit 1
run walk_s0m4 HSA_GPU_LIB=libhsa_gpu_walk.so HSA_WALK=1 HSA_WALK_STREAK=0 HSA_WALK_MIN=4 HSA_VERBOSE=1 || exit 1
run strie HSA_GPU_LIB=libhsa_gpu_strie.so HSA_TRIE_MODE=1 HSA_VERBOSE=1 || exit 1
