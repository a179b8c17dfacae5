#!/bin/bash
# Round 4: the select-tree pick4 and branch-free candidate masks (default build) against
# the round-4 base (libhsa_gpu_r04base.so: tools/build_variant.sh r04base "" built from the previous commit),
# configs 2 and 3, alternating so drift hits both.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
for c in ${CONFIGS:-2 3}; do
  for rep in 1 2; do
    for lib in libhsa_gpu.so libhsa_gpu_r04base.so; do
      t=r04_pick_c${c}_${lib%.so}_$rep
      HSA_GPU_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-20} --warmup 2 --dropin 0 \
          --ref-sample 0 --parity-sample 0 --cpu-sample 0 > gpurun_out/$t.json 2> gpurun_out/$t.err || exit 1
      python3 -c "import json;d=json.load(open('gpurun_out/$t.json'));r=d['roofline'];print('$t', d['value'], r['k_widths']['ms'], r['k_search_ms'])"
    done
  done
done
