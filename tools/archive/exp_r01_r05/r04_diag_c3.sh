#!/bin/bash
# Round 4: event counters and phase cycles of k_search (diagnostic build) on configs 3 and 2:
# pruned pops, pushes whose pop is pruned, hits, expansions, pool / virtual-top pops.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
for c in ${CONFIGS:-3 2}; do
  HSA_GPU_LIB=libhsa_gpu_diag.so HSA_DIAG_OUT=gpurun_out/r04_diag_c$c.json timeout -k 10 300 python bench.py --config $c \
      --steps 3 --warmup 1 --streams 1 --dropin 0 --ref-sample 0 --parity-sample 0 --cpu-sample 0 \
      > gpurun_out/r04_diag_c$c.out 2> gpurun_out/r04_diag_c$c.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r04_diag_c$c.json'));print('c$c', json.dumps(d['events_total']))"
done
