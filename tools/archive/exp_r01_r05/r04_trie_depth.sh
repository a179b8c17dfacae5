#!/bin/bash
# Round 4: k_widths / k_search and the step with width tries of 12..15 levels (config 2).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
for d in ${DEPTHS:-12 13 14 15}; do
  HSA_TRIE_DEPTH=$d timeout -k 10 300 python bench.py --steps 20 --warmup 2 --dropin 0 --ref-sample 0 \
      --parity-sample 0 --cpu-sample 0 > gpurun_out/r04_trie_d$d.json 2> gpurun_out/r04_trie_d$d.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r04_trie_d$d.json'));r=d['roofline'];print('D=$d', d['value'], r['k_widths']['ms'], r['k_search_ms'], r['tries'])"
done
