#!/bin/bash
# Round 5: config 4 on two handles (step s's splice path beside step s+1's main search) against one.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
for S in 2 1 2; do
  HSA_VERBOSE=1 timeout -k 10 500 python bench.py --config 4 --streams $S --steps 4 --warmup 2 --dropin 0 --ref-sample 0 \
      --parity-sample 1000 --cpu-sample 0 > gpurun_out/r05w_s$S.json 2> gpurun_out/r05w_s$S.err || { grep -E "hipMalloc|scratch|handle|Error|error" gpurun_out/r05w_s$S.err | tail -8; tail -3 gpurun_out/r05w_s$S.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05w_s$S.json'));r=d['roofline'];print('streams $S', d['value'], d['ms_per_step'], r.get('k_search_ms'), r.get('splice_path_ms'), d['config'].get('streams'), json.dumps(d.get('parity_sample'))[:90])"
  grep -E "hipMalloc|dropped" gpurun_out/r05w_s$S.err | cut -c1-160 | tail -4
done
echo done
