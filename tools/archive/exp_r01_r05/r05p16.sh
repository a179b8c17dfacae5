#!/bin/bash
# Round 5: config 3's main-pass pool at 16 384 entries per lane (half the scratch) on two and three handles.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # tag streams pool
  HSA_POOL_ENTRIES=$3 timeout -k 10 400 python bench.py --config 3 --streams $2 --steps 6 --warmup 2 --dropin 0 --ref-sample 0 \
      --parity-sample 0 --cpu-sample 0 --copies 0 > gpurun_out/r05p16_$1.json 2> gpurun_out/r05p16_$1.err || { tail -3 gpurun_out/r05p16_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05p16_$1.json'));r=d['roofline'];print('$1', d['value'], d['ms_per_step'], r.get('k_search_ms'), d['config']['streams'])"
}
run s2_p32k 2 0
run s2_p16k 2 16384
run s3_p16k 3 16384
run s2_p32k_b 2 0
run s3_p16k_b 3 16384
echo done
