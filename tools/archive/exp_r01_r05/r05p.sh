#!/bin/bash
# Round 5: 4-bit pruning rows for the gapped regimes (HSA_WFMT=nib: more waves per CU) against the
# 8-bit default, on the shipped build (more than 11 waves per CU for 39 buckets).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # tag config wfmt parity
  HSA_WFMT=$3 HSA_VERBOSE=1 timeout -k 10 400 python bench.py --config $2 --steps 3 --warmup 1 --dropin 0 --ref-sample 0 \
      --parity-sample $4 --cpu-sample 0 > gpurun_out/r05p_$1.json 2> gpurun_out/r05p_$1.err || { tail -5 gpurun_out/r05p_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05p_$1.json'));r=d['roofline'];print('$1', d['value'], r.get('k_search_ms'), json.dumps({k:v for k,v in d.items() if k.startswith('parity')})[:120])"
  grep -m1 "workgroups of" gpurun_out/r05p_$1.err | cut -c1-160
}
run c3_byte_a 3 byte 0
run c3_nib_a 3 nib 20000
run c3_byte_b 3 byte 0
run c3_nib_b 3 nib 0
run c4_byte_a 4 byte 0
run c4_nib_a 4 nib 2000
echo done
