#!/bin/bash
# Round 5: config 2 on three handles against two (consecutive steps alternate over the handles).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
for S in 2 3 2 3; do
  timeout -k 10 300 python bench.py --streams $S --steps 20 --warmup 3 --dropin 0 --ref-sample 0 --parity-sample 0 --cpu-sample 0 \
      --copies 0 > gpurun_out/r05s3_$S.json 2> gpurun_out/r05s3_$S.err || { tail -3 gpurun_out/r05s3_$S.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05s3_$S.json'));print('streams', d['config']['streams'], d['value'], d['ms_per_step'])"
done
echo done
