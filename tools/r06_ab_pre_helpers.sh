#!/bin/bash
# Same-box A/B of config 2 (the metric): the library before the helpers (libhsa_gpu_r06pre.so,
# built from the parent of the helpers commit) against the product, alternating.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--steps 20 --warmup 5 --dropin 0 --ref-sample 1600 --e2e-reads 0 --parity-sample 20000"
for r in a b; do
  for v in pre new; do
    if [ $v = pre ]; then L=libhsa_gpu_r06pre.so; else L=libhsa_gpu.so; fi
    HSA_GPU_LIB=$L timeout -k 10 300 python -u bench.py $B > gpurun_out/abh_${v}_$r.json 2> gpurun_out/abh_${v}_$r.err
    echo "$v $r $(grep -h 'serialized steps' gpurun_out/abh_${v}_$r.err) value $(python -c "import json;print(json.load(open('gpurun_out/abh_${v}_$r.json'))['value'])")"
  done
done
