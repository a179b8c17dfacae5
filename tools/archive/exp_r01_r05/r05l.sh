#!/bin/bash
# Round 5: A/B of the pool's top-slot reclaim (HSA_POOL_RECLAIM) on configs 3, 4 and 2, alternating builds;
# then main-pass pool depths with the reclaim (HSA_POOL_ENTRIES).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
run() {   # tag config lib pool parity
  HSA_GPU_LIB=$3 HSA_POOL_ENTRIES=$4 timeout -k 10 400 python bench.py --config $2 --steps 3 --warmup 1 --dropin 0 --ref-sample 0 \
      --parity-sample $5 --cpu-sample 0 > gpurun_out/r05l_$1.json 2> gpurun_out/r05l_$1.err || { tail -5 gpurun_out/r05l_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05l_$1.json'));r=d['roofline'];print('$1', d['value'], r.get('k_search_ms'), r.get('traffic'), json.dumps({k:v for k,v in d.items() if k.startswith('parity')})[:160])"
}
for c in 3 4; do
  run c${c}_recl_a $c libhsa_gpu.so 0 2000
  run c${c}_norecl_a $c libhsa_gpu_norecl.so 0 0
  run c${c}_recl_b $c libhsa_gpu.so 0 0
  run c${c}_norecl_b $c libhsa_gpu_norecl.so 0 0
  for p in 8192 4096 2048; do run c${c}_recl_p$p $c libhsa_gpu.so $p 2000; done
done
run c2_recl 2 libhsa_gpu.so 0 2000
run c2_norecl 2 libhsa_gpu_norecl.so 0 0
echo done
