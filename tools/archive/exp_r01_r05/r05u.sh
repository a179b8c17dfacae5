#!/bin/bash
# Round 5: the latest pool push kept in registers until evicted or popped (cq) -- parity tests, then an A/B
# against the build without it (libhsa_gpu_nocq.so) on configs 3, 4, 2 and 5.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_any.py \
    tests/test_gpu_match_gap.py tests/test_gpu_wide.py tests/test_gpu_nib.py > gpurun_out/r05u_tests.log 2>&1 || { tail -30 gpurun_out/r05u_tests.log; exit 1; }
tail -1 gpurun_out/r05u_tests.log
run() {   # tag config lib parity
  HSA_GPU_LIB=$3 timeout -k 10 400 python bench.py --config $2 --steps 3 --warmup 1 --dropin 0 --ref-sample 0 \
      --parity-sample $4 --cpu-sample 0 > gpurun_out/r05u_$1.json 2> gpurun_out/r05u_$1.err || { tail -5 gpurun_out/r05u_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05u_$1.json'));r=d['roofline'];print('$1', d['value'], r.get('k_search_ms'), json.dumps({k:v for k,v in d.items() if k.startswith('parity')})[:120])"
}
run c3_cq_a 3 libhsa_gpu.so 100000
run c3_nocq_a 3 libhsa_gpu_nocq.so 0
run c3_cq_b 3 libhsa_gpu.so 0
run c3_nocq_b 3 libhsa_gpu_nocq.so 0
run c4_cq_a 4 libhsa_gpu.so 2000
run c4_nocq_a 4 libhsa_gpu_nocq.so 0
run c2_cq_a 2 libhsa_gpu.so 100000
run c2_nocq_a 2 libhsa_gpu_nocq.so 0
run c2_cq_b 2 libhsa_gpu.so 0
run c2_nocq_b 2 libhsa_gpu_nocq.so 0
run c5_cq_a 5 libhsa_gpu.so 20000
run c5_nocq_a 5 libhsa_gpu_nocq.so 0
echo done
