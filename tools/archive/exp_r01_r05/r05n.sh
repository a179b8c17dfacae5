#!/bin/bash
# Round 5: the lean push loop (group heads in registers) -- parity tests, A/B against the previous loop
# (libhsa_gpu_oldpush.so), and the config-4 drop-in end to end with the attach-time splice warm-up.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_any.py \
    tests/test_gpu_match_gap.py tests/test_gpu_splice_device.py > gpurun_out/r05n_tests.log 2>&1 || { tail -30 gpurun_out/r05n_tests.log; exit 1; }
tail -2 gpurun_out/r05n_tests.log
run() {   # tag config lib parity
  HSA_GPU_LIB=$3 timeout -k 10 400 python bench.py --config $2 --steps 3 --warmup 1 --dropin 0 --ref-sample 0 \
      --parity-sample $4 --cpu-sample 0 > gpurun_out/r05n_$1.json 2> gpurun_out/r05n_$1.err || { tail -5 gpurun_out/r05n_$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05n_$1.json'));r=d['roofline'];print('$1', d['value'], r.get('k_search_ms'), json.dumps({k:v for k,v in d.items() if k.startswith('parity')})[:160])"
}
run c3_new_a 3 libhsa_gpu.so 100000
run c3_old_a 3 libhsa_gpu_oldpush.so 0
run c3_new_b 3 libhsa_gpu.so 0
run c3_old_b 3 libhsa_gpu_oldpush.so 0
run c4_new_a 4 libhsa_gpu.so 2000
run c4_old_a 4 libhsa_gpu_oldpush.so 0
run c2_new_a 2 libhsa_gpu.so 100000
run c2_old_a 2 libhsa_gpu_oldpush.so 0
HSA_E2E_LOG=gpurun_out/r05n_e2e_c4.log timeout -k 10 600 python -u bench.py --config 4 --steps 1 --warmup 1 --cpu-sample 0 \
    --parity-sample 0 --e2e-reads 1000000 > gpurun_out/r05n_bench_c4.json 2> gpurun_out/r05n_bench_c4.err || { tail -20 gpurun_out/r05n_bench_c4.err; exit 2; }
grep -E "hipMalloc|batch of|warm-up" gpurun_out/r05n_e2e_c4.log | cut -c1-160 | head -8
python3 -c "import json;d=json.load(open('gpurun_out/r05n_bench_c4.json'));print(json.dumps(d.get('dropin_e2e'))[:300])"
echo done
