#!/bin/bash
# Round 5: the splice seeds read their W1 row prefixes (no copy, no export); type-1 prefetch rows from the width trie.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_splice_device.py \
    tests/test_gpu_splice_prefetch.py tests/test_gpu_dropin.py > gpurun_out/r05j_tests.log 2>&1 \
    || { tail -30 gpurun_out/r05j_tests.log; exit 1; }
tail -3 gpurun_out/r05j_tests.log
HSA_E2E_LOG=gpurun_out/r05j_e2e_c4.log timeout -k 10 600 python -u bench.py --config 4 --steps 3 --warmup 1 --e2e-reads 300000 --ref-sample 0 --cpu-sample 0 \
    --parity-sample 1000 > gpurun_out/r05j_bench_c4.json 2> gpurun_out/r05j_bench_c4.err || { tail -20 gpurun_out/r05j_bench_c4.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/r05j_bench_c4.json'));print('c4', d['value'], d['ms_per_step'], json.dumps(d.get('splice_path'))[:400], d.get('parity_reference'), json.dumps(d.get('dropin_e2e'))[:300])"
grep -E "hipMalloc|batch of" gpurun_out/r05j_e2e_c4.log | head -20
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread tests/test_gpu_config4.py \
    > gpurun_out/r05j_config4.log 2>&1 || { tail -30 gpurun_out/r05j_config4.log; exit 3; }
grep "config 4 at" gpurun_out/r05j_config4.log | cut -c1-300
for c in 3 4; do
  HSA_GPU_LIB=libhsa_gpu_diag.so HSA_DIAG_OUT=gpurun_out/r05_diag_c$c.json timeout -k 10 400 python bench.py --config $c \
      --steps 2 --warmup 1 --streams 1 --dropin 0 --e2e-reads 0 --ref-sample 0 --parity-sample 0 --cpu-sample 0 \
      > gpurun_out/r05_diag_c$c.out 2> gpurun_out/r05_diag_c$c.err || { tail -5 gpurun_out/r05_diag_c$c.err; exit 4; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05_diag_c$c.json'));print('c$c', json.dumps(d['events_total']))"
done
echo done
