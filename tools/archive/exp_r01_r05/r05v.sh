#!/bin/bash
# Round 5: the BIG pass's scratch reserved for all its lanes (allocated by the attach-time warm-up):
# search tests, then the config-4 drop-in end to end (first call against the later ones).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_any.py \
    tests/test_gpu_dropin.py tests/test_gpu_config4.py > gpurun_out/r05v_tests.log 2>&1 || { tail -30 gpurun_out/r05v_tests.log; exit 1; }
tail -1 gpurun_out/r05v_tests.log
HSA_E2E_LOG=gpurun_out/r05v_e2e_c4.log timeout -k 10 600 python -u bench.py --config 4 --steps 1 --warmup 1 --cpu-sample 0 \
    --parity-sample 0 --e2e-reads 1000000 > gpurun_out/r05v_bench_c4.json 2> gpurun_out/r05v_bench_c4.err || { tail -20 gpurun_out/r05v_bench_c4.err; exit 2; }
grep -E "hipMalloc|batch of|attached" gpurun_out/r05v_e2e_c4.log | cut -c1-160 > gpurun_out/r05v_e2e_summary.txt; head -8 gpurun_out/r05v_e2e_summary.txt
python3 -c "import json;d=json.load(open('gpurun_out/r05v_bench_c4.json'));print(json.dumps(d.get('dropin_e2e'))[:400])"
echo done
