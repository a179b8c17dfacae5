#!/bin/bash
# Round 5: the whole GPU suite on the allocate-before-free build, then the config-4 drop-in end to end.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r05m_gpu_suite.log 2>&1 \
    || { tail -30 gpurun_out/r05m_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r05m_gpu_suite.log
HSA_E2E_LOG=gpurun_out/r05m_e2e_c4.log timeout -k 10 600 python -u bench.py --config 4 --steps 1 --warmup 1 --cpu-sample 0 \
    --parity-sample 0 --e2e-reads 1000000 > gpurun_out/r05m_bench_c4.json 2> gpurun_out/r05m_bench_c4.err || { tail -20 gpurun_out/r05m_bench_c4.err; exit 2; }
grep -E "hipMalloc|batch of" gpurun_out/r05m_e2e_c4.log | cut -c1-160 | head -14
python3 -c "import json;d=json.load(open('gpurun_out/r05m_bench_c4.json'));print(json.dumps(d.get('dropin_e2e'))[:400])"
echo done
