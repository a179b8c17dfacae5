#!/bin/bash
# Round 5: config 4 at hg19 size through the drop-in vs the reference; config-4 and
# config-2 benches with their end-to-end legs on the device splice path.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_config4.py \
    > gpurun_out/r05d_c4test.log 2>&1 || { tail -30 gpurun_out/r05d_c4test.log; exit 1; }
grep -E "config 4 at|passed|failed" gpurun_out/r05d_c4test.log
HSA_E2E_LOG=gpurun_out/r05d_e2e_c4.log timeout -k 10 900 python -u bench.py --config 4 --steps 3 --warmup 1 \
    > gpurun_out/r05d_bench_c4.json 2> gpurun_out/r05d_bench_c4.err || { tail -20 gpurun_out/r05d_bench_c4.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/r05d_bench_c4.json'));e=d.get('dropin_e2e');print('c4', d['value'], json.dumps(e)[:700])"
