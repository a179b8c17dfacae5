#!/bin/bash
# Round 5: splice tests on the in-place build, config-4 splice timing, config 3 and 5 benches,
# then >= 8 M config-3 reads of parity at hg19 size.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_splice_device.py \
    tests/test_gpu_dropin.py > gpurun_out/r05g_pytest.log 2>&1 || { tail -30 gpurun_out/r05g_pytest.log; exit 1; }
tail -1 gpurun_out/r05g_pytest.log
timeout -k 10 600 python -u bench.py --config 4 --steps 3 --warmup 1 --e2e-reads 0 --ref-sample 0 --cpu-sample 0 \
    --parity-sample 0 > gpurun_out/r05g_bench_c4.json 2> gpurun_out/r05g_bench_c4.err || { tail -20 gpurun_out/r05g_bench_c4.err; exit 2; }
grep "per-step kernels" gpurun_out/r05g_bench_c4.err
timeout -k 10 900 python -u bench.py --config 3 --steps 10 --warmup 2 > gpurun_out/r05g_bench_c3.json 2> gpurun_out/r05g_bench_c3.err || { tail -20 gpurun_out/r05g_bench_c3.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/r05g_bench_c3.json'));print('c3', d['value'], d['roofline']['k_search_ms'], d.get('parity_full'), d.get('dropin_e2e',{}).get('value'))"
timeout -k 10 900 python -u bench.py --config 5 --steps 10 --warmup 2 > gpurun_out/r05g_bench_c5.json 2> gpurun_out/r05g_bench_c5.err || { tail -20 gpurun_out/r05g_bench_c5.err; exit 4; }
python3 -c "import json;d=json.load(open('gpurun_out/r05g_bench_c5.json'));print('c5', d['value'], d['roofline']['k_search_ms'], d.get('parity_full'))"
