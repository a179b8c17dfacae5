#!/bin/bash
# Round 5: dense-bucket splice kernel -- its tests, the config-4 bench, then 10 M-read parity of config 2.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread tests/test_gpu_splice_device.py \
    tests/test_gpu_dropin.py tests/test_gpu_config4.py > gpurun_out/r05f_pytest.log 2>&1 || { tail -30 gpurun_out/r05f_pytest.log; exit 1; }
grep -E "config 4 at|passed|failed" gpurun_out/r05f_pytest.log
timeout -k 10 900 python -u bench.py --config 4 --steps 3 --warmup 1 --e2e-reads 0 --ref-sample 0 --cpu-sample 0 \
    --parity-sample 0 > gpurun_out/r05f_bench_c4.json 2> gpurun_out/r05f_bench_c4.err || { tail -20 gpurun_out/r05f_bench_c4.err; exit 2; }
grep "per-step kernels" gpurun_out/r05f_bench_c4.err
timeout -k 10 420 python -u tools/parity_10m.py --config 2 --batches 10 --out gpurun_out/r05_parity10m_c2.json \
    > gpurun_out/r05_parity10m_c2.log 2>&1 || { tail -5 gpurun_out/r05_parity10m_c2.log; exit 3; }
tail -1 gpurun_out/r05_parity10m_c2.log | cut -c1-300
