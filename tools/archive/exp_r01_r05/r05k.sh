#!/bin/bash
# Round 5: where the config-4 drop-in's first batch spends its 7 s (HSA_VERBOSE allocation timings).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
HSA_E2E_LOG=gpurun_out/r05k_e2e_c4.log timeout -k 10 600 python -u bench.py --config 4 --steps 1 --warmup 1 --cpu-sample 0 \
    --parity-sample 0 --e2e-reads 300000 > gpurun_out/r05k_bench_c4.json 2> gpurun_out/r05k_bench_c4.err || { tail -20 gpurun_out/r05k_bench_c4.err; exit 2; }
grep -E "hipMalloc|batch of|attached|search scratch" gpurun_out/r05k_e2e_c4.log | cut -c1-250 > gpurun_out/r05k_summary.txt
grep -E "hipMalloc|search scratch" gpurun_out/r05k_bench_c4.err | cut -c1-250 >> gpurun_out/r05k_summary.txt
cat gpurun_out/r05k_summary.txt | cut -c1-200
echo done
