#!/bin/bash
# Round 5 (final build): kernel trace + PMC passes of configs 2, 3, 4 and 5 (tools/profile_run.sh).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
bash tools/profile_run.sh r05f_c2 || exit 1
echo c2 done
BENCH_ARGS="--config 3" PASSES="fetch write sq" bash tools/profile_run.sh r05f_c3 || exit 2
echo c3 done
BENCH_ARGS="--config 4 --streams 1" PASSES="fetch write" PMC_REGEX="k_search|k_widths|k_splice|k_pf_|k_sp_prep" \
    bash tools/profile_run.sh r05f_c4 || exit 3
echo c4 done
BENCH_ARGS="--config 5" PASSES="fetch write sq" bash tools/profile_run.sh r05f_c5 || exit 4
echo c5 done
HSA_E2E_LOG=gpurun_out/r05q_e2e_c2.log timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 --parity-sample 0 \
    --dropin 0 > gpurun_out/r05q_bench_c2_e2e.json 2> gpurun_out/r05q_bench_c2_e2e.err || exit 5
grep -E "splice prefetch on|splice kernel:|batch of" gpurun_out/r05q_e2e_c2.log > gpurun_out/r05q_e2e_c2_stages.txt; head -6 gpurun_out/r05q_e2e_c2_stages.txt | cut -c1-220
echo done
