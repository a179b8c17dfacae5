#!/bin/bash
# Round 5: kernel trace + PMC passes of configs 4 (main path + the splice path) and 5.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
BENCH_ARGS="--config 4 --streams 1" PASSES="fetch write membench" PMC_REGEX="k_search|k_widths|k_splice|k_pf_|k_sp_prep" \
    bash tools/profile_run.sh r05_c4 || exit 1
echo c4 done
BENCH_ARGS="--config 5" PASSES="fetch write sq membench" bash tools/profile_run.sh r05_c5 || exit 2
echo c5 done
