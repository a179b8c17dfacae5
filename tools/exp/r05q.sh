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
