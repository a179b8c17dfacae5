#!/bin/bash
# Round 5 (final tree): kernel trace + PMC passes of config 3 with the 16 384-entry gapped pools.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
BENCH_ARGS="--config 3" PASSES="fetch write sq" bash tools/profile_run.sh r05g_c3 || exit 1
echo c3 done
