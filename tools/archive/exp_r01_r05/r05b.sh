#!/bin/bash
# Round 5: kernel trace + PMC passes of the shipped build, configs 2 and 3 (tools/profile_run.sh).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
bash tools/profile_run.sh r05_c2 || exit 1
echo c2 done
BENCH_ARGS="--config 3" PASSES="fetch write sq" bash tools/profile_run.sh r05_c3 || exit 2
echo c3 done
