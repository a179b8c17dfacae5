#!/bin/bash
# Profiling recipe run on the GPU box (see DESIGN.md "Measurement").
# usage: tools/profile_run.sh <tag>
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="$R/bench.py --steps 5 --warmup 1 --cpu-sample 0 --parity-sample 0"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.json 2> $OUT/trace.err || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex k_search --output-format csv -d $OUT/pmc_fetch -o run -- python3 $BENCH > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex k_search --output-format csv -d $OUT/pmc_write -o run -- python3 $BENCH > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-include-regex k_search --output-format csv -d $OUT/pmc_sq -o run -- python3 $BENCH > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_search --output-format csv -d $OUT/pmc_tcc -o run -- python3 $BENCH > $OUT/pmc_tcc.json 2> $OUT/pmc_tcc.err || exit 15
echo done
