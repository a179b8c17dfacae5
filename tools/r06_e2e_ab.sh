#!/bin/bash
# Round-6 A/B of the drop-in end-to-end leg (the reference's driver with our entry points,
# 100 000-read calls): the default small splice warm-up at attach vs none (config 2), and
# the strand-split main pass forced on (HSA_SPLIT=1) vs the default (configs 3 and 4), and
# the strand-split pass's helpers (HSA_HELP) off vs on (configs 2-4).
# Run on the GPU box from the repo root: bash tools/r06_e2e_ab.sh <set>
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--steps 2 --warmup 1 --dropin 0 --ref-sample 1600 --parity-sample 4000"
run() {   # name, env..., -- bench args
    local name=$1; shift
    env "$@" HSA_E2E_LOG=gpurun_out/e2e_$name.log timeout -k 10 500 python -u bench.py $B $EXTRA \
        > gpurun_out/e2e_$name.json 2> gpurun_out/e2e_$name.err
    grep "end to end" gpurun_out/e2e_$name.err
}
case "$1" in
warm) EXTRA="--config 2"
      run c2_warm0 HSA_SPLICE_WARM=0
      run c2_warmsmall HSA_SPLICE_WARM=64 ;;
warm4k) EXTRA="--config 2"
      run c2_warm4096 HSA_SPLICE_WARM_DEFAULT=1 ;;
c4)   EXTRA="--config 4"
      run c4_split_default HSA_SPLIT_UNSET=1
      run c4_split1 HSA_SPLIT=1 ;;
c3)   EXTRA="--config 3"
      run c3_split_default HSA_SPLIT_UNSET=1
      run c3_split1 HSA_SPLIT=1 ;;
help4) EXTRA="--config 4"
      run c4_help0 HSA_HELP=0
      run c4_help1 HSA_HELP=1 ;;
help3) EXTRA="--config 3"
      run c3_help0 HSA_HELP=0
      run c3_help1 HSA_HELP=1 ;;
help2) EXTRA="--config 2"
      run c2_help0 HSA_HELP=0
      run c2_help1 HSA_HELP=1 ;;
esac
