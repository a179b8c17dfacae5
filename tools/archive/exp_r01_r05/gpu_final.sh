#!/bin/bash
# Round-end validation on the GPU box: gpu tests, bench configs 2/3/4, kernel-trace stats.
# usage: tools/gpu_final.sh        outputs under gpurun_out/final/
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/final
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo pytest failed; exit 1; }
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
timeout -k 10 300 python -u bench.py --config 3 --steps 3 > $OUT/bench_config3.json 2> $OUT/bench_config3.err || exit 4
timeout -k 10 300 python -u bench.py --config 4 --steps 2 > $OUT/bench_config4.json 2> $OUT/bench_config4.err || exit 5
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 --parity-sample 0 > $OUT/trace.json 2> $OUT/trace.err || exit 6
echo ALLOK
