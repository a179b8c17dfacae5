#!/bin/bash
# Round-2 closing validation on the GPU box: every GPU test, smoke, bench configs 2/3/4,
# the spliced-read drop-in end to end, and the kernel-trace stats of the default bench.
# usage: [FINAL_DIR=name] tools/gpu_final_r02.sh      outputs under gpurun_out/${FINAL_DIR:-final2}/
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${FINAL_DIR:-final2}
mkdir -p $OUT
export TMPDIR=/tmp
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 2; }
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 3; }
cut -c1-300 $OUT/bench.json
timeout -k 10 300 python -u bench.py --config 3 --steps 3 > $OUT/bench_config3.json 2> $OUT/bench_config3.err || { echo bench3 failed; exit 4; }
timeout -k 10 300 python -u bench.py --config 4 --steps 2 > $OUT/bench_config4.json 2> $OUT/bench_config4.err || { echo bench4 failed; exit 5; }
timeout -k 10 400 python -u tools/splice_e2e.py --genome 50000005 --reads 20000 --out $OUT/splice_e2e.json > $OUT/splice_e2e.log 2>&1 || { echo e2e failed; tail -20 $OUT/splice_e2e.log; exit 6; }
grep "\[e2e\]" $OUT/splice_e2e.log | cut -c1-200
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 --parity-sample 0 --dropin 0 > $OUT/trace.json 2> $OUT/trace.err || { echo rocprof failed; exit 7; }
echo ALLOK
