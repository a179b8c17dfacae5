# Round 3: width trie at depth 12 by default -- the whole GPU suite, config 2 (the driver's
# default run at 200 steps), config 5 with the 64-bit width trie
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03h_pytest.log 2>&1 || { tail -40 gpurun_out/r03h_pytest.log; exit 1; }
tail -2 gpurun_out/r03h_pytest.log
timeout -k 10 900 python -u bench.py --steps 200 --warmup 5 > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err \
    || { tail -40 gpurun_out/r03h_bench.err; exit 2; }
tail -12 gpurun_out/r03h_bench.err
timeout -k 10 900 python -u bench.py --config 5 --steps 20 --warmup 2 --cpu-sample 0 --parity-sample 0 \
    > gpurun_out/r03h_bench_c5.json 2> gpurun_out/r03h_bench_c5.err || { tail -40 gpurun_out/r03h_bench_c5.err; exit 3; }
grep "per-step kernels\|index ready" gpurun_out/r03h_bench_c5.err
