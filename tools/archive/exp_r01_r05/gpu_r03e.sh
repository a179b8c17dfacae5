# Round 3: the root tries -- trie parity tests, the parity/wide/nib suites, then config 2
# with and without the tries (A/B), config 5 with the tries, and the depth histogram.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_trie.py tests/test_gpu_parity.py tests/test_gpu_nib.py -x -v \
    --timeout 300 --timeout-method thread > gpurun_out/r03e_pytest.log 2>&1 || { tail -40 gpurun_out/r03e_pytest.log; exit 1; }
tail -2 gpurun_out/r03e_pytest.log
timeout -k 10 600 python -u bench.py --steps 50 --warmup 3 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 \
    > gpurun_out/r03e_bench_trie.json 2> gpurun_out/r03e_bench_trie.err || { tail -30 gpurun_out/r03e_bench_trie.err; exit 2; }
grep "per-step kernels\|parity" gpurun_out/r03e_bench_trie.err
HSA_TRIE=0 timeout -k 10 600 python -u bench.py --steps 50 --warmup 3 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 \
    --parity-sample 0 > gpurun_out/r03e_bench_notrie.json 2> gpurun_out/r03e_bench_notrie.err || { tail -30 gpurun_out/r03e_bench_notrie.err; exit 3; }
grep "per-step kernels" gpurun_out/r03e_bench_notrie.err
timeout -k 10 300 python -u tools/exp/depth_hist.py --out gpurun_out/r03e_depth_hist.json > gpurun_out/r03e_depth_hist.log 2>&1 \
    || { tail -20 gpurun_out/r03e_depth_hist.log; exit 4; }
grep -v "^\[bench\]" gpurun_out/r03e_depth_hist.log
