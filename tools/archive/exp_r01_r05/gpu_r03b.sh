# Round 3: the threaded splice runner -- drop-in SAM tests, spliced end to end (1 vs 16
# host threads), then the default bench (its drop-in end-to-end leg)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_match_gap.py tests/test_gpu_extend.py -x -v \
    --timeout 300 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1 || { tail -40 gpurun_out/r03b_pytest.log; exit 1; }
tail -2 gpurun_out/r03b_pytest.log
HSA_SPLICE_THREADS=1 timeout -k 10 600 python -u tools/splice_e2e.py --reads 20000 --bins HSA HSA_gpu_all \
    --out gpurun_out/r03b_e2e_t1.json --stderr-dir gpurun_out > gpurun_out/r03b_e2e_t1.log 2>&1 || { tail -20 gpurun_out/r03b_e2e_t1.log; exit 2; }
mv gpurun_out/HSA_gpu_all.err gpurun_out/r03b_e2e_t1_HSA_gpu_all.err
timeout -k 10 600 python -u tools/splice_e2e.py --reads 20000 --bins HSA_gpu_all HSA_gpu_mg \
    --out gpurun_out/r03b_e2e_t16.json --stderr-dir gpurun_out > gpurun_out/r03b_e2e_t16.log 2>&1 || { tail -20 gpurun_out/r03b_e2e_t16.log; exit 3; }
grep "\[e2e\]" gpurun_out/r03b_e2e_t1.log gpurun_out/r03b_e2e_t16.log
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err \
    || { tail -40 gpurun_out/r03b_bench.err; exit 4; }
tail -5 gpurun_out/r03b_bench.err
