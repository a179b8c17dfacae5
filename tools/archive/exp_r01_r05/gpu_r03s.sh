# Round 3: the drop-in's outputs written on 8 host threads -- the drop-in SAM tests, then
# the end-to-end leg with its stage timings
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_match_gap.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03s_pytest.log 2>&1 || { tail -40 gpurun_out/r03s_pytest.log; exit 1; }
tail -2 gpurun_out/r03s_pytest.log
HSA_E2E_LOG=gpurun_out/r03s_e2e.log timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --parity-sample 0 \
    --ref-sample 16000 > gpurun_out/r03s_bench.json 2> gpurun_out/r03s_bench.err || { tail -30 gpurun_out/r03s_bench.err; exit 2; }
grep "drop-in end to end" gpurun_out/r03s_bench.err
grep -E "batch of" gpurun_out/r03s_e2e.log | head -12
