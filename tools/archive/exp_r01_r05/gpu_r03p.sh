# Round 3 closing validation (1 of 2): the whole GPU suite, smoke, the default bench
# (config 2, the driver's run) at 200 steps with every leg
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03p_pytest.log 2>&1 || { tail -40 gpurun_out/r03p_pytest.log; exit 1; }
tail -2 gpurun_out/r03p_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03p_smoke.log 2>&1 || { tail -20 gpurun_out/r03p_smoke.log; exit 2; }
cat gpurun_out/r03p_smoke.log
timeout -k 10 900 python -u bench.py --steps 200 --warmup 5 > gpurun_out/r03p_bench.json 2> gpurun_out/r03p_bench.err \
    || { tail -40 gpurun_out/r03p_bench.err; exit 3; }
grep -v "per-step device ms" gpurun_out/r03p_bench.err | tail -12
