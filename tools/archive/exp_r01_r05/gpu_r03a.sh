# Round 3, first GPU pass: the whole -m gpu suite, then the default bench (config 2)
# with the new reference legs.  Logs under gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03a_pytest.log 2>&1 || { tail -40 gpurun_out/r03a_pytest.log; exit 1; }
tail -3 gpurun_out/r03a_pytest.log
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err \
    || { tail -40 gpurun_out/r03a_bench.err; exit 2; }
tail -12 gpurun_out/r03a_bench.err
head -c 4000 gpurun_out/r03a_bench.json
