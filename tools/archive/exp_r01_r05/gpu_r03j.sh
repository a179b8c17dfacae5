# Round 3: the whole GPU suite with the chunked pool as the default build, then the
# profiling recipe (kernel trace + PMC passes) of configs 2 and 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03j_pytest.log 2>&1 || { tail -40 gpurun_out/r03j_pytest.log; exit 1; }
tail -2 gpurun_out/r03j_pytest.log
bash tools/profile_run.sh r03_c2 || exit 2
BENCH_ARGS="--config 3" PASSES="fetch write sq tcc" bash tools/profile_run.sh r03_c3 || exit 3
echo profiled
