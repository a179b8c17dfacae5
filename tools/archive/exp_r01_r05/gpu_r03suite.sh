# The GPU suite and smoke on the current build (drop-in slots as clones)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/suite_pytest.log 2>&1 || { tail -40 gpurun_out/suite_pytest.log; exit 1; }
tail -2 gpurun_out/suite_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite_smoke.log 2>&1 || { tail -20 gpurun_out/suite_smoke.log; exit 2; }
cat gpurun_out/suite_smoke.log
