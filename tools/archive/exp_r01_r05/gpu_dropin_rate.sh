# the drop-in (host arrays) rate of configs 2 and 3, plus the flat-API GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dropin
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dropin/pytest.log 2>&1 || { echo pytest failed; tail -20 gpurun_out/dropin/pytest.log; exit 1; }
tail -1 gpurun_out/dropin/pytest.log
timeout -k 10 300 python -u bench.py --steps 3 --cpu-sample 0 --parity-sample 0 > gpurun_out/dropin/bench2.json 2> gpurun_out/dropin/bench2.err || { echo bench failed; tail -5 gpurun_out/dropin/bench2.err; exit 2; }
grep "drop-in" gpurun_out/dropin/bench2.err
echo ALLOK
