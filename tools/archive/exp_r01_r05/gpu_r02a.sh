# round 2, first call: GPU tests, gather-shape probe, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; echo pytest failed; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 ./tools/gather_probe > gpurun_out/gather_probe.log 2>&1 || { echo probe failed; exit 2; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; exit 3; }
cat gpurun_out/bench.json
echo ALLOK
