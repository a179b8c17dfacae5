# round 2: GPU tests + benches of configs 2 and 3 on the current build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; echo pytest failed; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail gpurun_out/bench_c2.err; exit 3; }
grep "kernel split\|parity" gpurun_out/bench_c2.err; cut -c1-400 gpurun_out/bench_c2.json
timeout -k 10 400 python -u bench.py --config 3 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 4; }
grep "kernel split\|parity" gpurun_out/bench_c3.err; cut -c1-400 gpurun_out/bench_c3.json
echo ALLOK
