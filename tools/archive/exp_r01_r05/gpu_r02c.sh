# round 2: GPU tests (incl. hg19-sized parity), bench config 2 (full parity) and 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; echo pytest failed; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { tail gpurun_out/bench_c2.err; exit 3; }
grep "kernels\|parity" gpurun_out/bench_c2.err
timeout -k 10 400 python -u bench.py --config 3 --steps 3 --warmup 1 --cpu-sample 0 --parity-sample 20000 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail gpurun_out/bench_c3.err; exit 4; }
grep "kernels\|parity" gpurun_out/bench_c3.err
echo ALLOK
