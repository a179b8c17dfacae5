# quick GPU check: parity tests (+ hg19-sized) and benches of configs 2 and 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_hg19.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1 || { tail -30 gpurun_out/pytest_quick.log; echo pytest failed; exit 1; }
tail -2 gpurun_out/pytest_quick.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --parity-sample 20000 ${B2:-} > gpurun_out/q_c2.json 2> gpurun_out/q_c2.err || { tail gpurun_out/q_c2.err; exit 3; }
grep "kernels\|parity" gpurun_out/q_c2.err
timeout -k 10 300 python -u bench.py --config 3 --steps 3 --warmup 1 --cpu-sample 0 --parity-sample 10000 ${B3:-} > gpurun_out/q_c3.json 2> gpurun_out/q_c3.err || { tail gpurun_out/q_c3.err; exit 4; }
grep "kernels\|parity" gpurun_out/q_c3.err
echo ALLOK
