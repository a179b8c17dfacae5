# round 2: 32-bit regression (parity + drop-in), the 64-bit tests, bench config 2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP32" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_match_gap.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_32.log 2>&1 || { tail -30 gpurun_out/pytest_32.log; echo pytest32 failed; exit 1; }
[ -n "$SKIP32" ] || tail -2 gpurun_out/pytest_32.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -v --durations=0 --timeout 300 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1 || { tail -40 gpurun_out/pytest_wide.log; echo pytest_wide failed; exit 2; }
tail -25 gpurun_out/pytest_wide.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --parity-sample 100000 --dropin 0 > gpurun_out/w_c2.json 2> gpurun_out/w_c2.err || { tail gpurun_out/w_c2.err; exit 3; }
grep "kernels\|parity" gpurun_out/w_c2.err
echo ALLOK
