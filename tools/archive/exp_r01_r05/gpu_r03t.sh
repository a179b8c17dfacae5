# Round 3: the unique-interval walk -- its parity tests (arrays derived from the
# reference's .sa), the parity suite, the drop-in SAM tests (attach builds the arrays),
# then config 2 with and without it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03t_pytest_walk.log 2>&1 || { tail -60 gpurun_out/r03t_pytest_walk.log; exit 1; }
tail -2 gpurun_out/r03t_pytest_walk.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_match_gap.py tests/test_gpu_sa.py \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/r03t_pytest.log 2>&1 || { tail -40 gpurun_out/r03t_pytest.log; exit 2; }
tail -2 gpurun_out/r03t_pytest.log
B2="python -u bench.py --steps 40 --warmup 3 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 --parity-sample 200000"
for w in 0 1; do
  HSA_WALK=$w timeout -k 10 300 $B2 > gpurun_out/r03t_c2_w$w.json 2> gpurun_out/r03t_c2_w$w.err || { tail -20 gpurun_out/r03t_c2_w$w.err; exit 3; }
  echo "c2 walk $w: $(grep 'per-step kernels\|parity:\|walk arrays' gpurun_out/r03t_c2_w$w.err | tr '\n' ' ')"
done
