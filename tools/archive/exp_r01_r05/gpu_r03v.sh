# Round 3: lazy forward rows in one launch (HSA_LAZY=2, a lane per read: rc row, then its
# forward row when needed) against two launches (1) and none (0): parity tests, configs 2, 5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k lazy -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03v_pytest.log 2>&1 || { tail -60 gpurun_out/r03v_pytest.log; exit 1; }
tail -2 gpurun_out/r03v_pytest.log
B2="python -u bench.py --steps 40 --warmup 3 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 --parity-sample 100000"
B5="python -u bench.py --config 5 --steps 10 --warmup 2 --cpu-sample 0 --parity-sample 50000"
for l in 0 1 2; do
  HSA_LAZY=$l timeout -k 10 300 $B2 > gpurun_out/r03v_c2_l$l.json 2> gpurun_out/r03v_c2_l$l.err || { tail -20 gpurun_out/r03v_c2_l$l.err; exit 2; }
  echo "c2 lazy $l: $(grep 'per-step kernels\|parity:' gpurun_out/r03v_c2_l$l.err | tr '\n' ' ')"
done
for l in 1 2; do
  HSA_LAZY=$l timeout -k 10 400 $B5 > gpurun_out/r03v_c5_l$l.json 2> gpurun_out/r03v_c5_l$l.err || { tail -20 gpurun_out/r03v_c5_l$l.err; exit 4; }
  echo "c5 lazy $l: $(grep 'per-step kernels\|parity:' gpurun_out/r03v_c5_l$l.err | tr '\n' ' ')"
done
