# Round 3: cost-ordered read queue (HSA_ORDER) -- its parity tests, then configs 2, 3, 5
# with and without it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trie.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03n_pytest.log 2>&1 || { tail -40 gpurun_out/r03n_pytest.log; exit 1; }
tail -2 gpurun_out/r03n_pytest.log
B2="python -u bench.py --steps 40 --warmup 3 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 --parity-sample 100000"
B3="python -u bench.py --config 3 --steps 8 --warmup 1 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 --parity-sample 50000"
B5="python -u bench.py --config 5 --steps 10 --warmup 2 --cpu-sample 0 --parity-sample 50000"
for o in 0 1; do
  HSA_ORDER=$o timeout -k 10 300 $B2 > gpurun_out/r03n_c2_o$o.json 2> gpurun_out/r03n_c2_o$o.err || { tail -20 gpurun_out/r03n_c2_o$o.err; exit 2; }
  echo "c2 order $o: $(grep 'per-step kernels\|parity:' gpurun_out/r03n_c2_o$o.err | tr '\n' ' ')"
done
for o in 0 1; do
  HSA_ORDER=$o timeout -k 10 400 $B3 > gpurun_out/r03n_c3_o$o.json 2> gpurun_out/r03n_c3_o$o.err || { tail -20 gpurun_out/r03n_c3_o$o.err; exit 3; }
  echo "c3 order $o: $(grep 'per-step kernels\|parity:' gpurun_out/r03n_c3_o$o.err | tr '\n' ' ')"
done
for o in 0 1; do
  HSA_ORDER=$o timeout -k 10 400 $B5 > gpurun_out/r03n_c5_o$o.json 2> gpurun_out/r03n_c5_o$o.err || { tail -20 gpurun_out/r03n_c5_o$o.err; exit 4; }
  echo "c5 order $o: $(grep 'per-step kernels\|parity:' gpurun_out/r03n_c5_o$o.err | tr '\n' ' ')"
done
