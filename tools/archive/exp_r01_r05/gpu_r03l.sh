# Round 3: the pool-head register (pt) against the build without it (libhsa_gpu_nopt.so),
# configs 2 and 3, parity samples on both; then the pt build's GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libhsa_gpu_nopt.so libhsa_gpu.so; do
  HSA_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --cpu-sample 0 --ref-sample 0 \
      --dropin 0 --e2e-reads 0 --parity-sample 100000 > gpurun_out/r03l_c2_$lib.json 2> gpurun_out/r03l_c2_$lib.err \
      || { tail -20 gpurun_out/r03l_c2_$lib.err; exit 3; }
  echo "c2 $lib: $(grep 'per-step kernels\|parity:' gpurun_out/r03l_c2_$lib.err | tr '\n' ' ')"
  HSA_GPU_LIB=$lib timeout -k 10 400 python -u bench.py --config 3 --steps 8 --warmup 1 --cpu-sample 0 --ref-sample 0 \
      --dropin 0 --e2e-reads 0 --parity-sample 100000 > gpurun_out/r03l_c3_$lib.json 2> gpurun_out/r03l_c3_$lib.err \
      || { tail -20 gpurun_out/r03l_c3_$lib.err; exit 2; }
  echo "c3 $lib: $(grep 'per-step kernels\|parity:' gpurun_out/r03l_c3_$lib.err | tr '\n' ' ')"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03l_pytest.log 2>&1 || { tail -40 gpurun_out/r03l_pytest.log; exit 1; }
tail -2 gpurun_out/r03l_pytest.log
