# Round 3: chunked pool layout (HSA_POOL_CHUNK, libhsa_gpu_chunk.so) against the default,
# configs 3 and 2; the chunked build's timed batch checked against the restatement
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libhsa_gpu.so libhsa_gpu_chunk.so; do
  HSA_GPU_LIB=$lib timeout -k 10 400 python -u bench.py --config 3 --steps 8 --warmup 1 --cpu-sample 0 --ref-sample 0 \
      --dropin 0 --e2e-reads 0 --parity-sample 100000 > gpurun_out/r03i_c3_$lib.json 2> gpurun_out/r03i_c3_$lib.err \
      || { tail -20 gpurun_out/r03i_c3_$lib.err; exit 2; }
  echo "c3 $lib: $(grep 'per-step kernels\|parity:' gpurun_out/r03i_c3_$lib.err | tr '\n' ' ')"
done
for lib in libhsa_gpu.so libhsa_gpu_chunk.so; do
  HSA_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --steps 40 --warmup 3 --cpu-sample 0 --ref-sample 0 \
      --dropin 0 --e2e-reads 0 --parity-sample 100000 > gpurun_out/r03i_c2_$lib.json 2> gpurun_out/r03i_c2_$lib.err \
      || { tail -20 gpurun_out/r03i_c2_$lib.err; exit 3; }
  echo "c2 $lib: $(grep 'per-step kernels\|parity:' gpurun_out/r03i_c2_$lib.err | tr '\n' ' ')"
done
