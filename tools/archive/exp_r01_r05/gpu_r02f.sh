# round 2: compact 64-bit superblocks (16-byte entries) -- wide-index parity on the GPU,
# then the 64-bit search A/B against the previous build (32-byte entries) at 3 Gbp, and config 5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/pt_wide.log 2>&1 || { tail -20 gpurun_out/pt_wide.log; exit 1; }
tail -2 gpurun_out/pt_wide.log
for v in oldsup base oldsup base; do
  lib=libhsa_gpu_$v.so; [ "$v" = base ] && lib=libhsa_gpu.so
  HSA_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --config 5 --genome 3000000005 --intervals 64 --steps 3 --warmup 1 --cpu-sample 0 --parity-sample 4000 --dropin 0 > gpurun_out/sup_$v.json 2> gpurun_out/sup_$v.err || { tail gpurun_out/sup_$v.err; exit 2; }
  echo "$v: $(grep -h 'kernels\|parity:' gpurun_out/sup_$v.err | tr '\n' ' ')"
done
timeout -k 10 600 python -u bench.py --config 5 --steps 3 --warmup 1 --cpu-sample 0 --parity-sample 20000 --dropin 0 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail gpurun_out/c5.err; exit 3; }
grep -h 'kernels\|parity' gpurun_out/c5.err
timeout -k 10 900 python -u tools/splice_e2e.py --genome 50000005 --reads 5000 --workdir /tmp/e2e --out gpurun_out/splice_e2e.json > gpurun_out/splice_e2e.log 2>&1 || { tail -20 gpurun_out/splice_e2e.log; exit 4; }
grep "\[e2e\]" gpurun_out/splice_e2e.log
echo ALLOK
