# A/B: libhsa_gpu.so (new) vs libhsa_gpu_old.so on configs 2 and 3, after the parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_ab3.log 2>&1 || { tail -30 gpurun_out/pt_ab3.log; echo pytest failed; exit 1; }
tail -1 gpurun_out/pt_ab3.log
run() {  # tag lib config
  HSA_GPU_LIB=$2 timeout -k 10 300 python -u bench.py --config $3 --steps ${STEPS:-4} --warmup 1 --cpu-sample 0 --parity-sample 4000 --dropin 0 > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || { tail gpurun_out/ab_$1.err; exit 2; }
  echo "$1: $(grep -h 'kernels\|parity:' gpurun_out/ab_$1.err | tr '\n' ' ')"
}
for r in 1 2; do
  run c2_new_$r libhsa_gpu.so 2
  run c2_old_$r libhsa_gpu_old.so 2
done
run c3_new libhsa_gpu.so 3
run c3_old libhsa_gpu_old.so 3
echo ALLOK
