# A/B of experiment builds: VARS="lib1 lib2 ..." CFGS="2 3" (libhsa_gpu_<v>.so, "base" = libhsa_gpu.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in ${CFGS:-3}; do
  for v in ${VARS:-base}; do
    lib=libhsa_gpu_$v.so; [ "$v" = base ] && lib=libhsa_gpu.so
    HSA_GPU_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-3} --warmup 1 --cpu-sample 0 --parity-sample ${PAR:-2000} --dropin 0 > gpurun_out/var_${c}_$v.json 2> gpurun_out/var_${c}_$v.err || { tail gpurun_out/var_${c}_$v.err; exit 2; }
    echo "c$c $v: $(grep -h 'kernels\|parity:' gpurun_out/var_${c}_$v.err | tr '\n' ' ')"
  done
done
echo ALLOK
