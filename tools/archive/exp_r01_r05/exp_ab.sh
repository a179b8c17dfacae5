# A/B: default build vs an alternative in-tree build of libhsa_gpu (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --cpu-sample 0 --parity-sample 2000"
for L in ${LIBS:-libhsa_gpu.so}; do
  HSA_GPU_LIB=$L timeout -k 10 300 $B > gpurun_out/ab_$L.json 2> gpurun_out/ab_$L.err || exit 1
  echo "$L: $(grep per-step gpurun_out/ab_$L.err) $(grep 'parity sample' gpurun_out/ab_$L.err)"
done
