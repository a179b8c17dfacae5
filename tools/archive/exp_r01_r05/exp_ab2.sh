# A/B of library builds on one box (config 2, then config 3), alternating twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
for v in ${LIBS:-libhsa_gpu.so libhsa_gpu_old.so}; do
  HSA_GPU_LIB=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --cpu-sample 0 --parity-sample 0 ${BARGS:-} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail gpurun_out/ab_$v.err; exit 2; }
  echo "$v"; grep "kernels" gpurun_out/ab_$v.err
done
done
