# does k_search time follow its memory request count? extra random loads per strand start
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in libhsa_gpu.so libhsa_gpu_x20.so libhsa_gpu_x60.so; do
  HSA_GPU_LIB=$v timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --cpu-sample 0 --parity-sample 0 > gpurun_out/x_$v.json 2> gpurun_out/x_$v.err || { tail gpurun_out/x_$v.err; exit 2; }
  echo $v; grep "kernels" gpurun_out/x_$v.err
done
