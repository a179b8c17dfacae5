# round 2: unique-interval census (diagnostic build) on configs 2 and 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HSA_GPU_LIB=libhsa_gpu_diag.so
mkdir -p gpurun_out
for c in 2 3; do
  HSA_DIAG_OUT=$GRAFT_REPO_ROOT/gpurun_out/diag_c$c.json timeout -k 10 300 python -u bench.py --config $c --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 0 > gpurun_out/diag_c$c.out 2> gpurun_out/diag_c$c.err || { tail gpurun_out/diag_c$c.err; exit 2; }
  cat gpurun_out/diag_c$c.json; echo
done
