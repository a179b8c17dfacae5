# in-kernel clock + workgroup spread, plain and under rocprofv3 (diagnostic build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export HSA_GPU_LIB=${HSA_GPU_LIB:-libhsa_gpu_diag.so} HSA_VERBOSE=1
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --cpu-sample 0 --parity-sample 0 $BENCH_ARGS"
HSA_DIAG_OUT=$GRAFT_REPO_ROOT/gpurun_out/diag_plain.json timeout -k 10 300 $B > gpurun_out/d_plain.json 2> gpurun_out/d_plain.err || { tail gpurun_out/d_plain.err; exit 2; }
grep -h "per-step\|diag\|launch:" gpurun_out/d_plain.err
