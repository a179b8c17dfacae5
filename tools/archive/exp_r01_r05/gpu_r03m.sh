# Round 3: k_search at 5 waves per SIMD (libhsa_gpu_w5.so: launch bound 5, VGPRs <= 96):
# config 2 with 4-bit rows at 20 waves per CU, and 8-bit rows (LDS-bound at 16); config 5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B2="python -u bench.py --steps 40 --warmup 3 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 --parity-sample 100000"
B5="python -u bench.py --config 5 --steps 10 --warmup 2 --cpu-sample 0 --parity-sample 0"
run() {  # tag, env..., -- cmd
  local t=$1; shift
  env "$@" > gpurun_out/r03m_$t.json 2> gpurun_out/r03m_$t.err || { tail -20 gpurun_out/r03m_$t.err; exit 2; }
  echo "$t: $(grep 'per-step kernels\|parity:\|launch:' gpurun_out/r03m_$t.err | tr '\n' ' ')"
}
run c2_base HSA_VERBOSE=0 timeout -k 10 300 $B2
run c2_w5nib HSA_GPU_LIB=libhsa_gpu_w5.so HSA_WFMT=nib timeout -k 10 300 $B2 --waves 20
run c2_w5byte HSA_GPU_LIB=libhsa_gpu_w5.so timeout -k 10 300 $B2
run c5_base HSA_VERBOSE=0 timeout -k 10 400 $B5
run c5_w5 HSA_GPU_LIB=libhsa_gpu_w5.so timeout -k 10 400 $B5 --waves 20
