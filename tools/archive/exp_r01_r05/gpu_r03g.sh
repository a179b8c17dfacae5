# Round 3: in-kernel counters (diag build) of config 2, k_search without / with the search trie
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --steps 10 --warmup 2 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 --parity-sample 0"
for m in 0 1 2; do
  HSA_GPU_LIB=libhsa_gpu_diag.so HSA_DIAG_OUT=gpurun_out/r03g_diag_m$m.json HSA_TRIE_MODE=$m timeout -k 10 300 $B \
     > gpurun_out/r03g_m$m.json 2> gpurun_out/r03g_m$m.err || { tail -20 gpurun_out/r03g_m$m.err; exit 2; }
  echo "mode $m: $(grep 'per-step kernels' gpurun_out/r03g_m$m.err)"
  cat gpurun_out/r03g_diag_m$m.json; echo
done
