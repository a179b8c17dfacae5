# Round 3: root-trie variants on config 2 (k_widths / k_search ms per step)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --steps 40 --warmup 3 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 --parity-sample 0"
for v in "HSA_TRIE=0" "HSA_TRIE_MODE=0" "HSA_TRIE_MODE=1" "HSA_TRIE_MODE=2" "HSA_TRIE_SDEPTH=8" "HSA_TRIE_SDEPTH=6" "HSA_TRIE_DEPTH=12" "HSA_TRIE_DEPTH=9"; do
  env $v timeout -k 10 300 $B > gpurun_out/r03f_$v.json 2> gpurun_out/r03f_$v.err || { tail -20 gpurun_out/r03f_$v.err; exit 2; }
  echo "$v: $(grep 'per-step kernels' gpurun_out/r03f_$v.err)"
done
