# config 3: k_search time vs resident waves per CU (latency- vs issue-bound)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 4 6 8 11; do
  HSA_VERBOSE=1 timeout -k 10 300 python -u bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 2000 --dropin 0 --waves $w > gpurun_out/wv3_$w.json 2> gpurun_out/wv3_$w.err || { tail gpurun_out/wv3_$w.err; exit 2; }
  echo "w=$w: $(grep -h 'launch:' gpurun_out/wv3_$w.err | head -1) $(grep -h 'kernels' gpurun_out/wv3_$w.err)"
done
echo ALLOK
