# config 2's k_search at 8, 12 and 16 resident waves per CU (bench --waves): how much of
# the long-read configs' gap to the probe is occupancy
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/waves2
O=gpurun_out/waves2
for w in 8 12 16; do
  HSA_VERBOSE=1 timeout -k 10 300 python -u bench.py --config 2 --steps 3 --warmup 1 --cpu-sample 0 --parity-sample 2000 --dropin 0 --waves $w > $O/w$w.json 2> $O/w$w.err || { tail $O/w$w.err; exit 2; }
  echo "w$w: $(grep -h 'launch:' $O/w$w.err | sort | uniq -c | sort -rn | head -1) | $(grep -h 'kernels' $O/w$w.err | tr '\n' ' ')"
done
echo ALLOK
