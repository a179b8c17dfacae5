set -o pipefail
TAG=r01d
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="$R/bench.py --steps 5 --warmup 1 --cpu-sample 0 --parity-sample 0"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.json 2> $OUT/trace.err || exit 11
for n in fetch:FETCH_SIZE write:WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc ${n#*:} --kernel-include-regex "k_search|k_widths" --output-format csv -d $OUT/pmc_${n%%:*} -o run -- python3 $BENCH > $OUT/pmc_${n%%:*}.json 2> $OUT/pmc_${n%%:*}.err || exit 12
done
cp -r $R/gpurun_out/prof_r01c/pmc_membench $R/gpurun_out/prof_r01c/pmc_sq $R/gpurun_out/prof_r01c/pmc_tcc $OUT/ 2>/dev/null
echo done
