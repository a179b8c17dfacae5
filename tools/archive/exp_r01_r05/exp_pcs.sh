# PC sampling of k_search (config 2, or BENCH_ARGS): which instructions the waves sit on
set -o pipefail
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${M:-stochastic} --pc-sampling-unit ${U:-cycles} --pc-sampling-interval ${I:-65536} --output-format csv -d $R/gpurun_out/${PFX:-}pcs -o run -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 0 --dropin 0 $BENCH_ARGS > $R/gpurun_out/${PFX:-}pcs.log 2>&1
echo rc=$?
ls -la $R/gpurun_out/${PFX:-}pcs 2>/dev/null | head
tail -5 $R/gpurun_out/${PFX:-}pcs.log
