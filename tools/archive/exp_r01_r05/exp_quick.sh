# gpu tests, then the bench plain and under rocprofv3 --kernel-trace (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1 || { tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -1 gpurun_out/q_pytest.log
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --cpu-sample 0 --parity-sample 2000 $BENCH_ARGS"
timeout -k 10 300 $B > gpurun_out/q_plain.json 2> gpurun_out/q_plain.err || exit 2
grep -h "per-step\|parity\|split" gpurun_out/q_plain.err
if [ -n "$PROF" ]; then
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/q_kt -o run -- $B > $GRAFT_REPO_ROOT/gpurun_out/q_kt.json 2> $GRAFT_REPO_ROOT/gpurun_out/q_kt.err || exit 3
grep -h "per-step" $GRAFT_REPO_ROOT/gpurun_out/q_kt.err
fi
