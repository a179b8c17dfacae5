# Round 3, HEAD check after the container restore: the whole -m gpu suite (strand-split
# main pass included), smoke, then the default bench (config 2) at 200 steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03d_pytest.log 2>&1 || { tail -40 gpurun_out/r03d_pytest.log; exit 1; }
tail -3 gpurun_out/r03d_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03d_smoke.log 2>&1 || { tail -20 gpurun_out/r03d_smoke.log; exit 2; }
cat gpurun_out/r03d_smoke.log
timeout -k 10 900 python -u bench.py --steps 200 --warmup 5 > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err \
    || { tail -40 gpurun_out/r03d_bench.err; exit 3; }
tail -12 gpurun_out/r03d_bench.err
timeout -k 10 300 python -u tools/exp/depth_hist.py --out gpurun_out/r03d_depth_hist.json > gpurun_out/r03d_depth_hist.log 2>&1 \
    || { tail -20 gpurun_out/r03d_depth_hist.log; exit 4; }
cat gpurun_out/r03d_depth_hist.log | grep -v "^\[bench\]"
