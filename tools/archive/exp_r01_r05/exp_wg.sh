# 64-lane vs 256-lane search workgroups on the gapped configuration (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_match_gap.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_wg.log 2>&1 || { tail -30 gpurun_out/pytest_wg.log; exit 1; }
tail -1 gpurun_out/pytest_wg.log
B="python3 bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 2000"
HSA_VERBOSE=1 timeout -k 10 300 $B > gpurun_out/wg64.json 2> gpurun_out/wg64.err || { tail gpurun_out/wg64.err; exit 2; }
HSA_WG256=1 timeout -k 10 300 $B > gpurun_out/wg256.json 2> gpurun_out/wg256.err || { tail gpurun_out/wg256.err; exit 3; }
for f in wg64 wg256; do echo "$f: $(grep -m1 'launch:' gpurun_out/$f.err) $(grep per-step gpurun_out/$f.err) $(grep 'parity sample' gpurun_out/$f.err)"; done
