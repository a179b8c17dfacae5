# Round 3: drop-in stage timings at 100 000 and 1 M reads per call; config 4 profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
HSA_VERBOSE=1 timeout -k 10 300 python -u tools/dropin_time.py --reads 100000 > gpurun_out/r03k_dropin_100k.log 2>&1 || { tail -20 gpurun_out/r03k_dropin_100k.log; exit 1; }
grep -E "dropin_time|\[hsa\]" gpurun_out/r03k_dropin_100k.log | tail -14
BENCH_ARGS="--config 4" PASSES="fetch write" bash tools/profile_run.sh r03_c4 || exit 3
echo profiled
