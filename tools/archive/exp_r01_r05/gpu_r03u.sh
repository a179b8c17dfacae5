# Round 3: the unique-interval walk with a streak trigger -- its parity tests, then
# config 2 without it and with streaks 1, 2, 4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_walk.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03u_pytest_walk.log 2>&1 || { tail -60 gpurun_out/r03u_pytest_walk.log; exit 1; }
tail -2 gpurun_out/r03u_pytest_walk.log
B2="python -u bench.py --steps 40 --warmup 3 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 --parity-sample 100000"
for v in "HSA_WALK=0" "HSA_WALK_STREAK=1" "HSA_WALK_STREAK=2" "HSA_WALK_STREAK=4" "HSA_WALK_STREAK=8"; do
  env $v timeout -k 10 300 $B2 > gpurun_out/r03u_$v.json 2> gpurun_out/r03u_$v.err || { tail -20 gpurun_out/r03u_$v.err; exit 3; }
  echo "$v: $(grep 'per-step kernels\|parity:' gpurun_out/r03u_$v.err | tr '\n' ' ')"
done
