# Same bench under different runtime environments / the profiler (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --cpu-sample 0 --parity-sample 0"
i=0
for E in "X=1" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0"; do
  i=$((i+1))
  env $E timeout -k 10 300 $B > gpurun_out/env_$i.json 2> gpurun_out/env_$i.err || exit 1
  echo "$E: $(grep per-step gpurun_out/env_$i.err)"
done
timeout -k 10 120 ./tools/membench 2147483648 16 > gpurun_out/mb_plain.log 2>&1 || exit 2
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/mb_kt -o run -- $GRAFT_REPO_ROOT/tools/membench 2147483648 16 > $GRAFT_REPO_ROOT/gpurun_out/mb_kt.log 2>&1 || exit 3
cat $GRAFT_REPO_ROOT/gpurun_out/mb_plain.log; grep mode $GRAFT_REPO_ROOT/gpurun_out/mb_kt.log
