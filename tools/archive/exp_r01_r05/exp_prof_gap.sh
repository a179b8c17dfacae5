# Does the search kernel run at a different speed under rocprofv3? (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --cpu-sample 0 --parity-sample 0"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/exp_plain$i.json 2> gpurun_out/exp_plain$i.err || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/exp_kt -o run -- $B > $GRAFT_REPO_ROOT/gpurun_out/exp_kt.json 2> $GRAFT_REPO_ROOT/gpurun_out/exp_kt.err || exit 2
cd $GRAFT_REPO_ROOT
timeout -k 10 300 $B > gpurun_out/exp_plain3.json 2> gpurun_out/exp_plain3.err || exit 3
grep -h "per-step" gpurun_out/exp_*.err
