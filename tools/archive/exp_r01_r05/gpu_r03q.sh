# Round 3 closing validation (2 of 2): configs 3, 4, 5 (whole-batch parity for 3 and 5),
# and config 5's kernel trace + HBM counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --config 3 --steps 10 --warmup 1 --cpu-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 \
    > gpurun_out/r03q_c3.json 2> gpurun_out/r03q_c3.err || { tail -30 gpurun_out/r03q_c3.err; exit 1; }
grep "per-step kernels\|parity" gpurun_out/r03q_c3.err
timeout -k 10 600 python -u bench.py --config 4 --steps 5 --warmup 1 --cpu-sample 0 \
    > gpurun_out/r03q_c4.json 2> gpurun_out/r03q_c4.err || { tail -30 gpurun_out/r03q_c4.err; exit 2; }
grep "per-step kernels\|parity" gpurun_out/r03q_c4.err
timeout -k 10 600 python -u bench.py --config 5 --steps 20 --warmup 2 --cpu-sample 0 \
    > gpurun_out/r03q_c5.json 2> gpurun_out/r03q_c5.err || { tail -30 gpurun_out/r03q_c5.err; exit 3; }
grep "per-step kernels\|parity" gpurun_out/r03q_c5.err
BENCH_ARGS="--config 5" PASSES="fetch write" bash tools/profile_run.sh r03_c5 || exit 4
echo profiled
