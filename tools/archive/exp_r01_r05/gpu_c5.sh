# config 5: 15 Gbp synthetic plant-scale index (64-bit intervals), 1M x 250 bp per step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py --config 5 --steps 5 --warmup 1 ${C5ARGS:-} > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail -20 gpurun_out/bench_c5.err; exit 3; }
grep "built\|ready\|generated\|kernels\|parity\|probe" gpurun_out/bench_c5.err
cat gpurun_out/bench_c5.json
echo ALLOK
