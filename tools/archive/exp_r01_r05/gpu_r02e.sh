# round 2: PC sampling of config 3's k_search; the 64-bit instantiation's cost on the
# same 250 bp workload at 3 Gbp (32- vs 64-bit intervals); config 4 refresh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PFX=c3_ BENCH_ARGS="--config 3 --steps 1" bash tools/exp/exp_pcs.sh
for iv in 32 64; do
  timeout -k 10 300 python -u bench.py --config 5 --genome 3000000005 --intervals $iv --steps 3 --warmup 1 --cpu-sample 0 --parity-sample 4000 --dropin 0 > gpurun_out/iv_$iv.json 2> gpurun_out/iv_$iv.err || { tail gpurun_out/iv_$iv.err; exit 2; }
  echo "iv=$iv: $(grep -h 'kernels\|parity:' gpurun_out/iv_$iv.err | tr '\n' ' ')"
done
timeout -k 10 400 python -u bench.py --config 4 --steps 2 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail gpurun_out/bench_c4.err; exit 3; }
grep "kernels\|parity" gpurun_out/bench_c4.err
echo ALLOK
