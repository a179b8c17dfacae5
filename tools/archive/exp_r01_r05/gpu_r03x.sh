# Rehearsal of the N-rank bench path on a 1-GPU box: bench.py --gpus 2 spawns two
# ranks, both on GPU 0, collectives over gloo (HSA_BENCH_BACKEND=gloo); per-rank
# parity, the gather and its digest check are what is looked at, not the rate
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
export HSA_BENCH_BACKEND=gloo
timeout -k 10 500 python -u bench.py --gpus 2 --steps 6 --warmup 2 > gpurun_out/r03x_c2.json 2> gpurun_out/r03x_c2.err \
    || { tail -40 gpurun_out/r03x_c2.err; exit 1; }
grep -v "per-step device ms" gpurun_out/r03x_c2.err | tail -12
timeout -k 10 500 python -u bench.py --gpus 2 --config 3 --steps 4 --warmup 1 > gpurun_out/r03x_c3.json 2> gpurun_out/r03x_c3.err \
    || { tail -40 gpurun_out/r03x_c3.err; exit 2; }
grep -v "per-step device ms" gpurun_out/r03x_c3.err | tail -8
