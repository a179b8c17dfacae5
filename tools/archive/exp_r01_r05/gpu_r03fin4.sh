# Closing run of config 3 with every leg (the clones' scratch now freed before the
# drop-in end to end)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --config 3 --steps 10 --warmup 1 > gpurun_out/fin4_c3.json 2> gpurun_out/fin4_c3.err \
    || { tail -30 gpurun_out/fin4_c3.err; exit 2; }
grep -v "per-step device ms" gpurun_out/fin4_c3.err | tail -8
