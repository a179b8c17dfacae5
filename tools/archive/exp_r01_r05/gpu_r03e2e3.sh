# The drop-in end to end on config 3's reads (it failed in the closing run): full stderr kept
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
HSA_E2E_LOG=gpurun_out/e2e3_stderr.log timeout -k 10 900 python -u bench.py --config 3 --steps 2 --warmup 1 --parity-sample 0 --cpu-sample 0 --dropin 0 \
    > gpurun_out/e2e3.json 2> gpurun_out/e2e3.err || { tail -30 gpurun_out/e2e3.err; exit 1; }
grep -v "per-step device ms" gpurun_out/e2e3.err | tail -5
grep -v "^\[hsa\] " gpurun_out/e2e3_stderr.log | tail -20
