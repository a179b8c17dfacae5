# Round 3: the drop-in end to end with every stage timing (HSA_VERBOSE log of ref_probe_gpu)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
HSA_E2E_LOG=gpurun_out/r03r_e2e.log timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 --parity-sample 0 \
    --ref-sample 16000 > gpurun_out/r03r_bench.json 2> gpurun_out/r03r_bench.err || { tail -30 gpurun_out/r03r_bench.err; exit 1; }
grep "drop-in end to end" gpurun_out/r03r_bench.err
grep -E "prefetch|splice|batch of|cal_sa_reg_gap of" gpurun_out/r03r_e2e.log | head -30
