# the spliced-read drop-in with the extension runner traced (per-round and per-launch times)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HSA_EXT_TRACE=1
mkdir -p gpurun_out/e2e_trace
timeout -k 10 600 python -u tools/splice_e2e.py --genome 50000005 --reads ${E2E_READS:-20000} --bins ${E2E_BINS:-HSA_gpu_mg HSA_gpu_all} --stderr-dir gpurun_out/e2e_trace --out gpurun_out/e2e_trace/e2e.json > gpurun_out/e2e_trace/e2e.log 2>&1 || { echo e2e failed; tail -20 gpurun_out/e2e_trace/e2e.log; exit 2; }
grep "\[e2e\]" gpurun_out/e2e_trace/e2e.log | cut -c1-300
grep -c "hsa_extend_sliced" gpurun_out/e2e_trace/HSA_gpu_all.err
head -30 gpurun_out/e2e_trace/HSA_gpu_all.err
echo ALLOK
