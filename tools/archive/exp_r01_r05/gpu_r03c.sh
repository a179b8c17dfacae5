# spliced end to end, 1 vs 16 runner threads (HSA_gpu_all), timing breakdown in the stderr
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in 1 4 16; do
HSA_SPLICE_THREADS=$t timeout -k 10 300 python -u tools/splice_e2e.py --reads 20000 --bins HSA_gpu_all \
    --out gpurun_out/r03c_e2e_t$t.json --stderr-dir gpurun_out > gpurun_out/r03c_e2e_t$t.log 2>&1 || { tail -20 gpurun_out/r03c_e2e_t$t.log; exit 2; }
mv gpurun_out/HSA_gpu_all.err gpurun_out/r03c_e2e_t${t}_HSA_gpu_all.err
grep "HSA_gpu_all: wall" gpurun_out/r03c_e2e_t$t.log | cut -c1-120
grep "splice runner\|batch of" gpurun_out/r03c_e2e_t${t}_HSA_gpu_all.err
done
