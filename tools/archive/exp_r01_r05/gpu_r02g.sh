# round-2 session 2: GPU tests of the splice-path work + end-to-end spliced-read timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_extend.py tests/test_gpu_dropin.py tests/test_abi.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_ext.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_ext.log; exit 1; }
tail -3 gpurun_out/pytest_ext.log
timeout -k 10 600 python -u tools/splice_e2e.py --genome 50000005 --reads ${E2E_READS:-20000} --out gpurun_out/splice_e2e.json > gpurun_out/splice_e2e.log 2>&1 || { echo e2e failed; tail -20 gpurun_out/splice_e2e.log; exit 2; }
grep "\[e2e\]" gpurun_out/splice_e2e.log
echo ALLOK
