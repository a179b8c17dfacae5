# parity tests + config 2/3 timing (quick A/B loop)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_match_gap.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_q2.log 2>&1 || { tail -20 gpurun_out/pt_q2.log; exit 1; }
tail -1 gpurun_out/pt_q2.log
for k in ${KS:-16}; do
  HSA_BATCH_K=$k timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --cpu-sample 0 --parity-sample 20000 > gpurun_out/q2_$k.json 2> gpurun_out/q2_$k.err || { tail gpurun_out/q2_$k.err; exit 2; }
  echo "K=$k"; grep "kernels\|parity:" gpurun_out/q2_$k.err
done
HSA_BATCH_K=${K3:-16} timeout -k 10 300 python -u bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 4000 > gpurun_out/q3.json 2> gpurun_out/q3.err || { tail gpurun_out/q3.err; exit 3; }
echo "c3"; grep "kernels\|parity:" gpurun_out/q3.err
