# A/B of the rare-event batching threshold (HSA_BATCH_K) on configs 2 and 3, parity sampled
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_batch.log 2>&1 || { tail -20 gpurun_out/pt_batch.log; exit 1; }
tail -1 gpurun_out/pt_batch.log
for k in 1 4 8 16 32; do
  HSA_BATCH_K=$k timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --cpu-sample 0 --parity-sample 4000 > gpurun_out/bk_$k.json 2> gpurun_out/bk_$k.err || { tail gpurun_out/bk_$k.err; exit 2; }
  echo "K=$k"; grep "kernels\|parity:" gpurun_out/bk_$k.err
done
for k in 1 8 32; do
  HSA_BATCH_K=$k timeout -k 10 300 python -u bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 2000 > gpurun_out/bk3_$k.json 2> gpurun_out/bk3_$k.err || { tail gpurun_out/bk3_$k.err; exit 3; }
  echo "c3 K=$k"; grep "kernels\|parity:" gpurun_out/bk3_$k.err
done
