#!/bin/bash
# Round 5 (final tree): the whole GPU suite and smoke(), then >= 8 M config-3 reads against the restatement
# with the 16 384-entry gapped pools.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r05fin4_gpu_suite.log 2>&1 \
    || { tail -30 gpurun_out/r05fin4_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r05fin4_gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05fin4_smoke.log 2>&1 \
    || { tail -20 gpurun_out/r05fin4_smoke.log; exit 2; }
tail -1 gpurun_out/r05fin4_smoke.log
timeout -k 10 700 python -u tools/parity_10m.py --config 3 --batches 10 --max-seconds 560 --out gpurun_out/r05fin4_parity10m_c3.json \
    > gpurun_out/r05fin4_parity10m_c3.log 2>&1 || { tail -5 gpurun_out/r05fin4_parity10m_c3.log; exit 3; }
grep batch gpurun_out/r05fin4_parity10m_c3.log | tail -1 | cut -c1-250
echo done
