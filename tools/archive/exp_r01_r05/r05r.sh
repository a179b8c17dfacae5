#!/bin/bash
# Round 5 (final build): 10 M config-2 reads and >= 8 M config-3 reads against the restatement at hg19 size.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/parity_10m.py --config 2 --batches 10 --out gpurun_out/r05f_parity10m_c2.json \
    > gpurun_out/r05f_parity10m_c2.log 2>&1 || { tail -5 gpurun_out/r05f_parity10m_c2.log; exit 1; }
grep batch gpurun_out/r05f_parity10m_c2.log | tail -1 | cut -c1-250
timeout -k 10 760 python -u tools/parity_10m.py --config 3 --batches 10 --max-seconds 600 --out gpurun_out/r05f_parity10m_c3.json \
    > gpurun_out/r05f_parity10m_c3.log 2>&1 || { tail -5 gpurun_out/r05f_parity10m_c3.log; exit 2; }
grep batch gpurun_out/r05f_parity10m_c3.log | tail -1 | cut -c1-250
echo done
