#!/bin/bash
# Round 5: >= 8 M config-3 reads of parity at hg19 size on the final search kernels; config-4 drop-in end to end.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u tools/parity_10m.py --config 3 --batches 10 --max-seconds 560 --out gpurun_out/r05_parity10m_c3.json \
    > gpurun_out/r05_parity10m_c3.log 2>&1 || { tail -5 gpurun_out/r05_parity10m_c3.log; exit 1; }
grep batch gpurun_out/r05_parity10m_c3.log | tail -2 | cut -c1-250
HSA_E2E_LOG=gpurun_out/r05i_e2e_c4.log timeout -k 10 600 python -u bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 \
    --parity-sample 0 > gpurun_out/r05i_bench_c4.json 2> gpurun_out/r05i_bench_c4.err || { tail -20 gpurun_out/r05i_bench_c4.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/r05i_bench_c4.json'));print('c4', d['value'], json.dumps(d.get('dropin_e2e'))[:300], d.get('parity_reference'))"
