#!/bin/bash
# Round 5: 16 384-entry pools for gapped reads of <= 128 bases -- search tests, then configs 3 and 2 with the bench's defaults.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_any.py \
    tests/test_gpu_hg19.py tests/test_gpu_dropin.py tests/test_gpu_match_gap.py > gpurun_out/r05fin3_tests.log 2>&1 || { tail -20 gpurun_out/r05fin3_tests.log; exit 1; }
tail -1 gpurun_out/r05fin3_tests.log
timeout -k 10 900 python -u bench.py --config 3 > gpurun_out/r05fin3_c3.json 2> gpurun_out/r05fin3_c3.err || { tail -8 gpurun_out/r05fin3_c3.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/r05fin3_c3.json'));r=d['roofline'];print('c3', d['value'], r.get('k_search_ms'), r['frac'], d['config']['streams'], (d.get('cpu_baseline') or {}).get('value'), json.dumps(d.get('dropin_e2e'))[:120], json.dumps(d.get('parity_full'))[:80])"
echo done
