#!/bin/bash
# Round 5 (final build): search and drop-in tests after the short-search pool default, then config 4 with the
# bench's defaults (two handles, reference legs, end to end).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_any.py \
    tests/test_gpu_splice_device.py tests/test_gpu_splice_prefetch.py tests/test_gpu_dropin.py tests/test_gpu_config4.py \
    > gpurun_out/r05z_tests.log 2>&1 || { tail -20 gpurun_out/r05z_tests.log; exit 1; }
tail -1 gpurun_out/r05z_tests.log
HSA_E2E_LOG=gpurun_out/r05z_e2e_c4.log timeout -k 10 900 python -u bench.py --config 4 > gpurun_out/r05z_c4.json 2> gpurun_out/r05z_c4.err \
    || { tail -8 gpurun_out/r05z_c4.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/r05z_c4.json'));r=d['roofline'];print('c4', d['value'], r.get('k_search_ms'), r['frac'], (d.get('cpu_baseline') or {}).get('value'), json.dumps(d.get('dropin_e2e'))[:220], json.dumps(d.get('parity_reference'))[:100])"
echo done
