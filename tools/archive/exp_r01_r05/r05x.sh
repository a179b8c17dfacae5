#!/bin/bash
# Round 5 (final build): configs 3 and 5 with the bench's defaults (two handles, reference legs, end to end).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 3 5; do
  timeout -k 10 900 python -u bench.py --config $c > gpurun_out/r05x_c$c.json 2> gpurun_out/r05x_c$c.err || { tail -8 gpurun_out/r05x_c$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05x_c$c.json'));r=d['roofline'];print('c$c', d['value'], r.get('k_search_ms'), r['frac'], (d.get('cpu_baseline') or {}).get('value'), json.dumps(d.get('dropin_e2e'))[:160], json.dumps(d.get('parity_full'))[:100])"
done
echo done
