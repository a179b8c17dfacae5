#!/bin/bash
# Round 5: the default bench once more after config 2's default of three handles.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r05fin2_bench_default.json 2> gpurun_out/r05fin2_bench_default.err \
    || { tail -20 gpurun_out/r05fin2_bench_default.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/r05fin2_bench_default.json'));print(d['value'], d['roofline']['frac'], d['config']['streams'], (d.get('value_with_copies') or {}).get('value'), json.dumps(d.get('dropin_e2e'))[:160], json.dumps(d.get('parity_full'))[:80])"
echo done
