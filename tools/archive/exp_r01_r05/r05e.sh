#!/bin/bash
# Round 5: config 4 with the whole splice path in the timed step; the default config-2 bench.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --config 4 --steps 3 --warmup 1 --e2e-reads 0 \
    > gpurun_out/r05e_bench_c4.json 2> gpurun_out/r05e_bench_c4.err || { tail -20 gpurun_out/r05e_bench_c4.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r05e_bench_c4.json'));print('c4', d['value'], d['roofline'].get('splice_path_ms'), json.dumps(d.get('splice_path'))[:400], json.dumps(d.get('parity_reference'))[:300])"
timeout -k 10 900 python -u bench.py > gpurun_out/r05e_bench_c2.json 2> gpurun_out/r05e_bench_c2.err || { tail -20 gpurun_out/r05e_bench_c2.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/r05e_bench_c2.json'));print('c2', d['value'], d['roofline']['k_search_ms'], json.dumps(d.get('value_with_copies'))[:300], json.dumps(d.get('dropin'))[:200], d.get('dropin_e2e',{}).get('value'))"
