#!/bin/bash
# Round 5: rehearsal of the N = 2 bench path on the one-GPU box (ranks share the GPU, collectives over gloo).
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
HSA_BENCH_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --streams 2 --steps 3 --warmup 1 \
    > gpurun_out/r05rh_2rank.json 2> gpurun_out/r05rh_2rank.err || { tail -15 gpurun_out/r05rh_2rank.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r05rh_2rank.json'));print(d['n_gpus'], d['value'], d['roofline'].get('frac'), json.dumps(d.get('parity_ranks'))[:200], (d.get('cpu_baseline') or {}).get('value'))"
echo done
