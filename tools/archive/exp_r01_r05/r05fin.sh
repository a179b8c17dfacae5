#!/bin/bash
# Round 5 (final build): the whole GPU suite, smoke(), the default bench (config 2, as the driver runs it),
# at the end of round 5.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r05fin_gpu_suite.log 2>&1 \
    || { tail -30 gpurun_out/r05fin_gpu_suite.log; exit 1; }
tail -1 gpurun_out/r05fin_gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05fin_smoke.log 2>&1 \
    || { tail -20 gpurun_out/r05fin_smoke.log; exit 2; }
tail -1 gpurun_out/r05fin_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r05fin_bench_default.json 2> gpurun_out/r05fin_bench_default.err \
    || { tail -20 gpurun_out/r05fin_bench_default.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/r05fin_bench_default.json'));print(d['value'], d['roofline']['frac'], d.get('value_with_copies'), json.dumps(d.get('dropin_e2e'))[:200])"
echo done
