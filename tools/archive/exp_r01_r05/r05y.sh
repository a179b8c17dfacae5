#!/bin/bash
# Round 5: the 12-mer anchor searches' main-pass pool (HSA_POOL_SHORT) and config 4 on two handles.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "scratch_release" \
    > gpurun_out/r05y_tests.log 2>&1 || { tail -20 gpurun_out/r05y_tests.log; exit 1; }
tail -1 gpurun_out/r05y_tests.log
run() {   # tag streams pool_short
  HSA_VERBOSE=1 HSA_POOL_SHORT=$3 timeout -k 10 500 python bench.py --config 4 --streams $2 --steps 4 --warmup 2 --dropin 0 --ref-sample 0 \
      --parity-sample 1000 --cpu-sample 0 > gpurun_out/r05y_$1.json 2> gpurun_out/r05y_$1.err || { grep -E "hipMalloc|scratch" gpurun_out/r05y_$1.err | tail -4; tail -2 gpurun_out/r05y_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05y_$1.json'));r=d['roofline'];print('$1', d['value'], d['ms_per_step'], r.get('k_search_ms'), r.get('splice_path_ms'), d['config'].get('streams'), json.dumps(d.get('parity_sample'))[:90])"
}
run s1_default 1 0
run s1_short8k 1 8192
run s2_short8k 2 8192 && run s2_short8k_b 2 8192
echo done
