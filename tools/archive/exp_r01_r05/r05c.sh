#!/bin/bash
# Round 5: the device splice kernel's first GPU tests, then the profiles of configs 2 and 3.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_splice_device.py \
    tests/test_gpu_dropin.py > gpurun_out/r05c_pytest.log 2>&1
rc=$?
tail -25 gpurun_out/r05c_pytest.log
[ $rc -eq 0 ] || exit 1
bash tools/profile_run.sh r05_c2 || exit 2
echo c2 done
BENCH_ARGS="--config 3" PASSES="fetch write sq" bash tools/profile_run.sh r05_c3 || exit 3
echo c3 done
