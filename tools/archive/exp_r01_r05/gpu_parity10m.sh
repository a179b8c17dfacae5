# 10 M-read parity runs (tools/parity_10m.py): config 2 whole, config 3 up to a wall budget
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u tools/parity_10m.py --config 2 --batches 10 --out gpurun_out/parity10m_c2.json > gpurun_out/parity10m_c2.log 2>&1 || { echo c2 failed; tail -5 gpurun_out/parity10m_c2.log; exit 1; }
tail -1 gpurun_out/parity10m_c2.log | cut -c1-400
timeout -k 10 700 python -u tools/parity_10m.py --config 3 --batches 10 --max-seconds ${C3_SECONDS:-560} --out gpurun_out/parity10m_c3.json > gpurun_out/parity10m_c3.log 2>&1 || { echo c3 failed; tail -5 gpurun_out/parity10m_c3.log; exit 2; }
grep batch gpurun_out/parity10m_c3.log | tail -3
echo ALLOK
