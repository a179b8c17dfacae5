# overflow re-run grid size (HSA_BIG_LANES) on config 4 (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/big
B="python3 bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 1000"
for L in 4096 16384 32768; do
HSA_BIG_LANES=$L timeout -k 10 300 $B > gpurun_out/big/b$L.json 2> gpurun_out/big/b$L.err || { tail gpurun_out/big/b$L.err; exit 2; }
python3 -c "import json;d=json.loads(open('gpurun_out/big/b$L.json').read().strip().splitlines()[-1]);print($L,d['ms_per_step'],d['roofline']['kernel_split_ms'],d['parity_sample'])"
done
