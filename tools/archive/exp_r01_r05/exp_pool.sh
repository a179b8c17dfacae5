# main-pass pool capacity (bench --pool) on config 4: fewer overflow re-runs (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pool
B="python3 bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 1000"
for P in 0 24576 32768; do
timeout -k 10 300 $B --pool $P > gpurun_out/pool/p$P.json 2> gpurun_out/pool/p$P.err || { tail gpurun_out/pool/p$P.err; exit 2; }
python3 -c "import json;d=json.loads(open('gpurun_out/pool/p$P.json').read().strip().splitlines()[-1]);print($P,d['ms_per_step'],d['roofline']['kernel_split_ms'],d['parity_sample'])"
done
