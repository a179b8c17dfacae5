# main-pass pool capacity, larger values on config 4 and config 3's sensitivity (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pool
B="python3 bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 1000"
for P in 49152 65535; do
timeout -k 10 300 $B --pool $P > gpurun_out/pool/p$P.json 2> gpurun_out/pool/p$P.err || { tail gpurun_out/pool/p$P.err; exit 2; }
python3 -c "import json;d=json.loads(open('gpurun_out/pool/p$P.json').read().strip().splitlines()[-1]);print($P,d['ms_per_step'],d['roofline']['kernel_split_ms'],d['parity_sample'])"
done
B="python3 bench.py --config 3 --steps 3 --warmup 1 --cpu-sample 0 --parity-sample 1000"
for P in 0 32768; do
timeout -k 10 300 $B --pool $P > gpurun_out/pool/c3p$P.json 2> gpurun_out/pool/c3p$P.err || { tail gpurun_out/pool/c3p$P.err; exit 3; }
python3 -c "import json;d=json.loads(open('gpurun_out/pool/c3p$P.json').read().strip().splitlines()[-1]);print('c3',$P,d['ms_per_step'],d['roofline']['kernel_split_ms'],d['parity_sample'])"
done
