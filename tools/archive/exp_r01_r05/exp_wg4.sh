# 64-lane vs 256-lane search workgroups on config 4 (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/wg4
B="python3 bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 1000"
HSA_VERBOSE=1 timeout -k 10 300 $B > gpurun_out/wg4/wg64.json 2> gpurun_out/wg4/wg64.err || { tail gpurun_out/wg4/wg64.err; exit 2; }
HSA_VERBOSE=1 HSA_WG256=1 timeout -k 10 300 $B > gpurun_out/wg4/wg256.json 2> gpurun_out/wg4/wg256.err || { tail gpurun_out/wg4/wg256.err; exit 3; }
for f in wg64 wg256; do python3 -c "import json;d=json.loads(open('gpurun_out/wg4/$f.json').read().strip().splitlines()[-1]);print('$f',d['ms_per_step'],d['roofline']['kernel_split_ms'],d['parity_sample']['mismatching_reads'])"; grep -m2 'launch:' gpurun_out/wg4/$f.err; done
