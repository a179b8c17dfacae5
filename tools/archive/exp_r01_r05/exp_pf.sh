# pool-head prefetch (HSA_PREFETCH=1 variant) on the gapped configs 3 and 4 (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pf
for C in 3 4; do
B="python3 bench.py --config $C --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 1000"
for V in base pf; do
if [ $V = pf ]; then export HSA_GPU_LIB=libhsa_gpu_pf.so; else unset HSA_GPU_LIB; fi
timeout -k 10 300 $B > gpurun_out/pf/c$C$V.json 2> gpurun_out/pf/c$C$V.err || { tail gpurun_out/pf/c$C$V.err; exit 2; }
python3 -c "import json;d=json.loads(open('gpurun_out/pf/c$C$V.json').read().strip().splitlines()[-1]);print($C,'$V',d['ms_per_step'],d['roofline']['kernel_split_ms'],d['parity_sample']['mismatching_reads'])"
done; done
