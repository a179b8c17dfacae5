# A/B of the ski-rental batching trigger (HSA_BATCH_IDLE) against the fixed threshold
# (HSA_BATCH_K=16, idle trigger off) on configs 2 and 3, parity sampled
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # tag config env...
  local tag=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-4} --warmup 1 --cpu-sample 0 --parity-sample 4000 --dropin 0 > gpurun_out/id_$tag.json 2> gpurun_out/id_$tag.err || { tail gpurun_out/id_$tag.err; exit 2; }
  echo "$tag: $(grep -h 'kernels\|parity:' gpurun_out/id_$tag.err | tr '\n' ' ')"
}
run c2_k16 2 HSA_BATCH_K=16 HSA_BATCH_IDLE=100000000
run c2_i768 2 HSA_BATCH_IDLE=768
run c2_i384 2 HSA_BATCH_IDLE=384
run c2_i1536 2 HSA_BATCH_IDLE=1536
run c3_k16 3 HSA_BATCH_K=16 HSA_BATCH_IDLE=100000000
run c3_i768 3 HSA_BATCH_IDLE=768
run c3_i384 3 HSA_BATCH_IDLE=384
run c3_i1536 3 HSA_BATCH_IDLE=1536
echo ALLOK
