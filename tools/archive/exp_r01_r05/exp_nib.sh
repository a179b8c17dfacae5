# A/B of the 4-bit pruning rows (HSA_WFMT=byte keeps 8-bit rows; default picks 4-bit
# when 8-bit rows leave the CU short of 16 waves): configs 3, 4, config 5's reads on a
# 3 Gbp text, and config 5 itself
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HSA_VERBOSE=1
O=gpurun_out/nib
mkdir -p $O
A="--steps 3 --warmup 1 --cpu-sample 0 --parity-sample 4000 --dropin 0"
run() {  # name wfmt args...
  n=$1; w=$2; shift 2
  HSA_WFMT=$w timeout -k 10 400 python -u bench.py $A "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 2; }
  echo "$n: $(grep -h 'launch:' $O/$n.err | sort | uniq -c | sort -rn | head -1 | cut -c1-200) | $(grep -h 'kernels\|parity:' $O/$n.err | tr '\n' ' ' | cut -c1-300)"
}
run c3_byte byte --config 3
run c3_auto auto --config 3
run g3_250_byte byte --config 5 --genome 3000000005 --intervals 32
run g3_250_auto auto --config 5 --genome 3000000005 --intervals 32
run c4_byte byte --config 4 --steps 2
run c4_auto auto --config 4 --steps 2
run c5_auto auto --config 5
echo ALLOK
