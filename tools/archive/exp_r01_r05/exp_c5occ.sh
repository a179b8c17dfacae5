# config 5 launch shape and the cost of 64-bit intervals vs 250 bp reads: the 15 Gbp run
# under HSA_VERBOSE, then config 5's reads on a 3 Gbp text with 64- and 32-bit intervals
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c5occ
O=gpurun_out/c5occ
A="--config 5 --steps 3 --warmup 1 --cpu-sample 0 --parity-sample 2000 --dropin 0"
for v in "g3_i64:--genome 3000000005 --intervals 64" "g3_i32:--genome 3000000005 --intervals 32" ${EXTRA:-}; do
  n=${v%%:*}; x=${v#*:}
  HSA_VERBOSE=1 timeout -k 10 400 python -u bench.py $A $x > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 2; }
  echo "$n: $(grep -h 'launch:' $O/$n.err | sort | uniq -c | head -3 | tr '\n' ' ') | $(grep -h 'kernels\|parity:' $O/$n.err | tr '\n' ' ')"
done
echo ALLOK
