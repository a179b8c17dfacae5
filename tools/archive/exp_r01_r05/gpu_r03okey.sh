# A/B: cost key with the last segment's length (HSA_ORDER_KEY=1) against the final bid alone
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--dropin 0 --ref-sample 0 --cpu-sample 0 --parity-sample 100000"
for run in "2 60 0" "2 60 1" "2 60 0" "2 60 1" "3 8 0" "3 8 1" "5 20 0" "5 20 1"; do
  set -- $run
  f=gpurun_out/okey_c$1_k$3_$RANDOM
  HSA_ORDER_KEY=$3 timeout -k 10 400 python -u bench.py --config $1 --steps $2 --warmup 3 $Q > $f.json 2> $f.err || { tail -30 $f.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['k_search_ms'], r['k_widths']['ms'], d['parity_sample']['mismatching_reads'])" $f.json
done
