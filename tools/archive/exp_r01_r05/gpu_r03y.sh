# A/B: consecutive steps alternating over S handles of the index (hsa_index_clone), S = 1, 2, 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--dropin 0 --ref-sample 0 --cpu-sample 0 --parity-sample 100000"
for cfg in "2 60" "3 8" "5 30"; do
  set -- $cfg
  for S in 1 2 3; do
    timeout -k 10 400 python -u bench.py --config $1 --steps $2 --warmup 3 --streams $S $Q > gpurun_out/r03y_c$1_s$S.json 2> gpurun_out/r03y_c$1_s$S.err \
        || { tail -30 gpurun_out/r03y_c$1_s$S.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['k_search_ms'], r['k_widths']['ms'], d.get('parity_sample'))" gpurun_out/r03y_c$1_s$S.json
  done
done
