# A/B: handles (--streams) x resident waves per CU of each launch (--waves): two
# half-chip launches in flight against two full-chip ones
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--dropin 0 --ref-sample 0 --cpu-sample 0 --parity-sample 100000"
for cfg in "2 60 2 16" "2 60 2 8" "2 60 3 8" "2 60 4 8" "2 60 4 4" "3 8 2 16" "3 8 2 8" "3 8 4 8"; do
  set -- $cfg
  f=gpurun_out/r03sw_c$1_s$3_w$4
  timeout -k 10 400 python -u bench.py --config $1 --steps $2 --warmup 3 --streams $3 --waves $4 $Q > $f.json 2> $f.err \
      || { tail -30 $f.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['k_search_ms'], r['k_widths']['ms'], d['parity_sample']['mismatching_reads'])" $f.json
done
