# --streams 2 (default) on configs 5 and 4 (config 4 with its default 4 000-read parity sample)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "5 30 100000" "4 10 -1"; do
  set -- $cfg
  timeout -k 10 500 python -u bench.py --config $1 --steps $2 --warmup 3 --dropin 0 --ref-sample 0 --cpu-sample 0 --parity-sample $3 \
      > gpurun_out/r03z2_c$1.json 2> gpurun_out/r03z2_c$1.err || { tail -30 gpurun_out/r03z2_c$1.err; exit 2; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['k_search_ms'], r['frac'], r['k_widths']['ms'], r['step'], d.get('parity_sample',{}).get('mismatching_reads'))" gpurun_out/r03z2_c$1.json
done
