# Three handles by default (dropped to two where a gapped pool does not fit): configs 3,
# 5, 4 quick, then config 2 at 200 steps with every leg
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "3 8 1 100000" "5 20 2 -1" "4 5 1 -1"; do
  set -- $cfg
  timeout -k 10 500 python -u bench.py --config $1 --steps $2 --warmup $3 --parity-sample $4 --dropin 0 --ref-sample 0 --cpu-sample 0 \
      > gpurun_out/fin5_c$1.json 2> gpurun_out/fin5_c$1.err || { tail -30 gpurun_out/fin5_c$1.err; exit 2; }
  grep "dropped" gpurun_out/fin5_c$1.err || true
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], d['config']['streams'], r['k_search_ms'], r['k_widths']['ms'], d.get('parity_full', d.get('parity_sample'))['mismatching_reads'])" gpurun_out/fin5_c$1.json
done
timeout -k 10 900 python -u bench.py --steps 200 --warmup 5 > gpurun_out/fin5_bench.json 2> gpurun_out/fin5_bench.err \
    || { tail -40 gpurun_out/fin5_bench.err; exit 3; }
grep -v "per-step device ms" gpurun_out/fin5_bench.err | tail -12
