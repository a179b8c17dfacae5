# hsa_index_clone: the concurrent-handle parity test, then the bench with --streams 2
# (default) on configs 2, 3, 4, 5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hg19.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03z_pytest.log 2>&1 || { tail -40 gpurun_out/r03z_pytest.log; exit 1; }
tail -5 gpurun_out/r03z_pytest.log
Q="--dropin 0 --ref-sample 0 --cpu-sample 0 --parity-sample 100000"
for cfg in "2 60" "3 8" "4 20" "5 30"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --config $1 --steps $2 --warmup 3 $Q > gpurun_out/r03z_c$1.json 2> gpurun_out/r03z_c$1.err \
      || { tail -30 gpurun_out/r03z_c$1.err; exit 2; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['k_search_ms'], r['frac'], r['k_widths']['ms'], r['step'], d.get('parity_sample',{}).get('mismatching_reads'))" gpurun_out/r03z_c$1.json
done
