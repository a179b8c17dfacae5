# A/B: (1) the host-array drop-in split over 1, 2, 3 handles of one index on one GPU;
# (2) lazy forward rows for 100 bp reads once two handles overlap the launches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 2 3; do
  timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --parity-sample 0 --cpu-sample 0 --ref-sample 0 --dropin-slots $k \
      > gpurun_out/slots$k.json 2> gpurun_out/slots$k.err || { tail -30 gpurun_out/slots$k.err; exit 1; }
  grep "drop-in" gpurun_out/slots$k.err
done
for l in 0 1 0 1; do
  HSA_LAZY=$l timeout -k 10 400 python -u bench.py --steps 60 --warmup 3 --dropin 0 --ref-sample 0 --cpu-sample 0 --parity-sample 100000 \
      > gpurun_out/lazy2_$l.json 2> gpurun_out/lazy2_$l.err || { tail -30 gpurun_out/lazy2_$l.err; exit 2; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['k_search_ms'], r['k_widths']['ms'], d['parity_sample']['mismatching_reads'])" gpurun_out/lazy2_$l.json
done
for sw in "2 16" "3 8" "3 16" "2 16" "3 8"; do
  set -- $sw
  f=gpurun_out/sw2_s$1_w$2
  timeout -k 10 400 python -u bench.py --steps 60 --warmup 3 --streams $1 --waves $2 --dropin 0 --ref-sample 0 --cpu-sample 0 --parity-sample 100000 \
      > $f.json 2> $f.err || { tail -30 $f.err; exit 3; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['k_search_ms'], r['k_widths']['ms'], d['parity_sample']['mismatching_reads'])" $f.json
done
