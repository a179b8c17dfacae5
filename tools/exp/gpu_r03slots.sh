# A/B: the host-array drop-in split over 1, 2, 3 handles of one index on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 2 3; do
  timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --parity-sample 0 --cpu-sample 0 --ref-sample 0 --dropin-slots $k \
      > gpurun_out/slots$k.json 2> gpurun_out/slots$k.err || { tail -30 gpurun_out/slots$k.err; exit 1; }
  grep "drop-in" gpurun_out/slots$k.err
done
