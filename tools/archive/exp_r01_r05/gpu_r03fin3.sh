# Round 3 closing runs on the two-handle build (2 of 2): configs 3, 4, 5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "3 10 1" "5 20 2" "4 5 1"; do
  set -- $cfg
  timeout -k 10 600 python -u bench.py --config $1 --steps $2 --warmup $3 > gpurun_out/fin3_c$1.json 2> gpurun_out/fin3_c$1.err \
      || { tail -30 gpurun_out/fin3_c$1.err; exit 2; }
  grep -v "per-step device ms" gpurun_out/fin3_c$1.err | tail -6
done
