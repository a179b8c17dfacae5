# round 2 profiles: config 2 and config 3 (kernel trace + stats, PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BENCH_ARGS="--dropin 0" bash tools/profile_run.sh r02_c2 || { echo prof c2 failed; exit 1; }
BENCH_ARGS="--config 3 --dropin 0 --steps 3" PASSES="fetch write tcc" bash tools/profile_run.sh r02_c3 || { echo prof c3 failed; exit 2; }
echo ALLOK
