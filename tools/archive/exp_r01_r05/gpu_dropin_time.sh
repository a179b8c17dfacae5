set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HSA_VERBOSE=1
mkdir -p gpurun_out/dropin
timeout -k 10 300 python -u tools/dropin_time.py > gpurun_out/dropin/time.log 2>&1 || { echo failed; tail -20 gpurun_out/dropin/time.log; exit 1; }
grep -E "dropin_time|\[hsa\] (search|cal_sa)" gpurun_out/dropin/time.log | tail -12
echo ALLOK
