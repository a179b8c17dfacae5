# TA / TD / TCP (vector L1) counters of k_search (diagnostic)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 0"
p() { n=$1; shift; timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex k_search --output-format csv -d $R/gpurun_out/$n -o run -- python3 $B > $R/gpurun_out/$n.log 2>&1 || echo "$n failed"; }
p ta1 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
p td1 TD_TD_BUSY_sum TD_TC_STALL_sum
p tcp1 TCP_TCP_LATENCY_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
p tcp2 TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_READ_sum
echo done
