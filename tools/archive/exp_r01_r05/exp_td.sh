# TA/TD/TCP cost per request: the gather probe's shapes vs k_search (one PMC pass each)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C="TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_VMEM_WR TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $R/gpurun_out/td_probe -o run -- $R/tools/gather_probe sparse > $R/gpurun_out/td_probe.log 2>&1 || { echo probe failed; exit 2; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $C --kernel-include-regex "k_search|k_widths" --output-format csv -d $R/gpurun_out/td_bench -o run -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 0 > $R/gpurun_out/td_bench.log 2>&1 || { echo bench failed; exit 3; }
echo done
