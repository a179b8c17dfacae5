# SQ instruction-mix counters of k_search (diagnostic; two passes)
set -o pipefail
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 0"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SMEM --kernel-include-regex k_search --output-format csv -d $R/gpurun_out/sq1 -o run -- python3 $B > $R/gpurun_out/sq1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex k_search --output-format csv -d $R/gpurun_out/sq2 -o run -- python3 $B > $R/gpurun_out/sq2.log 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_FLAT SQ_IFETCH --kernel-include-regex k_search --output-format csv -d $R/gpurun_out/sq3 -o run -- python3 $B > $R/gpurun_out/sq3.log 2>&1 || echo "pass 3 failed"
echo done
