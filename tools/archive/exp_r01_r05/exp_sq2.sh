# instruction mix of k_search / k_widths (config 2): two SQ passes
set -o pipefail
cd /tmp
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="$R/bench.py --steps 2 --warmup 1 --cpu-sample 0 --parity-sample 0 $BENCH_ARGS"
p() { n=$1; shift; timeout -s KILL 200 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex "k_search|k_widths" --output-format csv -d $R/gpurun_out/${PFX:-}$n -o run -- python3 $B > $R/gpurun_out/${PFX:-}$n.log 2>&1 || { echo "$n failed"; exit 2; }; }
p sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY
p sqb SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
p sqc SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT SQ_ACCUM_PREV_HIRES GRBM_GUI_ACTIVE
echo done
