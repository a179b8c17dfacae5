#!/bin/bash
# Profiling recipe run on the GPU box (DESIGN.md "Measurement"):
#   kernel trace + stats, then one PMC pass per counter group (separate runs, no
#   tracing domains besides --kernel-trace), and a FETCH_SIZE calibration pass on
#   membench's random 64-byte gather (known byte count).
# usage: tools/profile_run.sh <tag>      outputs under gpurun_out/prof_<tag>/
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="$R/bench.py --steps 5 --warmup 1 --streams 1 --cpu-sample 0 --parity-sample 0 --ref-sample 0 --dropin 0 --e2e-reads 0 --copies 0 $BENCH_ARGS"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.json 2> $OUT/trace.err || exit 11
pmc() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc "$@" --kernel-include-regex "${PMC_REGEX:-k_search|k_widths}" --output-format csv -d $OUT/pmc_$n -o run -- python3 $BENCH > $OUT/pmc_$n.json 2> $OUT/pmc_$n.err || exit 12
}
# PASSES selects the counter passes (default: all)
PASSES=${PASSES:-"fetch write sq tcc membench"}
for p in $PASSES; do
  case $p in
    fetch) pmc fetch FETCH_SIZE ;;
    write) pmc write WRITE_SIZE ;;
    sq) pmc sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE ;;
    tcc) pmc tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum ;;
    membench) timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex k_indep --output-format csv -d $OUT/pmc_membench -o run -- $R/tools/membench 2147483648 16 > $OUT/pmc_membench.log 2>&1 || exit 13 ;;
  esac
done
echo done
