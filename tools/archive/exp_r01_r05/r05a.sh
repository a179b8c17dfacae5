#!/bin/bash
# Round 5, first call: the select-tree A/B (configs 2, 3) and the diagnostic counters of config 3.
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
nvidia-smi >/dev/null 2>&1; rocm-smi --showmeminfo vram > gpurun_out/r05a_smi.log 2>&1
bash tools/exp/r04_pick4_ab.sh > gpurun_out/r05a_ab.log 2>&1 || exit 1
cat gpurun_out/r05a_ab.log
CONFIGS=3 bash tools/exp/r04_diag_c3.sh > gpurun_out/r05a_diag.log 2>&1 || exit 2
cat gpurun_out/r05a_diag.log
