#!/bin/bash
# Round-6 profiles of the shipped build (run on the GPU box from the repo root):
#   config 2 and config 5: kernel trace + stats, then FETCH_SIZE, WRITE_SIZE, SQ and TCC
#   passes and the FETCH_SIZE calibration on membench (tools/profile_run.sh), each a
#   run of its own.  The summaries are made afterwards in the build container:
#     python tools/pmc_summary.py gpurun_out/prof_r06_config2 profiles/r06_pmc_summary_config2.json
#     python tools/pmc_summary.py gpurun_out/prof_r06_config5 profiles/r06_pmc_summary_config5.json --cal gpurun_out/prof_r06_config2
#     python tools/trace_summary.py gpurun_out/prof_r06_config{2,5}/trace ... (profiles/r06_rocprof_summary_config*.json)
set -e
export TMPDIR=/tmp
PASSES="fetch write sq tcc membench" BENCH_ARGS="--config 2" timeout -k 10 560 bash tools/profile_run.sh r06_config2
PASSES="fetch write tcc" BENCH_ARGS="--config 5" timeout -k 10 600 bash tools/profile_run.sh r06_config5
