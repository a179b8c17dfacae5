# Kernel trace of the bench's default command (two handles: overlapped timed steps, then
# the serialized roofline steps), summarized per kernel and per group
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/trace_default
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/trace_default/trace -o run -- \
    python3 $R/bench.py --steps 10 --warmup 2 --cpu-sample 0 --parity-sample 0 --ref-sample 0 --dropin 0 \
    > $R/gpurun_out/trace_default/bench.json 2> $R/gpurun_out/trace_default/bench.err || { tail -20 $R/gpurun_out/trace_default/bench.err; exit 1; }
cd $R
python3 tools/trace_summary.py gpurun_out/trace_default/trace gpurun_out/trace_default/summary.json > /dev/null
python3 -c "import json; s=json.load(open('gpurun_out/trace_default/summary.json')); print({k: (v['serialized_avg_ms'], v['overlapped_avg_ms'], v['serialized_launches'], v['overlapped_launches']) for k, v in s.items()}); d=json.load(open('gpurun_out/trace_default/bench.json')); print(d['value'], d['roofline']['k_search_ms'], d['roofline']['k_widths']['ms'])"
