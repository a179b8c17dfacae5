#!/usr/bin/env python3
"""Per-kernel launch durations from a rocprofv3 --kernel-trace CSV, separating each
search kernel's full-size launches (the step's pass over the batch) from its
near-empty capacity re-runs (the BIG / HUGE passes of a batch that did not overflow
take microseconds), so the average agrees with bench.py's per-pass HIP-event timing.

usage: tools/trace_summary.py <trace dir> <out.json>
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys


def short(name):
    n = name[5:] if name.startswith("void ") else name
    return n.split("(")[0]


def main():
    src, dst = sys.argv[1], sys.argv[2]
    path = glob.glob(os.path.join(src, "*kernel_trace.csv"))[0]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {}
    for k, v in d.items():
        if not (k.startswith("k_search") or k.startswith("k_widths") or k.startswith("k_seed")):
            continue
        top = max(v)
        full = [x for x in v if x >= 0.5 * top]
        out[k] = {"launches": len(v), "full_size_launches": len(full), "full_avg_ms": round(statistics.mean(full), 4),
                  "full_min_ms": round(min(full), 4), "full_max_ms": round(max(full), 4),
                  "other_launches_avg_ms": round(statistics.mean([x for x in v if x < 0.5 * top]), 4)
                  if len(full) < len(v) else None}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
