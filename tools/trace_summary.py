#!/usr/bin/env python3
"""Per-kernel launch durations from a rocprofv3 --kernel-trace CSV, separating each
search kernel's full-size launches (the step's pass over the batch) from its
near-empty capacity re-runs (the BIG / HUGE passes of a batch that did not overflow
take microseconds), so the average agrees with bench.py's per-pass HIP-event timing.
With bench.py's two handles, the timed steps' launches overlap those of the other
handle; the roofline steps after them run alone.  Full-size launches are split into
those two groups (a launch overlaps when any other full-size k_search / k_widths launch
runs during it), and serialized_avg_ms is the figure bench.py's roofline reports.

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
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d[short(r["Kernel_Name"])].append((t0, t1, (t1 - t0) / 1e6))
    heavy = {k: v for k, v in d.items() if k.startswith("k_search") or k.startswith("k_widths") or k.startswith("k_seed")}
    full_iv = {}
    for k, v in heavy.items():
        top = max(x[2] for x in v)
        full_iv[k] = [x for x in v if x[2] >= 0.2 * top]
    every = [(k, x) for k, v in full_iv.items() for x in v]

    def overlaps(k, x):
        return any((k2, y) != (k, x) and y[0] < x[1] and x[0] < y[1] for k2, y in every)
    out = {}
    for k, v in heavy.items():
        full = full_iv[k]
        ser = [x[2] for x in full if not overlaps(k, x)]
        ovl = [x[2] for x in full if overlaps(k, x)]
        rest = [x[2] for x in v if x not in full]
        out[k] = {"launches": len(v), "full_size_launches": len(full),
                  "full_avg_ms": round(statistics.mean(x[2] for x in full), 4),
                  "full_min_ms": round(min(x[2] for x in full), 4), "full_max_ms": round(max(x[2] for x in full), 4),
                  "serialized_launches": len(ser), "serialized_avg_ms": round(statistics.mean(ser), 4) if ser else None,
                  "overlapped_launches": len(ovl), "overlapped_avg_ms": round(statistics.mean(ovl), 4) if ovl else None,
                  "other_launches_avg_ms": round(statistics.mean(rest), 4) if rest else None}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
