#!/usr/bin/env python3
"""Summarise a tools/profile_run.sh output directory into one JSON (committed
under profiles/) -- the per-launch HBM traffic of k_search that bench.py reports
as roofline.traffic, and the SQ/TCC ratios.

FETCH_SIZE is in KiB.  Calibration (MI355X_MICROARCH.md, HBM section: access
widths other than 16 B/lane streaming are uncalibrated): membench's k_indep
issues a known number of random 64-byte block loads per dispatch; the ratio
FETCH_SIZE*1024 / known bytes on that pattern is applied to k_search.

usage: tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<round>_pmc_summary.json [step] [--cal DIR]

--cal DIR takes the FETCH_SIZE calibration pass (pmc_membench) from another profile
directory of the same box run; SQ / TCC passes are summarised when present.

With "step", a step's traffic sums every kernel instantiation of the step, each as
all its dispatches (overflow re-runs included) over its full-size launches: config
4's step launches k_search twice (main path, splice seeds) plus the re-runs.
"""
import collections
import csv
import json
import os
import statistics
import sys


STEP_KERNELS = ("k_widths", "k_widths_reads", "k_search", "k_seed_prep", "k_widths_import", "k_widths_export",
                "k_sp_prep", "k_pf_rows", "k_pf_seeds", "k_pf_anchors", "k_splice")


def counters(d, kernel, every=False):
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    names = {}
    for r in rows:
        name = r["Kernel_Name"]
        if name.startswith("void "):
            name = name[5:]
        # the kernel's own name only: k_widths must not match k_widths_import / _export
        if not (name.startswith(kernel) and (kernel.endswith(">") or name[len(kernel):len(kernel) + 1] in ("<", "("))):
            continue
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    # one step = one full-batch launch; the overflow re-run launches of the same kernel
    # (an empty or near-empty list, tens of microseconds) are not the step's launch
    if every:
        return agg, dur, names
    if dur:
        top = max(dur.values())
        keep = [d for d, ms in dur.items() if ms >= 0.5 * top]
        agg = {d: agg[d] for d in keep}
        dur = {d: dur[d] for d in keep}
    return agg, dur


def med(agg, name):
    return statistics.median(v[name] for v in agg.values())


def main():
    args = sys.argv[1:]
    cal_dir = None
    if "--cal" in args:
        i = args.index("--cal")
        cal_dir = args[i + 1]
        del args[i:i + 2]
    src, dst = args[0], args[1]
    out = {"source": src}
    # calibration on membench k_indep<1>: 1024 workgroups x 256 lanes x 2000 iterations x 64 B
    mb, _ = counters(os.path.join(cal_dir or src, "pmc_membench"), "k_indep<1>")
    known = 256 * 16 // 4 * 256 * 2000 * 64
    cal = med(mb, "FETCH_SIZE") * 1024 / known
    out["fetch_calibration_random64"] = round(cal, 4)
    launches = len(args) > 2 and args[2] == "step"
    if launches:
        out["per_kernel"] = {}
        # steps: the full-size launches (>= half the longest) of the longest-running
        # k_search instantiation, the step's main pass; every kernel's dispatches (overflow
        # re-runs, the lazy widths' two launches, the forward pass) are summed over them
        f0, dur0, names0 = counters(os.path.join(src, "pmc_fetch"), "k_search", every=True)
        main = max(set(names0.values()), key=lambda nm: sum(dur0[d] for d in names0 if names0[d] == nm))
        ds0 = [d for d in names0 if names0[d] == main]
        top0 = max(dur0[d] for d in ds0)
        nsteps = sum(1 for d in ds0 if dur0[d] >= 0.5 * top0)
        out["steps"] = nsteps
        for k in STEP_KERNELS:
            f, dur, names = counters(os.path.join(src, "pmc_fetch"), k, every=True)
            w, _, _ = counters(os.path.join(src, "pmc_write"), k, every=True)
            if not f:
                continue
            fb = sum(v["FETCH_SIZE"] for v in f.values()) * 1024 / cal / nsteps
            wb = sum(v["WRITE_SIZE"] for v in w.values()) * 1024 / nsteps
            ms = sum(dur.values()) / nsteps
            out["per_kernel"][k] = {"fetch_bytes": fb, "write_bytes": wb, "ms_per_step_pmc_pass": ms}
    else:
        # one step = k_widths + k_search launches: per-kernel medians, summed
        out["per_kernel"] = {}
    for k in (() if launches else ("k_widths", "k_widths_reads", "k_search")):
        f, dur = counters(os.path.join(src, "pmc_fetch"), k)
        w, _ = counters(os.path.join(src, "pmc_write"), k)
        if not f:
            continue
        out["per_kernel"][k] = {"fetch_bytes": med(f, "FETCH_SIZE") * 1024 / cal,
                                "write_bytes": med(w, "WRITE_SIZE") * 1024,
                                "ms_median_pmc_pass": statistics.median(dur.values())}
    out["fetch_bytes_per_launch"] = sum(v["fetch_bytes"] for v in out["per_kernel"].values())
    out["write_bytes_per_launch"] = sum(v["write_bytes"] for v in out["per_kernel"].values())
    if os.path.isdir(os.path.join(src, "pmc_sq")):
        sq, _ = counters(os.path.join(src, "pmc_sq"), "k_search")
        wc = med(sq, "SQ_WAVE_CYCLES")
        out["sq"] = {"wait_any_frac": med(sq, "SQ_WAIT_ANY") / wc,
                     "active_inst_any_frac": med(sq, "SQ_ACTIVE_INST_ANY") / wc,
                     "active_valu_frac": med(sq, "SQ_ACTIVE_INST_VALU") / wc,
                     "vmem_rd_wave_insts": med(sq, "SQ_INSTS_VMEM_RD"),
                     "waves": med(sq, "SQ_WAVES"),
                     "grbm_gui_active_per_xcd": med(sq, "GRBM_GUI_ACTIVE") / 8}
    if os.path.isdir(os.path.join(src, "pmc_tcc")):
        tcc, _ = counters(os.path.join(src, "pmc_tcc"), "k_search")
        h, m = med(tcc, "TCC_HIT_sum"), med(tcc, "TCC_MISS_sum")
        out["tcc"] = {"hit_rate": h / (h + m), "ea_rdreq": med(tcc, "TCC_EA0_RDREQ_sum")}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
