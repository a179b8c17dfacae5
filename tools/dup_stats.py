"""Experiment (CPU, test infrastructure): how much of a bwt_match_gap search (bwtgap.c:
118-331) re-expands a node it already expanded -- the same (i, k, l, rev_k, state) with
the same counts (exact repeat) or with counts >= an earlier expansion's (dominated) --
split by searches that end with and without hits.  For a search without hits, a repeated
or dominated expansion adds nothing (the order-independence argument of DESIGN.md,
round-5 verdict item 2), so this bounds what dominance pruning could save.

Uses the restatement built with -DOR_DUP_STATS (oracle/liboracle_dup.so) on an index
built by the reference's own `HSA index` (oracle/_ref/HSA) over a synthetic genome.

    python tools/dup_stats.py --genome 20000005 --reads 2000 --out profiles/r06_dup_stats.json
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome", type=int, default=20_000_005)
    ap.add_argument("--reads", type=int, default=2000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle_dup.so"], check=True, capture_output=True)
    import oracle_ctypes
    oracle_ctypes.LIB = os.path.join(ROOT, "oracle", "liboracle_dup.so")
    from hsa_amd import index_io, synth
    from oracle_ctypes import Opt, OracleIndex, default_opt, lib
    L = lib()
    L.or_dup_stats.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    d = tempfile.mkdtemp(prefix="dup_")
    fa = os.path.join(d, "g.fa")
    codes = synth.genome_codes(a.genome, 31)
    recs = synth.record_layout(a.genome, 4)
    synth.write_fasta(fa, codes, recs)
    t0 = time.time()
    subprocess.run([os.path.join(ROOT, "oracle", "_ref", "HSA"), "index", fa], check=True, capture_output=True, cwd=d)
    print(f"[dup] index of {a.genome} bp in {time.time() - t0:.0f} s", flush=True)
    fwd, rev = index_io.read_index(fa)
    ox = OracleIndex(fwd, rev)
    workloads = {
        "config3_indel_100bp": (synth.make_reads(codes, recs, a.reads, 100, 61, indel=True, max_mm_indel=2)[0], 1),
        "config4_spliced_150bp": (synth.make_spliced_reads(codes, recs, a.reads, 150, 71)[0], 1),
        "config2_subst_100bp": (synth.make_reads(codes, recs, a.reads, 100, 51, max_mm=4)[0], 0),
    }
    out = {"genome_bp": a.genome, "reads": a.reads, "options": "-n 4 -o 0|1 (steady state: GAPE cleared)",
           "note": "expansions of bwt_match_gap searches (main path, both strands searched as the reference does); "
                   "exact = same node and counts as an earlier expansion of the same search; dominated = same node, "
                   "counts >= an earlier one's", "workloads": {}}
    buf = (C.c_uint64 * 6)()
    for name, (reads, gapo) in workloads.items():
        od = default_opt()
        od.update(max_diff=4, fnr=-1.0, max_gapo=gapo, mode=od["mode"] & ~0x01)
        L.or_dup_stats(buf, 1)
        t0 = time.time()
        ox.cal_sa_reg_gap(np.full(len(reads), reads.shape[1], np.uint32), reads.reshape(-1), Opt.from_dict(od))
        L.or_dup_stats(buf, 0)
        v = [int(x) for x in buf]
        rec = {"with_hits": {"expansions": v[0], "exact_repeats": v[1], "dominated": v[2]},
               "without_hits": {"expansions": v[3], "exact_repeats": v[4], "dominated": v[5]},
               "seconds": round(time.time() - t0, 1)}
        for k in ("with_hits", "without_hits"):
            e = rec[k]
            e["repeat_or_dominated_frac"] = round((e["exact_repeats"] + e["dominated"]) / max(e["expansions"], 1), 4)
        out["workloads"][name] = rec
        print(f"[dup] {name}: {json.dumps(rec)}", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
