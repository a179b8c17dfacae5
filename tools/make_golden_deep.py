#!/usr/bin/env python3
"""Golden vectors for searches deeper than the GPU's fixed-capacity passes: reads on
the repeat-rich `rep` index with options under which bwt_match_gap pushes far more
than 65 535 stack entries per read (the big pass's capacity), so the parity tests
exercise the huge pass (reused slots up to max_entries + 16 live entries).  Recorded
from the reference compiled here (oracle/_ref/ref_probe, tools/make_golden.py's
recipe) on the committed tests/golden/index/rep.fa.index.* files.

usage: python tools/make_golden_deep.py   (needs oracle/_ref built: make -C oracle)"""
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import make_golden as mg  # noqa: E402
from hsa_amd import synth  # noqa: E402


def main():
    prefix = os.path.join(ROOT, "tests", "golden", "index", "rep.fa")
    gr = mg.repeat_genome(50001, 11)
    recr = synth.record_layout(50001, 1)
    r, _ = synth.make_reads(gr, recr, 60, 100, 31, max_mm=4)
    cases = [("rep_deep_n6o2N", list(r), ["-n", "6", "-o", "2", "-N"]),
             ("rep_deep_n6o2m", list(r), ["-n", "6", "-o", "2", "-m", "30000"])]
    # more stack buckets than 128 (n_stacks = aln_score(7, 3, 21) = 138): the score
    # table past the first 128 scores
    g = synth.genome_codes(200003, 7)
    rec = synth.record_layout(200003, 3)
    rt, _ = synth.make_reads(g, rec, 200, 100, 41, indel=True, max_mm_indel=2)
    tiny_cases = [("tiny_opts_bigstack", list(rt), ["-n", "6", "-o", "2", "-e", "20"])]
    man_path = os.path.join(mg.GOLD, "manifest_tiny.json")
    manifest = json.load(open(man_path))
    with tempfile.TemporaryDirectory() as work:
        for name, seqs, args in cases:
            n_aln, flags, hits, secs = mg.run_aln(prefix, seqs, args, work)
            mg.save_case(name, "rep", seqs, args, 100000, n_aln, flags, hits)
            manifest[name] = {"index": "rep", "args": args, "batch": 100000, "n": len(seqs),
                              "sha256": mg.hits_digest(n_aln, flags, hits), "ref_seconds": secs}
            print(f"  {name}: reference {secs:.2f} s, max hits per read {int(n_aln.max())}")
        tprefix = os.path.join(ROOT, "tests", "golden", "index", "tiny.fa")
        for name, seqs, args in tiny_cases:
            n_aln, flags, hits, secs = mg.run_aln(tprefix, seqs, args, work)
            mg.save_case(name, "tiny", seqs, args, 100000, n_aln, flags, hits)
            manifest[name] = {"index": "tiny", "args": args, "batch": 100000, "n": len(seqs),
                              "sha256": mg.hits_digest(n_aln, flags, hits), "ref_seconds": secs}
            print(f"  {name}: reference {secs:.2f} s")
    with open(man_path, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
