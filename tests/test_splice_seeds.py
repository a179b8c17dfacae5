"""The batched splice seeds (hsa_amd/splice.py) reproduce exactly the seed calls the
reference's bwt_splice_match makes (bwtgap.c:797-812): for the splice read set, the
six seeds of every fallback read are built with oracle widths, and every aliased-width
call recorded from the compiled reference (tests/golden/mgcap_default.npz) must be
among them -- same strand, length, sequence, widths, option block and stack -- with
the same answer from the restated search."""
import gzip
import os

import numpy as np

from golden_io import GOLD, INDEX, load_mgcap
from hsa_amd import index_io, splice
from oracle_ctypes import Opt, OracleIndex, default_opt, lib as oracle_lib

NT4 = np.full(256, 4, np.uint8)
for i, ch in enumerate(b"ACGT"):
    NT4[ch] = i
    NT4[ch + 32] = i


def read_fastq(path):
    lines = gzip.open(path).read().split(b"\n")
    seqs = [NT4[np.frombuffer(lines[i + 1], np.uint8)] for i in range(0, len(lines) - 3, 4)]
    return np.array([len(s) for s in seqs], np.uint32), np.concatenate(seqs)


def test_seed_calls_cover_the_reference_calls():
    import json
    man = json.load(open(os.path.join(GOLD, "manifest_dropin.json")))
    lens, codes = read_fastq(os.path.join(GOLD, man["splice_reads"]))
    ox = OracleIndex(*index_io.read_index(INDEX["tiny"]))
    opt = default_opt()
    n_aln, flags, _, _ = ox.cal_sa_reg_gap(lens, codes, Opt.from_dict(opt))
    fallback = np.flatnonzero(flags & 1)
    assert len(fallback) > 100
    # local_opt of the batch (bwtaln.c:254, :273-276)
    local = dict(default_opt())
    local["max_diff"] = oracle_lib().or_cal_maxdiff(int(lens.max()), 0.02, local["fnr"])
    local["max_gapo"] = min(local["max_gapo"], local["max_diff"])

    def width_fn(wl, wc):
        out, o = [], 0
        for L in wl:
            out.append(ox.cal_width(wc[o:o + int(L)]).reshape(-1))
            o += int(L)
        return np.concatenate(out).astype(np.uint32)

    b = splice.seed_calls(lens, codes, fallback, local, width_fn)
    so = b["opt"]
    n_stacks = splice.n_stacks_of(local)
    made = {}
    for c in b["calls"]:
        o = dict(so, seed_len=int(c["len"]))
        key = (int(c["strand"]), int(c["len"]), b["codes"][c["off"]:c["off"] + c["len"]].tobytes(),
               b["widths"][c["wb_off"]:c["wb_off"] + c["len"] + 1].tobytes(), bytes(Opt.from_dict(o)), n_stacks)
        made[key] = c
    rec = [c for c in load_mgcap("mgcap_default") if c["seed"] == 2]
    assert len(rec) > 1000
    missing, bad = 0, 0
    for c in rec:
        key = (c["strand"], c["len"], c["seq"].tobytes(), c["wb"].tobytes(), c["opt"].tobytes(), c["n_stacks"])
        if key not in made:
            missing += 1
            continue
        hits, w = ox.match_gap(Opt.from_buffer_copy(c["opt"].tobytes()), n_stacks, c["seq"], c["strand"], c["wb"], 2)
        bad += not (np.array_equal(hits, c["hits"]) and np.array_equal(w, c["wo"]))
    assert missing == 0 and bad == 0, (missing, bad, len(rec))


def test_fixed_length_layout_equals_general():
    """seed_calls_fixed (the bench's vectorised builder) lays out the same calls."""
    rng = np.random.default_rng(3)
    reads = rng.integers(0, 4, (7, 152), dtype=np.uint8)
    reads[2, 10] = 4
    local = dict(default_opt(), max_diff=4, max_gapo=1)

    def width_fn(wl, wc):   # a stand-in: any deterministic function of the sequences
        out, o = [], 0
        for L in wl:
            s = wc[o:o + int(L)].astype(np.uint32)
            out.append(np.stack([np.concatenate([s, [0]]), np.arange(L + 1, dtype=np.uint32)], 1).reshape(-1))
            o += int(L)
        return np.concatenate(out)

    a = splice.seed_calls(np.full(7, 152, np.uint32), reads.reshape(-1), np.arange(7), local, width_fn)
    f = splice.seed_calls_fixed(reads, local, width_fn)
    assert np.array_equal(a["calls"], f["calls"])
    assert np.array_equal(a["codes"], f["codes"])
    assert np.array_equal(a["widths"], f["widths"])
