#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the COMPILED REFERENCE.

Test infrastructure.  Runs in the build container only (it needs
/root/reference through oracle/_ref, built by `make -C oracle -f ref.mk`).
Every fixture is data: synthetic inputs plus the reference's outputs on them.

    python tools/make_golden.py            # tiny fixtures (committed)
    python tools/make_golden.py --ecoli    # E.coli-sized digests (committed)
    python tools/make_golden.py --dropin   # FASTQ + reference SAM for the drop-in test
    python tools/make_golden.py --sa       # SA -> position golden values (R11)
    python tools/make_golden.py --limits   # reads / options past the fast kernel's layouts
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hsa_amd import synth  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref")
GOLD = os.path.join(ROOT, "tests", "golden")
INDEX_EXT = ["bwt", "fmv", "rev.bwt", "rev.fmv", "sa", "pac", "rev.pac", "ann"]


def sh(*args, **kw):
    return subprocess.run(list(args), check=True, capture_output=True, text=True, **kw)


def build_index(fa: str) -> None:
    d = os.path.dirname(fa)
    sh(os.path.join(REF, "HSA"), "index", os.path.basename(fa), cwd=d)


def run_aln(prefix: str, seqs: list[np.ndarray], args: list[str], work: str):
    rb = os.path.join(work, "reads.bin")
    ob = os.path.join(work, "out.bin")
    synth.write_reads_bin(rb, seqs)
    r = sh(os.path.join(REF, "ref_probe"), "aln", prefix, rb, ob, *args)
    secs = float(r.stdout.strip().splitlines()[-1])
    raw = open(ob, "rb").read()
    n = int(np.frombuffer(raw[4:8], dtype=np.uint32)[0])
    off = 8
    n_aln = np.zeros(n, np.int32)
    flags = np.zeros(n, np.uint32)
    hits = []
    for i in range(n):
        na, fl = np.frombuffer(raw[off:off + 8], dtype=np.int32)
        off += 8
        n_aln[i] = na
        flags[i] = fl
        if na > 0:
            hits.append(np.frombuffer(raw[off:off + 36 * na], dtype=np.uint32).reshape(na, 9))
            off += 36 * na
    hits = np.concatenate(hits) if hits else np.zeros((0, 9), np.uint32)
    return n_aln, flags, hits, secs


def pack_reads(seqs):
    lens = np.array([len(s) for s in seqs], dtype=np.uint32)
    codes = np.concatenate([np.asarray(s, np.uint8) for s in seqs]) if seqs else np.zeros(0, np.uint8)
    return lens, codes


def save_case(name, index, seqs, args, batch, n_aln, flags, hits):
    lens, codes = pack_reads(seqs)
    np.savez_compressed(os.path.join(GOLD, name + ".npz"), lens=lens, codes=codes,
                        n_aln=n_aln, flags=flags, hits=hits,
                        args=np.array(" ".join(args)), batch=np.int64(batch),
                        index=np.array(index))
    print(f"{name}: {len(seqs)} reads, {int((n_aln > 0).sum())} with hits, "
          f"{hits.shape[0]} hits, {int(flags.sum())} splice calls")


def hits_digest(n_aln, flags, hits) -> str:
    """Digest of the main-path result: splice-fallback flags, and n_aln + hit words
    of every read that did NOT go to bwt_splice_match (splice hits are out of scope
    for the GPU path; their reads are marked -1)."""
    h = hashlib.sha256()
    splice = (np.asarray(flags) & 1).astype(bool)
    na = np.where(splice, -1, np.asarray(n_aln, np.int32)).astype(np.int32)
    h.update(na.tobytes())
    keep = np.repeat(~splice, np.maximum(np.asarray(n_aln, np.int64), 0))
    h.update(np.ascontiguousarray(np.asarray(hits, np.uint32)[keep], np.uint32).tobytes())
    return h.hexdigest()


def repeat_genome(T: int, seed: int) -> np.ndarray:
    """A repeat-rich text: random background, tandem repeats and near-copies."""
    g = synth.genome_codes(T, seed).copy()
    rng_words = synth.genome_words(4096, seed + 1)
    bits = ((rng_words[:, None] >> (np.arange(0, 64, 2, dtype=np.uint64))) & np.uint64(3)).reshape(-1)
    bits = bits.astype(np.int64)
    p = 1000
    k = 0
    while p + 1200 < T:
        kind = k % 3
        if kind == 0:      # microsatellite (tandem unit 1-6 bp) of 60-200 bp
            u = 1 + bits[k] % 6
            unit = g[p:p + u].copy()
            n = 60 + (bits[k + 1] * 16 + bits[k + 2]) % 140
            g[p + u:p + u + n] = np.resize(unit, n)
        elif kind == 1:    # exact copy of an earlier 300 bp segment
            src = (bits[k + 3] * 997 + 31 * k) % max(p - 300, 1)
            g[p:p + 300] = g[src:src + 300]
        else:              # near-copy with 3 substitutions
            src = (bits[k + 4] * 1231 + 17 * k) % max(p - 300, 1)
            g[p:p + 300] = g[src:src + 300]
            for j in range(3):
                q = p + (bits[k + 5 + j] * 64 + bits[k + 8 + j]) % 300
                g[q] = (g[q] + 1) % 4
        p += 1500 + (bits[k + 11] * 256) % 900
        k += 1
    return g


def edge_reads(genome, records, seed):
    """Reads that hit the filters and odd branches of bwa_cal_sa_reg_gap."""
    out = []
    base, _ = synth.make_reads(genome, records, 40, 100, seed, max_mm=2)
    for i in range(40):
        r = base[i].copy()
        if i % 8 == 0:
            r[10] = 4                 # one N
        elif i % 8 == 1:
            r[5:11] = 4               # many N: skipped by the #N > max_diff filter (bwtaln.c:314)
        elif i % 8 == 2:
            r[:15] = 0                # first 15 all A (bwtaln.c:324)
        elif i % 8 == 3:
            r[:15] = 3                # first 15 all T
        elif i % 8 == 4:
            r[50] = 5                 # '-' maps to code 5 (bwaseqio.c:12)
        elif i % 8 == 5:
            r[97] = 4                 # N near the end of the read
        elif i % 8 == 6:
            r[:] = synth.genome_codes(100, seed * 31 + i)   # random: unmappable -> splice
        out.append(r)
    short, _ = synth.make_reads(genome, records, 6, 36, seed + 1, max_mm=2)
    out += [short[i] for i in range(6)]
    for L in (37, 50, 64, 75, 120, 150):
        rr, _ = synth.make_reads(genome, records, 2, L, seed + L, max_mm=3)
        out += [rr[0], rr[1]]
    return out


def tiny_cases(work):
    T, seed = 200003, 7
    g = synth.genome_codes(T, seed)
    rec = synth.record_layout(T, 3)
    fa = os.path.join(work, "tiny.fa")
    synth.write_fasta(fa, g, rec)
    build_index(fa)
    idir = os.path.join(GOLD, "index")
    os.makedirs(idir, exist_ok=True)
    for e in INDEX_EXT:
        shutil.copy(f"{fa}.index.{e}", os.path.join(idir, f"tiny.fa.index.{e}"))
    prefix = fa

    Tr = 50001
    gr = repeat_genome(Tr, 11)
    recr = synth.record_layout(Tr, 1)
    far = os.path.join(work, "rep.fa")
    synth.write_fasta(far, gr, recr)
    build_index(far)
    for e in INDEX_EXT:
        shutil.copy(f"{far}.index.{e}", os.path.join(idir, f"rep.fa.index.{e}"))

    cases = []
    r, _ = synth.make_reads(g, rec, 2000, 36, 1)
    cases.append(("tiny_exact36_n0", "tiny", list(r), ["-n", "0"], 100000))
    r, _ = synth.make_reads(g, rec, 2000, 100, 5, max_mm=4)
    cases.append(("tiny_mm100_n4o0", "tiny", list(r), ["-n", "4", "-o", "0"], 100000))
    r, _ = synth.make_reads(g, rec, 1500, 100, 6, indel=True, max_mm_indel=2)
    cases.append(("tiny_gap100_n4o1", "tiny", list(r), ["-n", "4", "-o", "1"], 100000))
    # multi-batch with unmappable reads sprinkled in: the Q2 regime switch (bwtaln.c:363)
    r, _ = synth.make_reads(g, rec, 1200, 100, 8, indel=True, max_mm_indel=2)
    seqs = list(r)
    for j in (3, 250, 611, 900):
        seqs[j] = synth.genome_codes(100, 1000 + j)
    cases.append(("tiny_gap100_n4o1_b400", "tiny", seqs, ["-n", "4", "-o", "1", "-B", "400"], 400))
    # default options (-n 0.04 => per-length max_diff, GAPE semantics) on edge reads
    seqs = edge_reads(g, rec, 21)
    cases.append(("tiny_edge_default", "tiny", seqs, [], 100000))
    cases.append(("tiny_edge_n3o1e3L", "tiny", seqs, ["-n", "3", "-o", "1", "-e", "3", "-L"], 100000))
    r, _ = synth.make_reads(g, rec, 300, 75, 9, max_mm=3)
    seqs = list(r)
    cases.append(("tiny_opts_scores", "tiny", seqs, ["-n", "3", "-o", "1", "-M", "2", "-O", "7", "-E", "3", "-d", "3", "-i", "3"], 100000))
    cases.append(("tiny_opts_seed", "tiny", seqs, ["-n", "4", "-o", "0", "-l", "20", "-k", "1"], 100000))
    cases.append(("tiny_opts_maxentries", "tiny", seqs, ["-n", "4", "-o", "1", "-m", "40"], 100000))
    # repeat-rich text: top-2 accounting, duplicate-hit suppression in tandem repeats, gap_shadow
    r, _ = synth.make_reads(gr, recr, 800, 100, 12, max_mm=3)
    cases.append(("rep_mm100_n4o1", "rep", list(r), ["-n", "4", "-o", "1"], 100000))
    r, _ = synth.make_reads(gr, recr, 600, 60, 13, indel=True, max_mm_indel=1)
    cases.append(("rep_gap60_default", "rep", list(r), [], 100000))
    cases.append(("rep_gap60_R2", "rep", list(r), ["-n", "3", "-o", "1", "-R", "2"], 100000))
    cases.append(("rep_gap60_nonstop", "rep", list(r)[:200], ["-n", "2", "-o", "1", "-N"], 100000))

    manifest = {}
    for name, idx, seqs, args, batch in cases:
        pfx = prefix if idx == "tiny" else far
        n_aln, flags, hits, secs = run_aln(pfx, seqs, args, work)
        save_case(name, idx, seqs, args, batch, n_aln, flags, hits)
        manifest[name] = {"index": idx, "args": args, "batch": batch, "n": len(seqs),
                          "sha256": hits_digest(n_aln, flags, hits), "ref_seconds": secs}

    # rank golden: BWTAllOccValue at boundary and random positions of both BWTs
    isa0 = int(np.fromfile(f"{prefix}.index.bwt", dtype=np.uint32, count=1)[0])
    risa0 = int(np.fromfile(f"{prefix}.index.rev.bwt", dtype=np.uint32, count=1)[0])
    pos = set(range(0, 300)) | set(range(T - 300, T + 2))
    for b in (isa0, risa0):
        pos |= set(range(max(b - 3, 0), b + 4))
    for m in range(0, T, 256):
        pos |= {max(m - 129, 0), max(m - 128, 0), max(m - 127, 0), max(m - 1, 0), m, m + 1, min(m + 127, T + 1), min(m + 128, T + 1)}
    rnd = (synth._u(99, 3000, 0) % np.uint64(T + 2)).astype(np.int64)
    pos |= set(int(x) for x in rnd)
    pos = np.array(sorted(p for p in pos if 0 <= p <= T + 1), dtype=np.uint32)
    pb = os.path.join(work, "pos.bin")
    with open(pb, "wb") as f:
        f.write(np.uint32(len(pos)).tobytes())
        f.write(pos.tobytes())
    sh(os.path.join(REF, "ref_probe"), "occ", prefix, pb, os.path.join(work, "occ.bin"))
    occ = np.fromfile(os.path.join(work, "occ.bin"), dtype=np.uint32).reshape(2, len(pos), 4)
    np.savez_compressed(os.path.join(GOLD, "tiny_occ.npz"), pos=pos, occ=occ)
    print(f"tiny_occ: {len(pos)} positions")

    # width golden (bwt_cal_width type 1) on a few reads incl. N
    seqs = edge_reads(g, rec, 21)[:24]
    rb = os.path.join(work, "wr.bin")
    synth.write_reads_bin(rb, seqs)
    sh(os.path.join(REF, "ref_probe"), "width", prefix, rb, os.path.join(work, "w.bin"))
    w = np.fromfile(os.path.join(work, "w.bin"), dtype=np.uint32).reshape(-1, 2)
    lens, codes = pack_reads(seqs)
    np.savez_compressed(os.path.join(GOLD, "tiny_width.npz"), lens=lens, codes=codes, width=w)
    print(f"tiny_width: {len(seqs)} reads")

    with open(os.path.join(GOLD, "manifest_tiny.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


def limits_cases(work):
    """Cases past k_search's fixed layouts, which the drop-in serves with k_search_any
    (hsa_amd/csrc/hsa_search_any.h): reads of 1 100-1 500 bp mixed with 100 bp ones,
    n_stacks 298 with 250 reachable scores (-o 2 -e 60), and 15 gap opens (-o 15).  On
    the committed tiny index; manifest_limits.json."""
    T, seed = 200003, 7
    g = synth.genome_codes(T, seed)
    rec = synth.record_layout(T, 3)
    prefix = os.path.join(GOLD, "index", "tiny.fa")
    cases = []
    seqs = []
    r, _ = synth.make_reads(g, rec, 120, 1500, 41, max_mm=6)
    seqs += list(r)
    r, _ = synth.make_reads(g, rec, 80, 1500, 42, indel=True, max_mm_indel=3)
    seqs += list(r)
    r, _ = synth.make_reads(g, rec, 60, 1100, 43, max_mm=8)
    seqs += list(r)
    r, _ = synth.make_reads(g, rec, 100, 100, 44, max_mm=4)
    seqs += list(r)
    for j in range(0, len(seqs), 37):          # an N here and there
        q = seqs[j].copy()
        q[len(q) // 3] = 4
        seqs[j] = q
    seqs += [synth.genome_codes(1300, 5000 + j) for j in range(10)]   # unmappable: splice fallback
    order = np.argsort(synth._u(45, len(seqs), 0))                     # lengths interleaved
    seqs = [seqs[i] for i in order]
    cases.append(("long1500_n8o1", seqs, ["-n", "8", "-o", "1"]))
    r, _ = synth.make_reads(g, rec, 300, 100, 46, indel=True, max_mm_indel=2)
    cases.append(("gap100_o2e60", list(r), ["-n", "4", "-o", "2", "-e", "60"]))
    r, _ = synth.make_reads(g, rec, 200, 100, 47, indel=True, max_mm_indel=1)
    cases.append(("gap100_o15", list(r), ["-n", "16", "-o", "15", "-m", "20000"]))
    manifest = {}
    for name, seqs, args in cases:
        n_aln, flags, hits, secs = run_aln(prefix, seqs, args, work)
        save_case(name, "tiny", seqs, args, 100000, n_aln, flags, hits)
        manifest[name] = {"index": "tiny", "args": args, "batch": 100000, "n": len(seqs),
                          "sha256": hits_digest(n_aln, flags, hits), "ref_seconds": secs}
    with open(os.path.join(GOLD, "manifest_limits.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


def ecoli_cases(work):
    """E.coli-sized (config 1 and two heavier flavours): digests only."""
    T, seed = 4641652, 42
    g = synth.genome_codes(T, seed)
    rec = synth.record_layout(T, 1)
    fa = os.path.join(work, "ecoli.fa")
    synth.write_fasta(fa, g, rec)
    build_index(fa)
    man = {"genome": {"T": T, "seed": seed, "records": 1}, "index_sha256": {}}
    for e in ["bwt", "fmv", "rev.bwt", "rev.fmv", "sa", "pac", "rev.pac"]:
        man["index_sha256"][e] = hashlib.sha256(open(f"{fa}.index.{e}", "rb").read()).hexdigest()
    cases = [("ecoli_exact36_n0", 10000, 36, 1, dict(), ["-n", "0"]),
             ("ecoli_mm100_n4o0", 10000, 100, 5, dict(max_mm=4), ["-n", "4", "-o", "0"]),
             ("ecoli_gap100_n4o1", 4000, 100, 6, dict(indel=True, max_mm_indel=2), ["-n", "4", "-o", "1"])]
    for name, n, L, s, kw, args in cases:
        r, _ = synth.make_reads(g, rec, n, L, s, **kw)
        n_aln, flags, hits, secs = run_aln(fa, list(r), args, work)
        man[name] = {"n": n, "L": L, "read_seed": s, "kw": kw, "args": args,
                     "sha256": hits_digest(n_aln, flags, hits), "ref_seconds": secs,
                     "reads_with_hits": int((n_aln > 0).sum()), "hits": int(hits.shape[0]),
                     "splice_calls": int(flags.sum())}
        print(name, man[name])
    with open(os.path.join(GOLD, "manifest_ecoli.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


DROPIN_ARGS = {"default": [], "n4o0": ["-n", "4", "-o", "0"]}
# splice_n4o1O120: a gap open costs 120, so n_stacks is 283 -- more score LIFOs than an
# extension slice slot holds (the splice path's extensions take hsa_extend_batch)
DROPIN_SPLICE_ARGS = {"splice_default": [], "splice_n4o1": ["-n", "4", "-o", "1"],
                      "splice_n4o1O120": ["-n", "4", "-o", "1", "-O", "120"]}


def write_fastq_mixed(path, seqs):
    import gzip
    with gzip.GzipFile(path, "wb", compresslevel=9, mtime=0) as f:
        for i, s in enumerate(seqs):
            f.write(b"@r%d\n" % i)
            f.write(bytes(b"ACGTN"[min(int(c), 4)] for c in s) + b"\n+\n")
            f.write(b"I" * len(s) + b"\n")


def dropin_cases(work):
    """Reads + the reference HSA binary's SAM output on the tiny index: the
    fixture of the drop-in test (our bwa_cal_sa_reg_gap linked into the reference's
    own HSA, oracle/ref.mk HSA_gpu), which must reproduce it byte for byte."""
    T, seed = 200003, 7
    g = synth.genome_codes(T, seed)
    rec = synth.record_layout(T, 3)
    seqs = []
    r, _ = synth.make_reads(g, rec, 500, 100, 31, max_mm=4)
    seqs += list(r)
    r, _ = synth.make_reads(g, rec, 400, 100, 32, indel=True, max_mm_indel=2)
    seqs += list(r)
    # spliced: 45-60 bp exon + the rest 200-2000 bp downstream (GT..AG not enforced)
    a, _ = synth.make_reads(g, rec, 150, 60, 33)
    for i in range(150):
        st = int(synth._u(34, 1, i)[0] % np.uint64(T - 3000))
        cut = 45 + i % 16
        intron = 200 + (i * 37) % 1800
        seqs.append(np.concatenate([g[st:st + cut], g[st + cut + intron:st + 100 + intron]]).astype(np.uint8))
    seqs += edge_reads(g, rec, 35)
    fq = os.path.join(GOLD, "dropin_reads.fq.gz")
    write_fastq_mixed(fq, seqs)
    idx = os.path.join(GOLD, "index", "tiny.fa")
    man = {"reads": os.path.basename(fq), "n": len(seqs), "index": "tiny"}
    import gzip
    for name, args in DROPIN_ARGS.items():
        r = subprocess.run([os.path.join(REF, "HSA"), "aln", *args, idx, fq], check=True, capture_output=True)
        sam = r.stdout
        out = os.path.join(GOLD, f"dropin_ref_{name}.sam.gz")
        with gzip.GzipFile(out, "wb", compresslevel=9, mtime=0) as f:
            f.write(sam)
        man[name] = {"args": args, "sam_sha256": hashlib.sha256(sam).hexdigest(), "sam_lines": sam.count(b"\n")}
        print(name, man[name])
    # the splice read set: the drop-in with OUR bwt_match_gap under the host's
    # bwt_splice_match (oracle/ref.mk HSA_gpu_mg) must reproduce these SAMs too
    fq2 = os.path.join(GOLD, "dropin_splice_reads.fq.gz")
    write_fastq_mixed(fq2, splice_reads())
    man["splice_reads"] = os.path.basename(fq2)
    for name, args in DROPIN_SPLICE_ARGS.items():
        r = subprocess.run([os.path.join(REF, "HSA"), "aln", *args, idx, fq2], check=True, capture_output=True)
        sam = r.stdout
        with gzip.GzipFile(os.path.join(GOLD, f"dropin_ref_{name}.sam.gz"), "wb", compresslevel=9, mtime=0) as f:
            f.write(sam)
        man[name] = {"args": args, "sam_sha256": hashlib.sha256(sam).hexdigest(), "sam_lines": sam.count(b"\n")}
        print(name, man[name])
    with open(os.path.join(GOLD, "manifest_dropin.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


def nrun_genome_fasta(path):
    """A 3-record genome with N-runs: runs of >= 10 N split blocks, shorter runs become
    'G' (HSP.c:275-285), so the block table has offsets ('ori') to restate."""
    recs = []
    g = synth.genome_codes(70000, 77)
    lay = [(0, 21000, [(5000, 40), (12000, 7), (17000, 120)]),
           (21000, 26000, [(3000, 10), (9000, 9), (15000, 300), (20000, 55)]),
           (47000, 23000, [(1000, 15), (8000, 3), (14000, 1000)])]
    with open(path, "wb") as f:
        for r, (s0, n, runs) in enumerate(lay):
            txt = bytearray(b"ACGT"[int(c)] for c in g[s0:s0 + n])
            for p, k in runs:
                txt[p:p + k] = b"N" * k
            f.write(b">nr%d\n" % (r + 1))
            for o in range(0, n, 80):
                f.write(bytes(txt[o:o + 80]) + b"\n")


def sa_cases(work):
    """BWTSaValue + BWTRetrievePositionFromSAIndex golden values."""
    idir = os.path.join(GOLD, "index")
    fa = os.path.join(work, "nrun.fa")
    nrun_genome_fasta(fa)
    build_index(fa)
    for e in INDEX_EXT:
        shutil.copy(f"{fa}.index.{e}", os.path.join(idir, f"nrun.fa.index.{e}"))

    def run(prefix, idx, name):
        ib = os.path.join(work, "idx.bin")
        with open(ib, "wb") as f:
            f.write(np.uint32(len(idx)).tobytes())
            f.write(np.asarray(idx, np.uint32).tobytes())
        ob = os.path.join(work, "sa.bin")
        sh(os.path.join(REF, "ref_probe"), "sa", prefix, ib, ob)
        v = np.fromfile(ob, dtype=np.uint32).reshape(-1, 4)
        np.savez_compressed(os.path.join(GOLD, name + ".npz"), idx=np.asarray(idx, np.uint32), sa=v[:, 0],
                            seq_id=v[:, 1], ori_pos=v[:, 2], occ_pos=v[:, 3])
        print(f"{name}: {len(idx)} SA indices")

    T = int(np.fromfile(f"{fa}.index.bwt", dtype=np.uint32, count=5)[4])
    run(fa, np.arange(0, T + 1), "nrun_sa")               # every SA index of the N-run genome
    tiny = os.path.join(idir, "tiny.fa")
    Tt = 200003
    isa0 = int(np.fromfile(f"{tiny}.index.bwt", dtype=np.uint32, count=1)[0])
    idx = set(range(0, 300)) | set(range(Tt - 300, Tt + 1)) | set(range(max(isa0 - 20, 0), min(isa0 + 20, Tt + 1)))
    idx |= set(int(x) for x in (synth._u(123, 6000, 0) % np.uint64(Tt + 1)))
    run(tiny, np.array(sorted(idx)), "tiny_sa")


def read_mgcap(path):
    """Records of oracle/ref_mgcap.c: every bwt_match_gap call of a reference run."""
    raw = open(path, "rb").read()
    assert raw[:4] == b"MGCP"
    o = 4
    recs = []
    while o < len(raw):
        hdr = np.frombuffer(raw[o:o + 20], np.int32).copy()
        o += 20
        strand, L, seed, n_stacks, n_seed = (int(x) for x in hdr)
        opt = np.frombuffer(raw[o:o + 64], np.uint32).copy()
        o += 64
        seq = np.frombuffer(raw[o:o + L], np.uint8).copy()
        o += L
        wb = np.frombuffer(raw[o:o + 8 * (L + 1)], np.int32).reshape(L + 1, 2).copy()
        o += 8 * (L + 1)
        ws = np.frombuffer(raw[o:o + 8 * n_seed], np.int32).reshape(n_seed, 2).copy()
        o += 8 * n_seed
        na = int(np.frombuffer(raw[o:o + 4], np.int32)[0])
        o += 4
        hits = np.frombuffer(raw[o:o + 36 * max(na, 0)], np.uint32).reshape(-1, 9).copy()
        o += 36 * max(na, 0)
        wo = np.frombuffer(raw[o:o + 8 * (L + 1)], np.int32).reshape(L + 1, 2).copy()
        o += 8 * (L + 1)
        recs.append(dict(hdr=hdr, opt=opt, seq=seq, wb=wb, ws=ws, n_aln=na, hits=hits, wo=wo))
    return recs


def splice_reads():
    """Reads that exercise bwt_splice_match and its direct bwt_match_gap calls on the
    tiny index: mismatched and gapped reads, spliced reads of 75-150 bp, and 180-210 bp
    spliced reads whose seeds 1 and 2 map (the anchor call at bwtgap.c:1192)."""
    T, seed = 200003, 7
    g = synth.genome_codes(T, seed)
    rec = synth.record_layout(T, 3)
    seqs = []
    r, _ = synth.make_reads(g, rec, 60, 100, 41, max_mm=4)
    seqs += list(r)
    r, _ = synth.make_reads(g, rec, 60, 100, 42, indel=True, max_mm_indel=2)
    seqs += list(r)
    for i in range(400):   # spliced: exon A + exon B 200-2000 bp downstream
        st = int(synth._u(43, 1, i)[0] % np.uint64(T - 3000))
        L = (100, 150, 75, 120)[i % 4]
        cut = 30 + (i * 7) % (L - 50)
        intron = 200 + (i * 37) % 1800
        s = np.concatenate([g[st:st + cut], g[st + cut + intron:st + L + intron]]).astype(np.uint8)
        if i % 5 == 1:
            s = synth.revcomp_codes(s)
        if i % 7 == 3:
            s[(i * 13) % L] = (s[(i * 13) % L] + 1) % 4
        seqs.append(s)
    # the anchor call at bwtgap.c:1192 needs seeds 1 and 2 mapped > 50 bp apart with
    # seed 0 unmapped (seg_mtype 6): reads of 180-210 bp (seed_len >= 60) whose
    # junction lies inside the first third
    for i in range(200):
        st = int(synth._u(44, 1, i)[0] % np.uint64(T - 3000))
        L = 180 + 10 * (i % 4)
        cut = 15 + (i * 11) % 30
        intron = 300 + (i * 53) % 1500
        s = np.concatenate([g[st:st + cut], g[st + cut + intron:st + L + intron]]).astype(np.uint8)
        seqs.append(synth.revcomp_codes(s) if i % 2 else s)
    return seqs


def mgcap_cases(work):
    """bwt_match_gap called directly with caller widths: every call the
    reference makes on the drop-in read set -- the splice path's seed searches
    (width_seed aliased to width_back, bwtgap.c:809-812), its 12-mer anchors (width_seed
    NULL, :919 and :1192) -- plus a sample of main-path calls (own width_seed)."""
    seqs = splice_reads()
    rb = os.path.join(work, "mg_reads.bin")
    synth.write_reads_bin(rb, seqs)
    idx = os.path.join(GOLD, "index", "tiny.fa")
    for name, args in (("mgcap_default", []), ("mgcap_n4o1", ["-n", "4", "-o", "1"])):
        ob = os.path.join(work, name + ".bin")
        r = subprocess.run([os.path.join(REF, "ref_mgcap"), idx, rb, ob, *args], check=True, capture_output=True,
                           text=True)
        recs = read_mgcap(ob)
        main = [x for x in recs if x["hdr"][2] == 1]
        keep = [x for x in recs if x["hdr"][2] != 1] + main[:300]
        hdr = np.stack([x["hdr"] for x in keep])
        cnt = np.bincount(hdr[:, 2], minlength=3)
        out = dict(hdr=hdr, opt=np.stack([x["opt"] for x in keep]),
                   seq=np.concatenate([x["seq"] for x in keep]),
                   wb=np.concatenate([x["wb"] for x in keep]),
                   ws=np.concatenate([x["ws"] for x in keep]) if any(len(x["ws"]) for x in keep) else
                   np.zeros((0, 2), np.int32),
                   n_aln=np.array([x["n_aln"] for x in keep], np.int32),
                   hits=np.concatenate([x["hits"] for x in keep]),
                   wo=np.concatenate([x["wo"] for x in keep]))
        np.savez_compressed(os.path.join(GOLD, name + ".npz"), **out)
        changed = sum(int(not np.array_equal(x["wb"], x["wo"])) for x in keep)
        print(f"{name}: {len(recs)} calls recorded ({r.stderr.strip()}); kept {len(keep)}: "
              f"{cnt[0]} width_seed NULL, {cnt[2]} aliased, {cnt[1]} own; {int((out['n_aln'] > 0).sum())} with hits, "
              f"{changed} with widths changed by gap_shadow")


def width0_cases(work):
    """bwt_cal_width type 0 (bwtaln.c:98-115; the splice path's width_fore, bwtgap.c:868,
    :872) of the width reads and of the splice read set, on the tiny index."""
    T, seed, nrec = 200003, 7, 3
    g = synth.genome_codes(T, seed)
    rec = synth.record_layout(T, nrec)
    seqs = edge_reads(g, rec, 21)[:24] + splice_reads()[:200]
    rb = os.path.join(work, "w0.bin")
    synth.write_reads_bin(rb, seqs)
    prefix = os.path.join(GOLD, "index", "tiny.fa")
    sh(os.path.join(REF, "ref_probe"), "width", prefix, rb, os.path.join(work, "w0out.bin"), "0")
    w = np.fromfile(os.path.join(work, "w0out.bin"), dtype=np.uint32).reshape(-1, 2)
    lens, codes = pack_reads(seqs)
    np.savez_compressed(os.path.join(GOLD, "tiny_width0.npz"), lens=lens, codes=codes, width=w)
    print(f"tiny_width0: {len(seqs)} reads")


def read_extcap(path):
    """Records of oracle/ref_extcap.c: every seed extension of a reference run."""
    raw = open(path, "rb").read()
    assert raw[:4] == b"EXCP"
    o = 4
    recs = []
    while o < len(raw):
        hdr = np.frombuffer(raw[o:o + 32], np.int32).copy()
        o += 32
        n = int(hdr[6])
        opt = np.frombuffer(raw[o:o + 64], np.uint32).copy()
        o += 64
        aln_in = np.frombuffer(raw[o:o + 36], np.uint32).copy()
        o += 36
        seq = np.frombuffer(raw[o:o + n], np.uint8).copy()
        o += n
        bid = np.frombuffer(raw[o:o + 4 * n], np.int32).copy()
        o += 4 * n
        tail = np.frombuffer(raw[o:o + 8], np.int32).copy()
        o += 8
        aln_out = np.frombuffer(raw[o:o + 36], np.uint32).copy()
        o += 36
        recs.append(dict(hdr=hdr, opt=opt, aln_in=aln_in, seq=seq, bid=bid, tail=tail, aln_out=aln_out))
    return recs


def extcap_cases(work):
    """The splice path's seed extensions (bwt_extend_foreward / bwt_extend_backward,
    bwtgap.c:640-663 -> bwt_backtracing_search :346-511): every call the reference makes
    on the drop-in splice read set, recorded by oracle/ref_extcap.c with the window of
    sequence and widths each call reads."""
    seqs = splice_reads()
    rb = os.path.join(work, "ext_reads.bin")
    synth.write_reads_bin(rb, seqs)
    idx = os.path.join(GOLD, "index", "tiny.fa")
    for name, args in (("extcap_default", []), ("extcap_n4o1", ["-n", "4", "-o", "1"])):
        ob = os.path.join(work, name + ".bin")
        r = subprocess.run([os.path.join(REF, "ref_extcap"), idx, rb, ob, *args], check=True, capture_output=True,
                           text=True)
        recs = read_extcap(ob)
        out = dict(hdr=np.stack([x["hdr"] for x in recs]), opt=np.stack([x["opt"] for x in recs]),
                   aln_in=np.stack([x["aln_in"] for x in recs]), seq=np.concatenate([x["seq"] for x in recs]),
                   bid=np.concatenate([x["bid"] for x in recs]), tail=np.stack([x["tail"] for x in recs]),
                   aln_out=np.stack([x["aln_out"] for x in recs]))
        np.savez_compressed(os.path.join(GOLD, name + ".npz"), **out)
        ret = out["tail"][:, 0]
        print(f"{name}: {len(recs)} calls ({r.stderr.strip()}): {int((out['hdr'][:, 0] == 1).sum())} backward; "
              f"ret 1: {int((ret == 1).sum())}, 2: {int((ret == 2).sum())}, -1: {int((ret == -1).sum())}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ecoli", action="store_true")
    ap.add_argument("--dropin", action="store_true")
    ap.add_argument("--sa", action="store_true")
    ap.add_argument("--mgcap", action="store_true")
    ap.add_argument("--extcap", action="store_true")
    ap.add_argument("--width0", action="store_true")
    ap.add_argument("--limits", action="store_true")
    a = ap.parse_args()
    if not os.path.exists(os.path.join(REF, "ref_probe")):
        sys.exit("build oracle/_ref first: make -C oracle -f ref.mk")
    os.makedirs(GOLD, exist_ok=True)
    with tempfile.TemporaryDirectory() as work:
        if a.ecoli:
            ecoli_cases(work)
        elif a.dropin:
            dropin_cases(work)
        elif a.sa:
            sa_cases(work)
        elif a.mgcap:
            mgcap_cases(work)
        elif a.extcap:
            extcap_cases(work)
        elif a.width0:
            width0_cases(work)
        elif a.limits:
            limits_cases(work)
        else:
            tiny_cases(work)


if __name__ == "__main__":
    main()
