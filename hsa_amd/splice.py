"""The splice path's seed searches (bwt_splice_match, bwtgap.c:748-848) as one batch.

For a read that found no hit on either strand, bwt_splice_match searches up to six
seeds: for strand s (0 = the read, 1 = its reverse complement) and i = 0, 1, 2, the
seed of length seed_len = len // 3 (plus len % 3 for the last one) at offset
i * seed_len.  Its widths are those of the strand sequence's PREFIX of that length,
with width_seed aliased to width_back (bwtgap.c:804-809), and its options are the
batch's local_opt with GAPE cleared, max_gapo = max_gape = 0, max_diff =
max_seed_diff and seed_len = the seed's length (bwtgap.c:769-774, :802).  Which seeds
it asks for depends on earlier answers (bwtgap.c:821-847); all six are computed here,
in one GPU pass (the C drop-in does the same and answers bwt_splice_match from the
table, hsa_amd/csrc/bwtgap_gpu.c).
"""
from __future__ import annotations

import numpy as np

GAPE = 0x01
CALL_DTYPE = np.dtype([("read", "<i8"), ("i", "<i4"), ("strand", "<i4"), ("len", "<u4"), ("off", "<u8"),
                       ("wb_off", "<u8")])


def seed_options(local_opt: dict) -> dict:
    """The option block of the seed searches (bwtgap.c:769-774); seed_len per seed."""
    o = dict(local_opt)
    o["mode"] &= ~GAPE
    o["max_gapo"] = 0
    o["max_gape"] = 0
    o["max_diff"] = local_opt["max_seed_diff"]
    return o


def n_stacks_of(local_opt: dict) -> int:
    """aln_score(max_diff+1, max_gapo+1, max_gape+1) of local_opt: the batch stack
    every call shares (bwtaln.c:279, bwtgap.c:13-18)."""
    o = local_opt
    return (o["max_diff"] + 1) * o["s_mm"] + (o["max_gapo"] + 1) * o["s_gapo"] + (o["max_gape"] + 1) * o["s_gape"]


def revcomp_rows(a: np.ndarray) -> np.ndarray:
    """seq_reverse(len, seq, 1) (bwaseqio.c:73-84) of every row: codes > 3 are kept."""
    r = a[:, ::-1].copy()
    m = r < 4
    r[m] = 3 - r[m]
    return r


def seed_calls(lens, codes, reads, local_opt: dict, width_fn):
    """The six seed calls of every read in `reads` (indices into lens / codes), in read
    order, i = 0..5 within a read (bwtgap.c:797).

    width_fn(lens, codes) -> flat widths, 2 * (len + 1) words per sequence
    (bwt_cal_width type 1: hsa_width_batch on the GPU, or the oracle on the CPU).
    Returns dict(calls: CALL_DTYPE records, codes, widths (P, 2) int32, opt), or None."""
    lens = np.asarray(lens, np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)])
    reads = np.asarray(reads, np.int64)
    reads = reads[lens[reads] >= 3]
    if len(reads) == 0:
        return None
    groups = []
    for L in np.unique(lens[reads]):
        rr = reads[lens[reads] == L]
        L = int(L)
        sl = L // 3
        idx = offs[rr][:, None] + np.arange(L)[None, :]
        fwd = np.asarray(codes, np.uint8)[idx]
        strand_seq = (fwd, revcomp_rows(fwd))
        # prefix widths: per read and strand, prefixes of sl and of sl + L % 3
        ks = (0, 1) if L % 3 else (0,)
        pre_lens, pre_codes = [], []
        for s in (0, 1):
            for k in ks:
                la = sl + (L % 3 if k else 0)
                pre_lens.append(np.full(len(rr), la, np.uint32))
                pre_codes.append(strand_seq[s][:, :la].reshape(-1))
        w = np.asarray(width_fn(np.concatenate(pre_lens), np.concatenate(pre_codes)), np.uint32).view(np.int32)
        pw = {}
        o = 0
        for s in (0, 1):
            for k in ks:
                la = sl + (L % 3 if k else 0)
                n = len(rr) * 2 * (la + 1)
                pw[(s, k)] = w[o:o + n].reshape(len(rr), la + 1, 2)
                o += n
        groups.append((rr, L, sl, strand_seq, pw))
    # assemble calls in read order
    order = np.argsort(reads, kind="stable")
    per_read = {}
    for rr, L, sl, strand_seq, pw in groups:
        for j, r in enumerate(rr):
            per_read[int(r)] = (j, L, sl, strand_seq, pw)
    calls = np.zeros(6 * len(reads), CALL_DTYPE)
    c_codes, c_widths = [], []
    co = po = 0
    q = 0
    for r in reads[order]:
        j, L, sl, strand_seq, pw = per_read[int(r)]
        for i in range(6):
            s = i // 3
            la = sl + (L % 3 if i % 3 == 2 else 0)
            k = 1 if (i % 3 == 2 and L % 3) else 0
            c_codes.append(strand_seq[s][j, (i % 3) * sl:(i % 3) * sl + la])
            c_widths.append(pw[(s, k)][j])
            calls[q] = (r, i, s, la, co, po)
            co += la
            po += la + 1
            q += 1
    return dict(calls=calls, codes=np.concatenate(c_codes).astype(np.uint8),
                widths=np.concatenate(c_widths).astype(np.int32), opt=seed_options(local_opt))


def seed_calls_fixed(reads2d: np.ndarray, local_opt: dict, width_fn):
    """seed_calls for reads of one length given as an (n, L) array (vectorised: the
    bench's path).  Same call order and layout as seed_calls."""
    n, L = reads2d.shape
    sl = L // 3
    fwd = np.asarray(reads2d, np.uint8)
    strand_seq = (fwd, revcomp_rows(fwd))
    ks = (0, 1) if L % 3 else (0,)
    pre_lens, pre_codes, keys = [], [], []
    for s in (0, 1):
        for k in ks:
            la = sl + (L % 3 if k else 0)
            pre_lens.append(np.full(n, la, np.uint32))
            pre_codes.append(strand_seq[s][:, :la].reshape(-1))
            keys.append((s, k, la))
    w = np.asarray(width_fn(np.concatenate(pre_lens), np.concatenate(pre_codes)), np.uint32).view(np.int32)
    pw, o = {}, 0
    for s, k, la in keys:
        m = n * 2 * (la + 1)
        pw[(s, k)] = w[o:o + m].reshape(n, la + 1, 2)
        o += m
    las = [sl + (L % 3 if i % 3 == 2 else 0) for i in range(6)]
    per_read_codes = sum(las)
    per_read_pairs = sum(la + 1 for la in las)
    codes = np.empty((n, per_read_codes), np.uint8)
    widths = np.empty((n, per_read_pairs, 2), np.int32)
    calls = np.zeros((n, 6), CALL_DTYPE)
    co = po = 0
    for i in range(6):
        s, la = i // 3, las[i]
        k = 1 if (i % 3 == 2 and L % 3) else 0
        codes[:, co:co + la] = strand_seq[s][:, (i % 3) * sl:(i % 3) * sl + la]
        widths[:, po:po + la + 1] = pw[(s, k)]
        calls[:, i]["read"] = np.arange(n)
        calls[:, i]["i"] = i
        calls[:, i]["strand"] = s
        calls[:, i]["len"] = la
        calls[:, i]["off"] = np.arange(n, dtype=np.uint64) * per_read_codes + co
        calls[:, i]["wb_off"] = np.arange(n, dtype=np.uint64) * per_read_pairs + po
        co += la
        po += la + 1
    return dict(calls=calls.reshape(-1), codes=codes.reshape(-1), widths=widths.reshape(-1, 2),
                opt=seed_options(local_opt))


def seed_jobs(batch):
    """hsa_job_t / hsa_mg_job_t arrays of a seed batch (width_seed aliased)."""
    from hsa_amd._lib import JOB_DTYPE, MG_DTYPE, SEED_ALIAS
    c = batch["calls"]
    so = batch["opt"]
    jobs = np.zeros(len(c), JOB_DTYPE)
    jobs["off"] = c["off"]
    jobs["len"] = c["len"]
    jobs["max_diff"] = so["max_diff"]
    jobs["seed_len"] = c["len"]
    mg = np.zeros(len(c), MG_DTYPE)
    mg["wb_off"] = c["wb_off"]
    mg["strand"] = c["strand"]
    mg["seed"] = SEED_ALIAS
    return jobs, mg


def run_seed_calls(gi, batch, n_stacks: int):
    """All seed calls of `batch` in one hsa_match_gap_batch pass.
    Returns (n_aln, hit_off, hits, widths after, stats)."""
    from hsa_amd._lib import regime_of
    jobs, mg = seed_jobs(batch)
    so = batch["opt"]
    rg = regime_of(so, n_stacks, so["max_diff"])
    return gi.match_gap([rg], jobs, mg, batch["codes"], batch["widths"])
