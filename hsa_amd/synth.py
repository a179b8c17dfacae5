"""Deterministic synthetic genomes and reads for the HSA inexact-alignment path.

Every generator here is counter based (splitmix64 over a block / read index),
so the same bytes come out on any host and can be regenerated on the GPU box
without shipping data.  Layouts follow the reference's conventions:

* base codes are 0..3 for A,C,G,T and 4 for N (bwaseqio.c:10-27 `nst_nt4_table`);
* a reverse complement keeps codes >3 unchanged (bwaseqio.c:73 `seq_reverse`);
* FASTA/FASTQ text is what `HSA index` / `HSA aln` read (HSP.c:133, bwaseqio.c:161).

The genome is one concatenated stream split into records; reads never straddle a
record boundary.  Nothing here is on the timed path.
"""
from __future__ import annotations

import numpy as np

ACGT = np.frombuffer(b"ACGTN", dtype=np.uint8)
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 finaliser over uint64 (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = (x + _GOLD).astype(np.uint64, copy=False)
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def _stream(seed: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        base = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) * _GOLD
        return splitmix64(base ^ idx.astype(np.uint64))


def genome_words(T: int, seed: int) -> np.ndarray:
    """Packed genome: 32 bases per uint64, base j of word w at bits 2j..2j+1."""
    nw = (T + 31) // 32
    w = _stream(seed, np.arange(nw, dtype=np.uint64))
    if T % 32:
        w[-1] &= np.uint64((1 << (2 * (T % 32))) - 1)
    return w


def genome_codes(T: int, seed: int) -> np.ndarray:
    """Unpacked genome codes (uint8 0..3), length T."""
    w = genome_words(T, seed)
    shifts = (np.arange(32, dtype=np.uint64) * np.uint64(2))
    codes = ((w[:, None] >> shifts[None, :]) & np.uint64(3)).astype(np.uint8)
    return codes.reshape(-1)[:T]


class PackedGenome:
    """A genome held as genome_words() (2 bits per base): 4x smaller than codes,
    enough for a 3 Gbp text on the host.  Indexable by integer arrays."""

    def __init__(self, T: int, seed: int):
        self.T = T
        self.words = genome_words(T, seed)

    def __len__(self):
        return self.T

    def __getitem__(self, pos):
        pos = np.asarray(pos, dtype=np.int64)
        w = self.words[pos >> 5]
        return ((w >> ((pos & 31).astype(np.uint64) * np.uint64(2))) & np.uint64(3)).astype(np.uint8)


def record_layout(T: int, n_records: int) -> list[tuple[int, int]]:
    """(start, length) of each record; the last record takes the remainder."""
    if n_records <= 1:
        return [(0, T)]
    per = T // n_records
    out = [(i * per, per) for i in range(n_records - 1)]
    out.append(((n_records - 1) * per, T - (n_records - 1) * per))
    return out


def write_fasta(path: str, codes: np.ndarray, records: list[tuple[int, int]],
                width: int = 80, names: list[str] | None = None) -> None:
    with open(path, "wb") as f:
        for r, (s, n) in enumerate(records):
            name = names[r] if names else f"chr{r + 1}"
            f.write(b">" + name.encode() + b"\n")
            txt = ACGT[codes[s:s + n]]
            for o in range(0, n, width):
                f.write(txt[o:o + width].tobytes())
                f.write(b"\n")


def revcomp_codes(seq: np.ndarray) -> np.ndarray:
    """Reverse complement over the last axis; codes >3 are kept (bwaseqio.c:73-89)."""
    rc = seq[..., ::-1].copy()
    m = rc < 4
    rc[m] = 3 - rc[m]
    return rc


def _u(seed: int, n: int, k: int) -> np.ndarray:
    """k-th uniform uint64 draw for reads 0..n-1."""
    idx = np.arange(n, dtype=np.uint64) * np.uint64(4096) + np.uint64(k)
    return _stream(seed, idx)


def _starts(seed, n, L, span, records, slot):
    # a record chosen proportionally to its length, then a start inside it
    lens = np.array([r[1] for r in records], dtype=np.int64)
    offs = np.array([r[0] for r in records], dtype=np.int64)
    usable = np.maximum(lens - span, 1)
    cum = np.cumsum(usable)
    x = (_u(seed, n, slot) % np.uint64(cum[-1])).astype(np.int64)
    rec = np.searchsorted(cum, x, side="right")
    before = np.concatenate([[0], cum[:-1]])
    return offs[rec] + (x - before[rec])


def _mutate(seed, reads, n_mm, slot0):
    """Substitute n_mm[r] distinct positions of read r by base+(1..3) mod 4."""
    n, L = reads.shape
    if n == 0 or int(n_mm.max(initial=0)) == 0:
        return reads
    keys = np.empty((n, L), dtype=np.uint64)
    for p in range(L):
        keys[:, p] = _u(seed, n, slot0 + p)
    order = np.argsort(keys, axis=1, kind="stable")
    shift = np.empty((n, L), dtype=np.uint8)
    for p in range(L):
        shift[:, p] = (1 + (_u(seed, n, slot0 + L + p) % np.uint64(3))).astype(np.uint8)
    rank = np.empty_like(order)
    np.put_along_axis(rank, order, np.arange(L)[None, :].repeat(n, 0), axis=1)
    hit = rank < n_mm[:, None]
    out = reads.copy()
    out[hit] = (out[hit] + shift[hit]) & 3
    return out


def make_reads(genome: np.ndarray, records, n: int, L: int, seed: int,
               max_mm: int = 0, indel: bool = False, max_mm_indel: int = 2,
               rc_frac: float = 0.5, chunk: int = 200_000):
    """Synthetic reads (uint8 codes, shape (n, L)) plus their truth.

    * `max_mm`: number of substitutions uniform in {0..max_mm}.
    * `indel`: one deletion or insertion of 1-3 bp at a read position in [20, 80)
      (scaled to L) plus 0..max_mm_indel substitutions (config 3).
    * `rc_frac`: fraction of reads reverse-complemented.
    Returns (reads, truth) with truth a dict of int64 arrays: start, strand, n_mm,
    indel_len (negative = deletion from the read's point of view).
    """
    reads = np.empty((n, L), dtype=np.uint8)
    truth = {k: np.zeros(n, dtype=np.int64) for k in ("start", "strand", "n_mm", "indel_len")}
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        sub = seed * 1_000_003 + c0
        span = L + 3
        st = _starts(sub, m, L, span, records, 0)
        strand = (_u(sub, m, 1) % np.uint64(1 << 20)).astype(np.float64) / float(1 << 20) < rc_frac
        if indel:
            is_del = (_u(sub, m, 2) & np.uint64(1)).astype(bool)
            ilen = (1 + (_u(sub, m, 3) % np.uint64(3))).astype(np.int64)
            lo, hi = (20 * L) // 100, (80 * L) // 100
            ipos = lo + (_u(sub, m, 4) % np.uint64(max(hi - lo, 1))).astype(np.int64)
            nmm = (_u(sub, m, 5) % np.uint64(max_mm_indel + 1)).astype(np.int64)
            idx = np.arange(L)[None, :]
            src = st[:, None] + idx
            # deletion: read skips ilen genome bases after ipos
            d_src = np.where(idx >= ipos[:, None], src + ilen[:, None], src)
            # insertion: ilen random bases at ipos, then genome continues
            i_src = np.where(idx >= ipos[:, None], src - ilen[:, None], src)
            gsrc = np.where(is_del[:, None], d_src, i_src)
            r = np.asarray(genome[gsrc], dtype=np.uint8)
            ins_mask = (~is_del[:, None]) & (idx >= ipos[:, None]) & (idx < (ipos + ilen)[:, None])
            rnd = np.empty((m, L), dtype=np.uint8)
            for p in range(L):
                rnd[:, p] = (_u(sub, m, 8 + p) & np.uint64(3)).astype(np.uint8)
            r = np.where(ins_mask, rnd, r).astype(np.uint8)
            truth["indel_len"][c0:c0 + m] = np.where(is_del, -ilen, ilen)
            slot = 8 + L
        else:
            nmm = (_u(sub, m, 5) % np.uint64(max_mm + 1)).astype(np.int64) if max_mm else np.zeros(m, np.int64)
            r = np.asarray(genome[st[:, None] + np.arange(L)[None, :]], dtype=np.uint8)
            slot = 8
        r = _mutate(sub, r, nmm, slot)
        r = np.where(strand[:, None], revcomp_codes(r), r)
        reads[c0:c0 + m] = r
        truth["start"][c0:c0 + m] = st
        truth["strand"][c0:c0 + m] = strand
        truth["n_mm"][c0:c0 + m] = nmm
    return reads, truth


def make_spliced_reads(genome, records, n: int, L: int, seed: int, rc_frac: float = 0.5, tries: int = 64,
                       chunk: int = 200_000):
    """Spliced reads: exon A of 40-110 bases, an intron of
    200-5000 bases that reads GT...AG on the + strand, then exon B up to L bases; 50 %
    reverse-complemented.  Exon-A and intron lengths are drawn uniformly and rejected
    until the motifs match (a read with no match among `tries` draws redraws its start).
    Returns (reads (n, L) uint8, truth dict of start, exon_a, intron, strand)."""
    reads = np.empty((n, L), dtype=np.uint8)
    truth = {k: np.zeros(n, dtype=np.int64) for k in ("start", "exon_a", "intron", "strand")}
    span = 110 + 5000 + L
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        sub = seed * 1_000_003 + c0
        todo = np.arange(m)
        st = np.zeros(m, np.int64)
        ea = np.zeros(m, np.int64)
        it = np.zeros(m, np.int64)
        rnd = 0
        while len(todo):
            k = len(todo)
            st[todo] = _starts(sub + 7919 * rnd, k, L, span, records, 0)
            # donor: GT right after exon A
            ca = 40 + (_u(sub + 7919 * rnd, k * tries, 1) % np.uint64(71)).astype(np.int64).reshape(k, tries)
            d = st[todo][:, None] + ca
            okd = (np.asarray(genome[d], np.uint8) == 2) & (np.asarray(genome[d + 1], np.uint8) == 3)
            # acceptor: AG as the intron's last two bases
            ci = 200 + (_u(sub + 7919 * rnd, k * tries, 2) % np.uint64(4801)).astype(np.int64).reshape(k, tries)
            fd = np.argmax(okd, axis=1)
            dd = st[todo] + ca[np.arange(k), fd]
            a = dd[:, None] + ci
            oka = (np.asarray(genome[a - 2], np.uint8) == 0) & (np.asarray(genome[a - 1], np.uint8) == 2)
            fa = np.argmax(oka, axis=1)
            good = okd.any(axis=1) & oka.any(axis=1)
            ea[todo[good]] = ca[np.arange(k), fd][good]
            it[todo[good]] = ci[np.arange(k), fa][good]
            todo = todo[~good]
            rnd += 1
        pos = np.arange(L)[None, :]
        src = np.where(pos < ea[:, None], st[:, None] + pos, st[:, None] + it[:, None] + pos)
        r = np.asarray(genome[src], dtype=np.uint8)
        strand = (_u(sub, m, 3) % np.uint64(1 << 20)).astype(np.float64) / float(1 << 20) < rc_frac
        r = np.where(strand[:, None], revcomp_codes(r), r)
        reads[c0:c0 + m] = r
        truth["start"][c0:c0 + m] = st
        truth["exon_a"][c0:c0 + m] = ea
        truth["intron"][c0:c0 + m] = it
        truth["strand"][c0:c0 + m] = strand
    return reads, truth


def write_fastq(path: str, reads: np.ndarray, prefix: str = "r", qual_seed: int | None = None) -> None:
    """FASTQ of the reads; quality 'I' everywhere, or (qual_seed) a random Phred+33 string
    in '#'..'J' per read (so that a reverse-strand SAM line's reversed quality shows)."""
    n, L = reads.shape
    quals = None if qual_seed is None else np.random.default_rng(qual_seed).integers(35, 75, (n, L), dtype=np.uint8)
    qual = b"I" * L
    with open(path, "wb") as f:
        for i in range(n):
            f.write(b"@%s%d\n" % (prefix.encode(), i))
            f.write(ACGT[reads[i]].tobytes())
            f.write(b"\n+\n")
            f.write(qual if quals is None else quals[i].tobytes())
            f.write(b"\n")


def write_reads_bin(path: str, reads) -> None:
    """Binary read file for the oracle probe: u32 n, u32 len[n], then codes."""
    if isinstance(reads, np.ndarray):
        seqs = [reads[i] for i in range(reads.shape[0])]
    else:
        seqs = list(reads)
    lens = np.array([len(s) for s in seqs], dtype=np.uint32)
    with open(path, "wb") as f:
        f.write(np.uint32(len(seqs)).tobytes())
        f.write(lens.tobytes())
        for s in seqs:
            f.write(np.asarray(s, dtype=np.uint8).tobytes())
