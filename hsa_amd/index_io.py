"""Readers/writers for the 2BWT on-disk index format (the files `HSA index` writes).

Formats (little-endian u32 words):
* `.bwt` / `.rev.bwt`: inverseSa0, C[1..4] (C[4] = T), then ceil(T/16) words of
  2-bit codes, MSB-first inside a word; `$` is not encoded (BWT.c:156-181,
  BWTConstruct.c:1209-1224).
* `.fmv` / `.rev.fmv`: inverseSa0, C[1..4], then the 16-bit-pair minor Occ samples
  every 256 characters, then the major samples every 65 536 (BWT.c:163-189,
  BWTOccValueMinorSizeInWord / MajorSizeInWord BWT.c:1097-1117).
* `.sa`: inverseSa0, C[1..4], saInterval, then (T+s)/s words (BWT.c:206-223).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np


@dataclass
class BwtFile:
    T: int
    isa0: int
    C: np.ndarray          # uint32[5], C[0] = 0
    code: np.ndarray       # uint32 words, MSB-first 2-bit codes


def read_bwt(path: str) -> BwtFile:
    raw = np.fromfile(path, dtype=np.uint32)
    C = np.zeros(5, np.uint32)
    C[1:] = raw[1:5]
    T = int(C[4])
    nw = (T + 15) // 16
    return BwtFile(T=T, isa0=int(raw[0]), C=C, code=np.ascontiguousarray(raw[5:5 + nw]))


def read_index(prefix: str) -> tuple[BwtFile, BwtFile]:
    """`prefix` as given to `HSA aln` (the FASTA path); files are prefix.index.*"""
    p = prefix + ".index"
    return read_bwt(p + ".bwt"), read_bwt(p + ".rev.bwt")


def unpack_codes(b: BwtFile) -> np.ndarray:
    sh = (30 - 2 * np.arange(16)).astype(np.uint32)
    return ((b.code[:, None] >> sh[None, :]) & np.uint32(3)).astype(np.uint8).reshape(-1)[:b.T]


def pack_codes_msb(codes: np.ndarray) -> np.ndarray:
    """2-bit codes -> .bwt word layout (16 per u32, first code in the top bits)."""
    n = len(codes)
    nw = (n + 15) // 16
    pad = np.zeros(nw * 16, np.uint32)
    pad[:n] = codes
    sh = (30 - 2 * np.arange(16)).astype(np.uint32)
    return (pad.reshape(nw, 16) << sh[None, :]).sum(axis=1, dtype=np.uint64).astype(np.uint32)


def occ_files(codes: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """The reference's sampled Occ arrays for a $-less code string.

    Minor sample e (every 256 chars) holds the count of each character in
    [256*(e - e%256), 256*e) as 16-bit halves, even e in the high half; major
    sample m holds counts in [0, 65536*m).  Sizes follow BWT.c:1097-1117.  When the
    sample count is odd the low half of the last minor word is never read by
    BWTOccValue; the reference's builder repeats the previous sample there, as here."""
    T = len(codes)
    n_occ = (T + 255) // 256 + 1
    minor = np.zeros(((n_occ + 1) // 2) * 4, np.uint32)
    n_major = (n_occ + 255) // 256
    major = np.zeros(n_major * 4, np.uint32)
    pref = np.zeros((n_occ, 4), np.int64)
    # samples past T count the zero padding of the code array as 'A', as the
    # builder does (BWTConstruct.c:997-1090 reads the cleared tail words)
    padded = np.zeros(n_occ * 256, np.uint8)
    padded[:T] = codes
    for c in range(4):
        cs = np.concatenate([[0], np.cumsum(padded == c)])
        pref[:, c] = cs[np.arange(n_occ) * 256]
    maj = pref[(np.arange(n_major) * 256)]
    major[:] = maj.reshape(-1).astype(np.uint32)
    rel = (pref - maj[np.arange(n_occ) // 256]).astype(np.uint32)
    if n_occ % 2:
        rel = np.concatenate([rel, rel[-1:]])
    minor[:] = ((rel[0::2] << np.uint32(16)) | rel[1::2]).reshape(-1)
    return minor, major


def write_bwt_files(prefix: str, T: int, isa0: int, C: np.ndarray, codes: np.ndarray,
                    suffix: str = "") -> None:
    """Write prefix.index{suffix}.bwt and .fmv in the reference's format."""
    head = np.concatenate([[isa0], np.asarray(C, np.uint32)[1:5]]).astype(np.uint32)
    with open(f"{prefix}.index{suffix}.bwt", "wb") as f:
        f.write(head.tobytes())
        f.write(pack_codes_msb(codes).tobytes())
    minor, major = occ_files(codes)
    with open(f"{prefix}.index{suffix}.fmv", "wb") as f:
        f.write(head.tobytes())
        f.write(minor.tobytes())
        f.write(major.tobytes())


@dataclass
class SaFile:
    interval: int
    values: np.ndarray     # uint32[(T+s)/s]; values[0] = -1 as BWTLoad sets it (BWT.c:222)


def read_sa(prefix: str) -> SaFile:
    """prefix.index.sa: inverseSa0, C[1..4], saInterval, then (T+s)/s sampled SA
    values (BWT.c:206-223)."""
    raw = np.fromfile(prefix + ".index.sa", dtype=np.uint32)
    T, s = int(raw[4]), int(raw[5])
    vals = np.ascontiguousarray(raw[6:6 + (T + s) // s]).copy()
    vals[0] = 0xFFFFFFFF
    return SaFile(interval=s, values=vals)


def read_blocks(prefix: str) -> np.ndarray:
    """Chromosome blocks of prefix.index.ann (HSP.c:325-337, ChrBlock HSP.h:41-46) as
    uint32 rows (chrID, blockStart, blockEnd, ori), in file order."""
    with open(prefix + ".index.ann") as f:
        lines = f.read().split("\n")
    n_chr = int(lines[0].split()[1])
    i = 1 + n_chr
    nb = int(lines[i].split()[0])
    rows = [list(map(int, lines[i + 1 + k].split()[:4])) for k in range(nb)]
    return np.array(rows, dtype=np.int64).astype(np.uint32).reshape(-1, 4)


def exists(prefix: str) -> bool:
    return all(os.path.exists(f"{prefix}.index.{e}") for e in ("bwt", "rev.bwt"))


def read_pac(prefix: str, T: int | None = None) -> np.ndarray:
    """Forward text from prefix.index.pac: 4 codes per byte, first code in the high
    bits, then (T%4==0 ? a 0 byte : nothing) and a final byte T%4 (HSP.c:313-323)."""
    raw = np.fromfile(prefix + ".index.pac", dtype=np.uint8)
    if T is None:
        with open(prefix + ".index.ann") as f:
            T = int(f.readline().split()[0])
    sh = np.array([6, 4, 2, 0], np.uint8)
    codes = ((raw[:, None] >> sh[None, :]) & 3).reshape(-1)
    return codes[:T].astype(np.uint8)


def read_packed_dna(prefix: str):
    """prefix.index.pac as the HSP holds it in memory (DNALoadPacked with word packing,
    TextConverter.c:677-725): dnaLength = (file bytes - 1) * 4 + the last byte; then
    (dnaLength + 15) / 16 + 1 words, the file's bytes (less the last) read into them,
    the last two words zeroed first, and every word but the last byte-swapped so that
    code k sits at bits (~k & 15) * 2.  Returns (words, dnaLength)."""
    raw = np.fromfile(prefix + ".index.pac", dtype=np.uint8)
    flen = len(raw) - 1
    T = flen * 4 + int(raw[-1])
    wtp = (T + 15) // 16
    buf = np.zeros(4 * (wtp + 1), np.uint8)
    n = min(flen, len(buf))
    buf[:n] = raw[:n]
    w = buf.view("<u4").copy()
    w[:wtp] = buf[:4 * wtp].view(">u4")
    return w.astype(np.uint32), T


def pack_lsb_u32(codes: np.ndarray) -> np.ndarray:
    """2-bit codes -> 16 per u32, code j at bits 2j..2j+1 (the device text layout)."""
    n = len(codes)
    nw = (n + 15) // 16
    pad = np.zeros(nw * 16, np.uint64)
    pad[:n] = codes
    sh = (2 * np.arange(16)).astype(np.uint64)
    return (pad.reshape(nw, 16) << sh[None, :]).sum(axis=1).astype(np.uint32)


def unpack_lsb_u32(words: np.ndarray, n: int) -> np.ndarray:
    sh = (2 * np.arange(16)).astype(np.uint32)
    return ((words[:, None] >> sh[None, :]) & np.uint32(3)).astype(np.uint8).reshape(-1)[:n]
