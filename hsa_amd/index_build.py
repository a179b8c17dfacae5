"""From-scratch 2BWT index builder: a FASTA file -> every file `HSA index` writes
(`.pac .ann .rev.pac .bwt .fmv .rev.bwt .rev.fmv .sa`), byte-identical, with the
suffix sorting on the GPU.

The reference builds its BWTs with an incremental CPU construction
(BWTIncConstructFromPacked, BWTConstruct.c:108; hours at hg19 size) and its sampled
suffix array by an LF walk over the finished BWT (BWTGenerateSaValue,
BWTConstruct.c:1241).  Here both come from one device suffix sort per direction
(hsa_build_bwt_index_device: the BWT characters and every saInterval-th SA value of
the same sorted order).  The host part restates the reference's file semantics,
quirks included, since the search depends on them:

* FASTA -> packed text + annotation (HSPParseFASTAToPacked, HSP.c:133-343): records
  under 75 characters are dropped; runs of >= 10 ambiguous characters split a
  record into blocks (a leading run shifts the first block's origin, a trailing one is
  cut), shorter runs become 'G'; the .pac length byte counts the record lengths WITH
  their ambiguous characters (HSP.c:311, :318-323), so the text the BWT is built
  from may differ from the packed characters by up to three 'A's at the end;
* the reversed text (BuildReversePacked, 2BWT-Builder.c:116-213), including the loss of
  its last 16 characters when the text length is a multiple of 16;
* text length of a .pac file: (bytes - 2) * 4 + last byte (TextLengthFromBytePacked,
  TextConverter.c:178, as BWTConstruct.c:128-134 calls it).

Checked against the reference's own index files (tests/test_gpu_build.py).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import index_io

MIN_RECORD = 75            # HSP.c:222
MIN_N_RUN = 10             # HSP.c:250, :275
SA_INTERVAL = 8            # 2BWT-Builder.c:97 (SaValueFreq)
# HSP.h:102-105: dnaChar order; ambiguityCount == 1 only for A, C, G, T
_ACGT = np.full(256, 255, np.uint8)
for _i, _c in enumerate(b"ACGT"):
    _ACGT[_c] = _i


def _records(data: bytes):
    """(name, sequence bytes) per FASTA record as HSPParseFASTAToPacked reads them:
    the name runs to the first tab, space or newline (at most 256 characters), the rest
    of the header line is skipped, and every other byte up to the next '>' except '\\n'
    is sequence, a-z upper-cased."""
    if not data.startswith(b">"):
        raise ValueError("FASTA file does not begin with '>'")
    pos = 1
    n = len(data)
    while pos < n:
        end = data.find(b">", pos)
        if end < 0:
            end = n
        nl = data.find(b"\n", pos, end)
        head = data[pos:nl if nl >= 0 else end]
        name = head
        for sep in (b"\t", b" "):
            k = name.find(sep)
            if k >= 0:
                name = name[:k]
        name = name[:256]
        body = data[nl + 1:end] if nl >= 0 else b""
        seq = np.frombuffer(body, np.uint8)
        seq = seq[seq != 10]
        low = (seq >= 97) & (seq <= 122)
        if low.any():
            seq = seq.copy()
            seq[low] -= 32
        yield name.decode("latin-1"), seq
        pos = end + 1


def parse_fasta(data: bytes):
    """HSPParseFASTAToPacked (HSP.c:133-343): returns (packed codes, annotation rows,
    total characters).  Annotation rows: (name, blocks) with blocks (start, end, ori) in
    packed-text coordinates (end may be start - 1: an all-ambiguous record)."""
    parts, ann = [], []
    useful = 0
    total = 0
    for name, seq in _records(data):
        L = len(seq)
        if L < MIN_RECORD:
            continue
        code = _ACGT[seq]
        amb = code == 255
        blocks = []
        if not amb.any():
            parts.append(code)
            blocks.append((useful, useful + L - 1, 0))
            useful += L
        else:
            # first unambiguous character (HSP.c:249); a leading run shorter than 10 is
            # not skipped but turned into 'G' below (HSP.c:250)
            nz = np.flatnonzero(~amb)
            i = int(nz[0]) if len(nz) else L
            if i < MIN_N_RUN:
                i = 0
            start, ln, ori = useful, 0, i
            # runs of ambiguous characters from i on
            a = amb[i:].astype(np.int8)
            edges = np.flatnonzero(np.diff(np.concatenate([[0], a, [0]])))
            runs = list(zip(edges[0::2] + i, edges[1::2] + i))      # [s, e) ambiguous
            out = []
            for s, e in runs:
                if s > i:                                          # unambiguous stretch
                    out.append(code[i:s])
                    useful += s - i
                    ln += s - i
                i = e
                k = e - s
                if k < MIN_N_RUN:                                  # HSP.c:275-285
                    out.append(np.full(k, 2, np.uint8))
                    useful += k
                    ln += k
                elif i < L:                                        # a new block (HSP.c:287-296)
                    blocks.append((start, useful - 1, i - k - ln))
                    start, ln = useful, 0
                else:                                              # trailing run: cut (HSP.c:298)
                    i -= k
                    break
            else:
                if i < L:
                    out.append(code[i:L])
                    useful += L - i
                    ln += L - i
                    i = L
            blocks.append((start, useful - 1, i - ln))
            if out:
                parts.append(np.concatenate(out))
        ann.append((name, blocks))
        total += L
    codes = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return codes.astype(np.uint8), ann, total


def pac_bytes(codes: np.ndarray, total: int) -> bytes:
    """.pac (HSP.c:313-323): 4 codes per byte, first code in the high bits; then a 0
    byte when total % 4 == 0, then the byte total % 4 -- total counting the records'
    ambiguous characters too."""
    n = len(codes)
    pad = np.zeros((n + 3) // 4 * 4, np.uint8)
    pad[:n] = codes
    packed = (pad.reshape(-1, 4) << np.array([6, 4, 2, 0], np.uint8)).sum(axis=1, dtype=np.uint32).astype(np.uint8)
    tail = (b"\x00" if total % 4 == 0 else b"") + bytes([total % 4])
    return packed.tobytes() + tail


def ann_text(ann, total: int, seed: int = 0) -> str:
    """.ann (HSP.c:325-337).  `seed` is the ini's RandomSeed field (0 without an ini)."""
    lines = [f"{total}\t{len(ann)}\t{seed}"]
    lines += [f"{len(name)}\t{name}" for name, _ in ann]
    lines.append(str(sum(len(b) for _, b in ann)))
    for r, (_, blocks) in enumerate(ann):
        lines += [f"{r}\t{s & 0xFFFFFFFF}\t{e & 0xFFFFFFFF}\t{o & 0xFFFFFFFF}" for s, e, o in blocks]
    return "\n".join(lines) + "\n"


def pac_text(pac: bytes) -> np.ndarray:
    """The text a .pac holds as the BWT construction reads it: (bytes - 2) * 4 + last
    byte codes (TextLengthFromBytePacked), from the packed bytes (zero bits past them)."""
    T = (len(pac) - 2) * 4 + pac[-1]
    raw = np.frombuffer(pac[:-1], np.uint8)
    codes = ((raw[:, None] >> np.array([6, 4, 2, 0], np.uint8)[None, :]) & 3).reshape(-1)
    out = np.zeros(T, np.uint8)
    m = min(T, len(codes))
    out[:m] = codes[:m]
    return out


def reverse_pac(pac: bytes) -> bytes:
    """BuildReversePacked (2BWT-Builder.c:116-213): the text reversed and re-packed 16
    codes per word; the last partial word is written with 1-4 bytes by its code count,
    and a full last word (T % 16 == 0) is never written; then the input's
    length byte."""
    codes = pac_text(pac)
    T = len(codes)
    rev = codes[::-1]
    full = T // 16 * 16 if T % 16 else T - 16           # the codes that leave in whole words
    rem = T - full if T % 16 else 0
    body = pac_bytes(rev[:full], 1)[:-1] if full > 0 else b""   # whole words: 4 bytes each
    if rem:
        nb = 1 if rem < 4 else 2 if rem < 8 else 3 if rem < 12 else 4
        word = np.zeros(16, np.uint8)
        word[:rem] = rev[full:full + rem]
        body += pac_bytes(word, 1)[:nb]
    return body + bytes([pac[-1]])


def _device_bwt(codes: np.ndarray, sa_interval: int = 0, device: int = 0):
    """The BWT of `codes` (and every sa_interval-th SA value) from the device suffix
    sort: (bwt codes, isa0, C[5], SA samples or None)."""
    import torch
    from ._lib import check, lib
    T = len(codes)
    nw = (T + 15) // 16
    text = torch.from_numpy(np.concatenate([index_io.pack_lsb_u32(codes), np.zeros(8, np.uint32)]).view(np.int32)).cuda()
    out = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
    isa0 = C.c_uint64()
    Cc = np.zeros(5, np.uint64)
    ns = (T + sa_interval) // sa_interval if sa_interval else 0
    sa = torch.zeros(max(ns, 1), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    check(lib().hsa_build_bwt_index_device(device, T, text.data_ptr(), out.data_ptr(), C.byref(isa0), Cc,
                                           sa_interval, sa.data_ptr() if ns else None))
    bwt = index_io.unpack_lsb_u32(out.cpu().numpy().view(np.uint32), T)
    return bwt, int(isa0.value), Cc.astype(np.uint32), (sa.cpu().numpy().view(np.uint32)[:ns] if ns else None)


def write_sa(prefix: str, T: int, isa0: int, Cc: np.ndarray, interval: int, sa: np.ndarray) -> None:
    """.sa (BWTSaveSaValue, BWTConstruct.c:1373-1392): inverseSa0, C[1..4], saInterval,
    then SA[0] = T and the samples SA[s], SA[2s], ..."""
    head = np.concatenate([[isa0], np.asarray(Cc, np.uint32)[1:5], [interval]]).astype(np.uint32)
    vals = np.asarray(sa, np.uint32).copy()
    vals[0] = T
    with open(f"{prefix}.index.sa", "wb") as f:
        f.write(head.tobytes())
        f.write(vals.tobytes())


def build_index(fasta: str, prefix: str | None = None, device: int = 0, sa_interval: int = SA_INTERVAL,
                seed: int = 0) -> dict:
    """Write every `HSA index` file of `fasta` under `prefix` (default: the FASTA path):
    prefix.index.{pac,ann,rev.pac,bwt,fmv,rev.bwt,rev.fmv,sa}.  Returns the lengths."""
    prefix = prefix or fasta
    with open(fasta, "rb") as f:
        data = f.read()
    codes, ann, total = parse_fasta(data)
    pac = pac_bytes(codes, total)
    rpac = reverse_pac(pac)
    with open(f"{prefix}.index.pac", "wb") as f:
        f.write(pac)
    with open(f"{prefix}.index.rev.pac", "wb") as f:
        f.write(rpac)
    with open(f"{prefix}.index.ann", "w") as f:
        f.write(ann_text(ann, total, seed))
    text = pac_text(pac)
    bwt, isa0, Cc, sa = _device_bwt(text, sa_interval, device)
    index_io.write_bwt_files(prefix, len(text), isa0, Cc, bwt)
    write_sa(prefix, len(text), isa0, Cc, sa_interval, sa)
    rtext = pac_text(rpac)
    rbwt, risa0, rCc, _ = _device_bwt(rtext, 0, device)
    index_io.write_bwt_files(prefix, len(rtext), risa0, rCc, rbwt, suffix=".rev")
    return {"T": len(text), "rev_T": len(rtext), "records": len(ann), "characters": total}


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="Build the 2BWT index files of a FASTA on the GPU "
                                             "(byte-identical to `HSA index`).")
    ap.add_argument("fasta")
    ap.add_argument("--prefix", default=None)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--sa-interval", type=int, default=SA_INTERVAL)
    a = ap.parse_args(argv)
    print(build_index(a.fasta, a.prefix, a.device, a.sa_interval))


if __name__ == "__main__":
    main()
