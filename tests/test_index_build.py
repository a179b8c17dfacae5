"""The index builder's host half (hsa_amd/index_build.py): FASTA -> .pac / .ann /
.rev.pac, byte-identical to the files the reference's `HSA index` wrote for the same
FASTA (tests/golden/index/, E.coli-sized digests in manifest_ecoli.json).  The FASTAs
are regenerated with the generators that made them (tools/make_golden.py)."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from golden_io import GOLD, INDEX
from hsa_amd import index_build, synth

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def fasta(name, path):
    import make_golden as mg
    if name == "tiny":
        T = 200003
        synth.write_fasta(path, synth.genome_codes(T, 7), synth.record_layout(T, 3))
    elif name == "rep":
        synth.write_fasta(path, mg.repeat_genome(50001, 11), synth.record_layout(50001, 1))
    elif name == "nrun":
        mg.nrun_genome_fasta(path)
    elif name == "ecoli":
        T = 4641652
        synth.write_fasta(path, synth.genome_codes(T, 42), synth.record_layout(T, 1))
    return path


def host_files(path):
    codes, ann, total = index_build.parse_fasta(open(path, "rb").read())
    pac = index_build.pac_bytes(codes, total)
    return pac, index_build.reverse_pac(pac), index_build.ann_text(ann, total)


@pytest.mark.parametrize("name", ["tiny", "rep", "nrun"])
def test_pac_ann_rev_match_reference(tmp_path, name):
    pac, rpac, ann = host_files(fasta(name, str(tmp_path / f"{name}.fa")))
    pre = os.path.join(GOLD, "index", f"{name}.fa.index")
    assert pac == open(pre + ".pac", "rb").read()
    assert rpac == open(pre + ".rev.pac", "rb").read()
    assert ann == open(pre + ".ann").read()


def test_ecoli_pac_digests(tmp_path):
    man = json.load(open(os.path.join(GOLD, "manifest_ecoli.json")))
    pac, rpac, _ = host_files(fasta("ecoli", str(tmp_path / "ecoli.fa")))
    assert hashlib.sha256(pac).hexdigest() == man["index_sha256"]["pac"]
    assert hashlib.sha256(rpac).hexdigest() == man["index_sha256"]["rev.pac"]


def test_text_lengths_and_quirks():
    """a text of 16k characters loses 20 in the reversed index; the .pac
    length byte counts ambiguous characters (HSP.c:311) while the packed text does not."""
    g = synth.genome_codes(1600, 3)
    rec = b">r\n" + bytes(b"ACGT"[int(c)] for c in g) + b"\n"
    codes, ann, total = index_build.parse_fasta(rec)
    pac = index_build.pac_bytes(codes, total)
    assert len(index_build.pac_text(pac)) == 1600
    assert len(index_build.pac_text(index_build.reverse_pac(pac))) == 1580
    assert np.array_equal(index_build.pac_text(index_build.reverse_pac(pac)), g[::-1][:1580])
    # 101 bases + a 9-base N-run turned into G + 2 bases + 13 N cut at the end: 112
    # packed, 125 counted -> the length byte says 125 % 4 = 1: the text read back from
    # the .pac is (29 - 2) * 4 + 1 = 109 characters
    seq = bytes(b"ACGT"[int(c)] for c in g[:101]) + b"N" * 9 + b"AC" + b"N" * 13
    codes, ann, total = index_build.parse_fasta(b">x y\n" + seq + b"\n>short\nACGT\n")
    assert total == len(seq) == 125 and len(codes) == 112 and ann[0][0] == "x"
    assert len(ann) == 1 and ann[0][1] == [(0, 111, 0)]
    assert np.array_equal(codes[101:110], np.full(9, 2))
    assert len(index_build.pac_text(index_build.pac_bytes(codes, total))) == 109
