"""Device BWT construction (hsa_build_bwt_device) against the reference's own index
files, and the device synthetic genome against hsa_amd/synth.py."""
import ctypes as C
import os

import numpy as np
import pytest

from golden_io import GOLD, INDEX
from hsa_amd import index_io, synth

pytestmark = pytest.mark.gpu


def _build(codes, reverse):
    import torch
    from hsa_amd._lib import check, lib
    T = len(codes)
    text = torch.from_numpy(index_io.pack_lsb_u32(codes).view(np.int32)).cuda()
    out = torch.zeros((T + 15) // 16 + 4, dtype=torch.int32, device="cuda")
    isa0 = C.c_uint32()
    Cc = np.zeros(5, np.uint32)
    torch.cuda.synchronize()
    check(lib().hsa_build_bwt_device(0, T, text.data_ptr(), reverse, out.data_ptr(), C.byref(isa0), Cc))
    w = out.cpu().numpy().view(np.uint32)
    return index_io.unpack_lsb_u32(w, T), int(isa0.value), Cc


@pytest.mark.parametrize("name", ["tiny", "rep"])
def test_bwt_build_matches_reference_files(name):
    fwd, rev = index_io.read_index(INDEX[name])
    text = index_io.read_pac(INDEX[name])
    for ref, reverse in ((fwd, 0), (rev, 1)):
        codes, isa0, Cc = _build(text, reverse)
        assert isa0 == ref.isa0
        assert np.array_equal(Cc, ref.C)
        assert np.array_equal(codes, index_io.unpack_codes(ref))


def test_bwt_build_small_edge_texts():
    """Run-off ties ('$' ordering), homopolymers and tiny lengths vs a direct sort."""
    def naive(codes):
        T = len(codes)
        s = codes.tobytes()
        order = sorted(range(T), key=lambda i: s[i:])
        rows = [T] + order
        isa0 = rows.index(0)
        bwt = [codes[(r - 1) % T] if r != 0 else None for r in rows]
        return np.array([b for b in bwt if b is not None], np.uint8), isa0
    for codes in (np.zeros(37, np.uint8), np.array([0, 1] * 40 + [0], np.uint8),
                  synth.genome_codes(1000, 3), np.array([3, 2, 1, 0, 0, 1, 2, 3] * 9 + [1], np.uint8)):
        got, isa0, _ = _build(codes, 0)
        exp, eisa0 = naive(codes)
        assert isa0 == eisa0 and np.array_equal(got, exp)


def test_synth_genome_device_matches_host():
    import torch
    from hsa_amd._lib import check, lib
    for T in (1, 31, 32, 1000, 100003):
        out = torch.zeros((T + 15) // 16 + 2, dtype=torch.int32, device="cuda")
        check(lib().hsa_synth_genome_device(0, T, 1234, out.data_ptr()))
        got = index_io.unpack_lsb_u32(out.cpu().numpy().view(np.uint32), T)
        assert np.array_equal(got, synth.genome_codes(T, 1234))


@pytest.mark.parametrize("name", ["tiny", "rep", "nrun"])
def test_full_index_build_matches_reference(tmp_path, name):
    """hsa_amd/index_build.py: FASTA -> every file `HSA index` writes (.pac .ann .rev.pac
    .bwt .fmv .rev.bwt .rev.fmv .sa), suffix sorting and SA sampling on the device,
    byte-identical to the reference's files for the same FASTA (nrun: N-runs that split
    blocks, short runs turned into G, the .pac length byte counting the Ns)."""
    from test_index_build import fasta
    from hsa_amd import index_build
    fa = fasta(name, str(tmp_path / f"{name}.fa"))
    index_build.build_index(fa)
    for e in ("pac", "ann", "rev.pac", "bwt", "fmv", "rev.bwt", "rev.fmv", "sa"):
        got = open(f"{fa}.index.{e}", "rb").read()
        exp = open(os.path.join(GOLD, "index", f"{name}.fa.index.{e}"), "rb").read()
        assert got == exp, f"{name}.index.{e} differs ({len(got)} vs {len(exp)} bytes)"


def test_full_index_build_ecoli_digests(tmp_path):
    """The E.coli-sized genome (4.6 Mbp): every index file's SHA-256 equals the
    reference's (manifest_ecoli.json)."""
    import hashlib
    import json
    from test_index_build import fasta
    from hsa_amd import index_build
    man = json.load(open(os.path.join(GOLD, "manifest_ecoli.json")))
    fa = fasta("ecoli", str(tmp_path / "ecoli.fa"))
    index_build.build_index(fa)
    for e, digest in man["index_sha256"].items():
        assert hashlib.sha256(open(f"{fa}.index.{e}", "rb").read()).hexdigest() == digest, e
