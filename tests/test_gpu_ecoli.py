"""E.coli-sized parity (BASELINE config 1 and two heavier flavours): the genome is
regenerated on the device, indexed by the device BWT builder, and both the index
files and the search results are checked against SHA-256 digests the compiled
reference produced on the same inputs (tests/golden/manifest_ecoli.json)."""
import ctypes as C
import hashlib

import numpy as np
import pytest

from golden_io import ecoli_manifest, main_path_digest, parse_opts
from hsa_amd import index_io, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ecoli():
    import torch
    from hsa_amd import _lib
    man = ecoli_manifest()
    T, seed = man["genome"]["T"], man["genome"]["seed"]
    L = _lib.lib()
    nw = (T + 15) // 16
    text = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
    _lib.check(L.hsa_synth_genome_device(0, T, seed, text.data_ptr()))
    out = {}
    for rev in (0, 1):
        bw = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
        isa0 = C.c_uint32()
        Cc = np.zeros(5, np.uint32)
        _lib.check(L.hsa_build_bwt_device(0, T, text.data_ptr(), rev, bw.data_ptr(), C.byref(isa0), Cc))
        out[rev] = (bw, int(isa0.value), Cc)
    gi = _lib.GpuIndex.from_device_codes(T, out[0][1], out[0][2], out[0][0].data_ptr(),
                                         T, out[1][1], out[1][2], out[1][0].data_ptr())
    return man, gi, out


def test_index_files_byte_identical(ecoli, tmp_path):
    man, gi, out = ecoli
    T = man["genome"]["T"]
    for rev, suf in ((0, ""), (1, ".rev")):
        bw, isa0, Cc = out[rev]
        codes = index_io.unpack_lsb_u32(bw.cpu().numpy().view(np.uint32), T)
        index_io.write_bwt_files(str(tmp_path / "e"), T, isa0, Cc, codes, suf)
        for ext in ("bwt", "fmv"):
            got = hashlib.sha256(open(tmp_path / f"e.index{suf}.{ext}", "rb").read()).hexdigest()
            assert got == man["index_sha256"][suf.lstrip(".") + ("." if suf else "") + ext], (suf, ext)


@pytest.mark.parametrize("case", ["ecoli_exact36_n0", "ecoli_mm100_n4o0", "ecoli_gap100_n4o1"])
def test_search_digest_matches_reference(ecoli, case):
    from hsa_amd._lib import GapOpt
    man, gi, _ = ecoli
    c = man[case]
    T, seed = man["genome"]["T"], man["genome"]["seed"]
    g = synth.genome_codes(T, seed)
    reads, _ = synth.make_reads(g, synth.record_layout(T, 1), c["n"], c["L"], c["read_seed"], **c["kw"])
    lens = np.full(c["n"], c["L"], np.uint32)
    n_aln, flags, per_read, _ = gi.run_batches(lens, reads.reshape(-1), parse_opts(c["args"],
                                                GapOpt.default().as_dict()), 100000)
    hits = np.concatenate([p for p in per_read if len(p)]) if any(len(p) for p in per_read) else np.zeros((0, 9))
    assert int((flags & 1).sum()) == c["splice_calls"]
    assert main_path_digest(n_aln, flags, hits) == c["sha256"]
