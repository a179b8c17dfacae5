"""k_search with 4-bit pruning elements (WFmt<WNib>, hsa_search_kernels.h): the layout
long reads get when the 8-bit rows leave the CU short of 16 waves.  HSA_WFMT=nib forces
it wherever it is exact (bid bounds <= 6), so the golden cases -- short reads that would
otherwise use 8-bit rows -- run through it; HSA_VERBOSE's launch line shows that they did."""
import numpy as np
import pytest

from golden_io import cases, load_case, parse_opts, split_hits
from test_gpu_parity import _compare, _device_run

pytestmark = pytest.mark.gpu


@pytest.fixture
def nib(monkeypatch):
    monkeypatch.setenv("HSA_WFMT", "nib")
    monkeypatch.setenv("HSA_VERBOSE", "1")


def _eligible(name):
    from oracle_ctypes import default_opt
    o = parse_opts(load_case(name)["args"], default_opt())
    return 0 <= o["max_diff"] <= 6 and o["max_seed_diff"] <= 6


@pytest.mark.parametrize("name", sorted(cases().keys()))
def test_search_matches_reference_4bit(name, nib, capfd):
    _compare(name)
    err = capfd.readouterr().err
    if _eligible(name):
        assert "4-bit rows" in err, "the 4-bit layout was not used"


@pytest.mark.parametrize("case", ["tiny_mm100_n4o0", "tiny_gap100_n4o1", "rep_mm100_n4o1", "tiny_edge_n3o1e3L"])
def test_device_path_4bit_matches_oracle(case, nib, capfd):
    """hsa_search_device (the bench's path) under the 4-bit layout: every hit, the
    splice-fallback flags and the rank-query / pop counts equal the oracle's (an N in
    an exact tail drops its speculative rank step from the count)."""
    got, (e_n, e_f, e_h, st) = _device_run(case)
    assert "4-bit rows" in capfd.readouterr().err
    assert np.array_equal(got["f"] & 1, e_f & 1)
    assert np.array_equal(got["n"], e_n)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(exp)) if not np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)],
                                                             exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"
    if got["c"][8] == 0:
        assert int(got["c"][2]) == int(st[0]), (int(got["c"][2]), int(st[0]))
        assert int(got["c"][4]) == int(st[1]), "gap_pop count"


def test_device_path_4bit_rerun_is_exact(nib):
    """The big re-run pass uses the 4-bit layout too (the huge pass keeps 8-bit rows)."""
    got, (e_n, e_f, e_h, _) = _device_run("tiny_gap100_n4o1", pool_entries=8)
    assert got["c"][8] > 0 and got["c"][11] == 0
    assert np.array_equal(got["n"], e_n)
    exp = split_hits(e_n, e_h)
    assert all(np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)], exp[i]) for i in range(len(exp)))


@pytest.mark.parametrize("index,opts", [("tiny", ["-n", "4", "-o", "0"]), ("rep", ["-n", "3", "-o", "0", "-l", "40"])])
def test_long_reads_pick_4bit_and_match_oracle(index, opts, monkeypatch, capfd):
    """250 bp reads (0-4 substitutions, half reverse-complemented, a few with an N)
    drawn from the golden index's own text: the planner picks 4-bit rows by itself
    (8-bit rows of 250 bp leave the CU at 8 waves) and every hit equals the oracle's."""
    from hsa_amd import index_io
    from hsa_amd._lib import GapOpt
    from golden_io import INDEX
    from oracle_ctypes import Opt, OracleIndex, default_opt
    from test_gpu_parity import gpu_index
    monkeypatch.setenv("HSA_VERBOSE", "1")
    monkeypatch.delenv("HSA_WFMT", raising=False)
    fwd, rev = index_io.read_index(INDEX[index])
    text = index_io.read_pac(INDEX[index], fwd.T)
    rng = np.random.default_rng(250)
    L, n = 250, 3000
    reads = []
    for r in range(n):
        s = int(rng.integers(0, len(text) - L))
        q = text[s:s + L].astype(np.uint8).copy()
        for p in rng.choice(L, int(rng.integers(0, 5)), replace=False):
            q[p] = (q[p] + rng.integers(1, 4)) & 3
        if r % 2:
            q = (3 - q[::-1]).astype(np.uint8)
        if r % 97 == 0:
            q[int(rng.integers(0, L))] = 4
        reads.append(q)
    codes = np.concatenate(reads)
    lens = np.full(n, L, np.uint32)
    od = parse_opts(opts, default_opt())
    e_n, e_f, e_h, _ = OracleIndex(fwd, rev).cal_sa_reg_gap(lens, codes, Opt.from_dict(od))
    ix = gpu_index(index)
    n_aln, flags, hoff, hits, _ = ix.cal_sa_reg_gap(lens, codes, GapOpt.from_dict(od))
    assert "4-bit rows" in capfd.readouterr().err
    assert np.array_equal(flags & 1, e_f & 1)
    assert np.array_equal(n_aln, e_n)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(n) if not np.array_equal(hits[int(hoff[i]):int(hoff[i]) + max(int(n_aln[i]), 0)], exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"
    assert (n_aln > 0).sum() > n // 2
