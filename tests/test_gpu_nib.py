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
