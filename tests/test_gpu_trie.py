"""The root tries (hsa_amd/csrc/hsa_trie.h): k_search answers the steps of strings
shorter than the trie depth D from the search trie (ungapped regimes: expansions from
the child masks and the last level, exact tails in one jump with the L field's step
count), k_widths the first D steps after each reset from the width trie.  Every search
must equal the oracle's bit for bit -- hits, flags, pops and the rank-query count --
whatever D, including tries far deeper than the text (most strings empty: the L
accounting of exact tails that empty inside the trie) and D = 0 (no trie)."""
import numpy as np
import pytest

from golden_io import INDEX, split_hits
from hsa_amd import index_io

pytestmark = pytest.mark.gpu

# (case, options): the ungapped golden cases, and gapped read sets searched ungapped
CASES = [("tiny_mm100_n4o0", None), ("tiny_exact36_n0", None), ("tiny_gap100_n4o1", "-n 4 -o 0"),
         ("rep_mm100_n4o1", "-n 4 -o 0"), ("tiny_edge_default", "-n 3 -o 0"), ("tiny_opts_seed", "-n 4 -o 0 -l 20 -k 1")]


def _index(genome, depth, monkeypatch, mode=1):
    """An index with width-trie depth `depth` and, for mode >= 1, a search trie of the
    same depth (k_search uses it under the same HSA_TRIE_MODE)."""
    from hsa_amd._lib import GpuIndex
    monkeypatch.setenv("HSA_TRIE_DEPTH", str(depth))
    monkeypatch.setenv("HSA_TRIE_SDEPTH", str(depth))
    monkeypatch.setenv("HSA_TRIE_MODE", str(mode))
    return GpuIndex(*index_io.read_index(INDEX[genome]))


@pytest.mark.parametrize("depth,mode", [(0, 1), (3, 1), (9, 1), (12, 1), (9, 2), (12, 0)])
@pytest.mark.parametrize("case,args", CASES)
def test_trie_search_matches_oracle(case, args, depth, mode, monkeypatch):
    """mode 1: both tries; 2: exact tails one trie level per step; 0: the width trie
    only (the default)."""
    from golden_io import load_case
    from test_gpu_parity import _device_run
    ix = _index(load_case(case)["index"], depth, monkeypatch, mode)
    got, (e_n, e_f, e_h, st) = _device_run(case, ix=ix, args=args)
    assert got["c"][11] == 0
    assert np.array_equal(got["f"] & 1, e_f & 1)
    assert np.array_equal(got["n"], e_n)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(exp)) if not np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)],
                                                             exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"
    assert int(got["c"][2]) == int(st[0]), ("rank queries", int(got["c"][2]), int(st[0]))
    assert int(got["c"][4]) == int(st[1]), "gap_pop count"
    if depth == 0:
        assert got["c"][10] == 0
    else:
        assert got["c"][10] > 0, "no step answered from the tries"


def test_trie_off_switch(monkeypatch):
    """HSA_TRIE=0 at search time: rank steps only, the same results."""
    from test_gpu_parity import _device_run
    ix = _index("tiny", 9, monkeypatch)
    on, (e_n, _, _, st) = _device_run("tiny_mm100_n4o0", ix=ix)
    monkeypatch.setenv("HSA_TRIE", "0")
    off, _ = _device_run("tiny_mm100_n4o0", ix=ix)
    assert on["c"][10] > 0 and off["c"][10] == 0
    assert int(on["c"][2]) == int(off["c"][2]) == int(st[0])
    assert np.array_equal(on["n"], off["n"]) and np.array_equal(on["n"], e_n)
