"""The root width trie (hsa_amd/csrc/hsa_trie.h): k_widths answers the first D steps
after each reset of bwt_cal_width's chain (bwtaln.c:84-97) from the trie.  Every search
must equal the oracle's bit for bit -- hits, flags, pops and the rank-query count --
whatever D, including tries far deeper than the text (most strings empty) and D = 0
(no trie)."""
import numpy as np
import pytest

from golden_io import INDEX, split_hits
from hsa_amd import index_io

pytestmark = pytest.mark.gpu

# (case, options): the ungapped golden cases, and gapped read sets searched ungapped
CASES = [("tiny_mm100_n4o0", None), ("tiny_exact36_n0", None), ("tiny_gap100_n4o1", "-n 4 -o 0"),
         ("rep_mm100_n4o1", "-n 4 -o 0"), ("tiny_edge_default", "-n 3 -o 0"), ("tiny_opts_seed", "-n 4 -o 0 -l 20 -k 1")]


def _index(genome, depth, monkeypatch):
    """An index with a width trie of `depth` levels."""
    from hsa_amd._lib import GpuIndex
    monkeypatch.setenv("HSA_TRIE_DEPTH", str(depth))
    return GpuIndex(*index_io.read_index(INDEX[genome]))


@pytest.mark.parametrize("depth", [0, 3, 9, 12])
@pytest.mark.parametrize("case,args", CASES)
def test_trie_search_matches_oracle(case, args, depth, monkeypatch):
    from golden_io import load_case
    from test_gpu_parity import _device_run
    ix = _index(load_case(case)["index"], depth, monkeypatch)
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
        assert got["c"][10] > 0, "no step answered from the trie"


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
