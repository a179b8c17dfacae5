"""The unique-interval walk (hsa_index_build_walk; k_search PH_WALK): an ungapped
search node whose interval holds one suffix is matched against the text -- SA[k], text
chunks, ISA[p] -- instead of one rank pair per position.  The searches must equal the
oracle's bit for bit -- hits, flags, the rank-query and the pop counts (the walk counts
the expansions and virtual-top pops the reference makes) -- with the walk's arrays
derived from the reference's own sampled .sa and the BWT (the drop-in's case), and with
the walk forced onto every one-suffix node (HSA_WALK_MIN=1).  The product build
compiles the walk out (measured slower): there these tests check that the
arrays build and the searches stay exact; a -DHSA_UNIQUE_WALK=1 build
(tools/build_variant.sh, HSA_GPU_LIB) runs them on the walk itself."""
import numpy as np
import pytest

from golden_io import INDEX, load_case, split_hits
from hsa_amd import index_io

pytestmark = pytest.mark.gpu

CASES = [("tiny_mm100_n4o0", None), ("tiny_exact36_n0", None), ("tiny_gap100_n4o1", "-n 4 -o 0"),
         ("rep_mm100_n4o1", "-n 4 -o 0"), ("tiny_edge_default", "-n 3 -o 0"), ("tiny_opts_seed", "-n 4 -o 0 -l 20 -k 1"),
         ("tiny_mm100_n4o0", "-n 6 -o 0 -N")]

_IX = {}


def _walk_index(genome):
    from hsa_amd._lib import GpuIndex
    if genome not in _IX:
        gi = GpuIndex(*index_io.read_index(INDEX[genome]))
        gi.set_sa(index_io.read_sa(INDEX[genome]), index_io.read_blocks(INDEX[genome]))
        gi.build_walk()
        _IX[genome] = gi
    return _IX[genome]


@pytest.mark.parametrize("wmin,streak", [("8", "2"), ("1", "0")])
@pytest.mark.parametrize("case,args", CASES)
def test_walk_search_matches_oracle(case, args, wmin, streak, monkeypatch):
    """The default trigger (8 positions left, 2 one-suffix match steps in a row), and the
    walk on every one-suffix node (1, 0)."""
    from test_gpu_parity import _device_run
    monkeypatch.setenv("HSA_WALK_MIN", wmin)
    monkeypatch.setenv("HSA_WALK_STREAK", streak)
    monkeypatch.setenv("HSA_SPLIT", "0")
    ix = _walk_index(load_case(case)["index"])
    got, (e_n, e_f, e_h, st) = _device_run(case, ix=ix, args=args)
    assert got["c"][11] == 0
    assert np.array_equal(got["f"] & 1, e_f & 1)
    assert np.array_equal(got["n"], e_n)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(exp)) if not np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)],
                                                             exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"
    assert int(got["c"][2]) == int(st[0]), ("rank queries", int(got["c"][2]), int(st[0]))
    assert int(got["c"][4]) == int(st[1]), ("pops", int(got["c"][4]), int(st[1]))


def test_walk_off_switch(monkeypatch):
    """HSA_WALK=0 at search time: rank steps only; the same results and counts."""
    from test_gpu_parity import _device_run
    monkeypatch.setenv("HSA_SPLIT", "0")
    ix = _walk_index("tiny")
    on, (e_n, _, _, st) = _device_run("tiny_mm100_n4o0", ix=ix)
    monkeypatch.setenv("HSA_WALK", "0")
    off, _ = _device_run("tiny_mm100_n4o0", ix=ix)
    assert int(on["c"][2]) == int(off["c"][2]) == int(st[0])
    assert int(on["c"][4]) == int(off["c"][4]) == int(st[1])
    assert np.array_equal(on["n"], off["n"]) and np.array_equal(on["n"], e_n)
