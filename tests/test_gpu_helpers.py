"""Helpers in the strand-split main pass (k_search, SearchArgs::fr_*): lanes that find the
queue empty search sub-trees of the strands still running, and an owner whose offered
entries all end without a hit stops with no hits.  Before a hit a strand search expands
the same entries in any order (bwtgap.c:144-331: only a hit changes max_diff, the widths
(gap_shadow) or the best_score break), so the answers, the rank-query count and the pop
count stay the reference's.  Forced here on the golden cases with a tiny budget and no
demand threshold, so that nearly every strand offers its entries at once."""
import numpy as np
import pytest

from golden_io import cases, load_case, parse_opts, split_hits

pytestmark = pytest.mark.gpu

# -m 40: max_entries below the pool, the helpers stay off (help_args); every other case
CASES = sorted(k for k in cases().keys() if k != "tiny_opts_maxentries")


def _force(monkeypatch, budget="16"):
    monkeypatch.setenv("HSA_SPLIT", "1")
    monkeypatch.setenv("HSA_HELP", "1")
    monkeypatch.setenv("HSA_HELP_BUDGET", budget)
    monkeypatch.setenv("HSA_HELP_DEMAND", "0")
    monkeypatch.setenv("HSA_VERBOSE", "1")


def _gapped(name):
    """Helpers run in the gapped 32-bit kernels only (k_search's FRH): gap opens allowed
    (max_gapo > 0, and max_diff not 0, which clears them, bwtaln.c:256)."""
    from oracle_ctypes import default_opt
    o = parse_opts(load_case(name)["args"], default_opt())
    return o["max_gapo"] > 0 and o["max_diff"] != 0


def _helper_stats(err):
    lines = [ln for ln in err.splitlines() if ln.startswith("[hsa] helpers:")]
    tot = np.zeros(6, np.int64)
    for ln in lines:
        w = ln.replace("(", " ").replace(")", " ").replace(",", " ").split()
        nums = [int(x) for x in w if x.isdigit()]
        tot += np.array(nums[:6])
    return dict(offers=tot[0], refused=tot[1], entries=tot[2], subsearches=tot[3], answered=tot[4], queries=tot[5])


@pytest.mark.parametrize("name", CASES)
def test_helpers_match_reference(name, monkeypatch, capfd):
    """The drop-in path (host arrays, the reference's batches) with helpers forced: every
    read's hits and fallback flag equal the compiled reference's golden output."""
    from test_gpu_parity import _compare
    _force(monkeypatch)
    _compare(name)
    st = _helper_stats(capfd.readouterr().err)
    if name.startswith(("tiny_gap", "rep_gap", "rep_mm", "rep_deep")):   # deep enough to outlast the budget
        assert st["offers"] > 0 and st["subsearches"] > 0, st


@pytest.mark.parametrize("case", ["tiny_mm100_n4o0", "tiny_gap100_n4o1", "rep_mm100_n4o1", "rep_gap60_R2",
                                  "tiny_opts_scores", "tiny_edge_n3o1e3L"])
def test_helpers_keep_rank_queries_and_pops(case, monkeypatch, capfd):
    """The device path with helpers forced: hits, flags, and the rank-query and pop counts
    (d_counters[2], [4]) equal the oracle's, and some strands were answered by helpers."""
    from test_gpu_parity import _device_run
    _force(monkeypatch)
    got, (e_n, e_f, e_h, st) = _device_run(case)
    hs = _helper_stats(capfd.readouterr().err)
    assert got["c"][8] == 0
    assert np.array_equal(got["n"], e_n) and np.array_equal(got["f"] & 1, e_f & 1)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(exp)) if not np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)],
                                                             exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"
    assert int(got["c"][2]) == int(st[0]), (int(got["c"][2]), int(st[0]), hs)
    assert int(got["c"][4]) == int(st[1]), ("gap_pop count", hs)
    print(case, hs)
    # (whether an owner is answered by its helpers before it ends by itself depends on
    # timing; the drop-in's long no-hit searches answer thousands: profiles/r06_helpers_ab.log)
    if _gapped(case):
        assert hs["offers"] > 0 and hs["subsearches"] > 0, hs


@pytest.mark.parametrize("budget", ["1", "64"])
def test_helpers_budgets(budget, monkeypatch, capfd):
    """Other budgets (1: a strand offers its entries on its first poll; 64) on the deepest
    gapped case: the reference's answers and counts."""
    from test_gpu_parity import _device_run
    _force(monkeypatch, budget)
    got, (e_n, e_f, e_h, st) = _device_run("rep_gap60_R2")
    capfd.readouterr()
    assert np.array_equal(got["n"], e_n) and np.array_equal(got["f"] & 1, e_f & 1)
    assert int(got["c"][2]) == int(st[0]) and int(got["c"][4]) == int(st[1])


def test_helpers_small_frontier(monkeypatch, capfd):
    """A frontier of 64 entries: most offers are refused (the strand searches on alone)
    and the answers stay exact."""
    from test_gpu_parity import _device_run
    _force(monkeypatch)
    monkeypatch.setenv("HSA_HELP_CAP", "64")
    got, (e_n, e_f, e_h, st) = _device_run("tiny_gap100_n4o1")
    hs = _helper_stats(capfd.readouterr().err)
    assert hs["refused"] > 0, hs
    assert np.array_equal(got["n"], e_n) and np.array_equal(got["f"] & 1, e_f & 1)
    assert int(got["c"][2]) == int(st[0]) and int(got["c"][4]) == int(st[1])
