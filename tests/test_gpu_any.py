"""k_search_any (hsa_amd/csrc/hsa_search_any.h): the search for reads and options past
k_search's fixed layouts -- reads longer than 1 023 bases, n_stacks past 512, more than
128 reachable scores, more than 14 gap opens, max_diff past 125.  The reference accepts
them all (bwa_seq_t.len:19, bwtaln.h:96; gap_entry_t.info's 16-bit position,
bwtgap.c:157), so the drop-in must serve them, on the device.

* golden cases recorded from the compiled reference (tools/make_golden.py --limits,
  manifest_limits.json): 1 100-1 500 bp reads mixed with 100 bp ones (-n 8 -o 1),
  -n 4 -o 2 -e 60 (298 scores, 250 reachable), -n 16 -o 15;
* every tiny golden case with HSA_FORCE_ANY set, i.e. k_search_any alone against the
  reference's hits, and the bwt_match_gap calls the reference's splice path made;
* the device path (hsa_search_device: long reads partitioned on the device) against the
  oracle, rank queries and pops included."""
import numpy as np
import pytest

from golden_io import cases, limits_cases, load_case, parse_opts, split_hits
from test_gpu_parity import _compare, _device_run

pytestmark = pytest.mark.gpu


@pytest.fixture
def verbose(monkeypatch):
    monkeypatch.setenv("HSA_VERBOSE", "1")
    monkeypatch.delenv("HSA_FORCE_ANY", raising=False)


@pytest.mark.parametrize("name", sorted(limits_cases().keys()))
def test_limits_cases_match_reference(name, verbose, capfd):
    """The drop-in's batch path (hsa_cal_sa_reg_gap_flat) on the limit cases: every
    read's bwt_aln1_t list equals the reference's, splice-fallback flags agree, and
    k_search_any is what served the out-of-layout reads."""
    _compare(name)
    assert "k_search_any" in capfd.readouterr().err


@pytest.mark.parametrize("name", sorted(cases().keys()))
def test_forced_any_matches_reference(name, monkeypatch):
    """Every tiny golden case (Q1-Q13 quirks, NONSTOP, top-2, capacity bounds) through
    k_search_any alone."""
    monkeypatch.setenv("HSA_FORCE_ANY", "1")
    _compare(name)


def test_forced_any_match_gap_calls(monkeypatch):
    """Direct bwt_match_gap calls with the caller's widths (the splice path's seeds and
    anchors, aliased and NULL width_seed) through k_search_any: hits and the widths
    after gap_shadow equal the reference's."""
    from test_gpu_match_gap import run_calls
    from golden_io import load_mgcap
    from hsa_amd import _lib, index_io
    from golden_io import INDEX
    monkeypatch.setenv("HSA_FORCE_ANY", "1")
    gi = _lib.GpuIndex(*index_io.read_index(INDEX["tiny"]))
    for name in ("mgcap_default", "mgcap_n4o1"):
        calls = load_mgcap(name)
        out = run_calls(gi, calls)
        bad = [j for j, c in enumerate(calls) if not (np.array_equal(out[id(c)][0], c["hits"]) and
                                                       np.array_equal(out[id(c)][1], c["wo"]))]
        assert not bad, f"{name}: {len(bad)} of {len(calls)} calls differ; first {bad[0]}"


@pytest.mark.parametrize("name", ["long1500_n8o1", "gap100_o2e60", "gap100_o15"])
def test_device_path_limits_match_oracle(name, verbose, capfd):
    """hsa_search_device on a device-resident batch: the long reads of a mixed batch
    are split off on the device (k_partition) and searched by k_search_any after
    k_search has taken the others; an out-of-layout regime sends every read there.
    Every hit, the fallback flags, and the rank-query and pop counts equal the oracle's."""
    got, (e_n, e_f, e_h, st) = _device_run(name)
    assert "k_search_any" in capfd.readouterr().err
    assert got["c"][11] == 0
    assert np.array_equal(got["f"] & 1, e_f & 1)
    assert np.array_equal(got["n"], e_n)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(exp)) if not np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)],
                                                             exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"
    if got["c"][8] == 0:
        assert int(got["c"][2]) == int(st[0]), (int(got["c"][2]), int(st[0]))
        assert int(got["c"][4]) == int(st[1]), "gap_pop count"


def test_device_path_limits_64bit(verbose, capfd):
    """The 64-bit instantiation of k_search_any (hsa_search_device64) on the long-read
    case: the 64-bit restatement's hits."""
    import test_gpu_wide as W
    from oracle_ctypes import Opt, OracleIndex64, default_opt
    from hsa_amd import index_io
    from golden_io import INDEX
    g = load_case("long1500_n8o1")
    od = parse_opts(g["args"], default_opt())
    od["mode"] &= ~0x01
    lens, codes = W._device_jobs(g, od)
    n64, f64, o64, h64, c64 = W.search(W.index64("tiny"), lens, codes, od, True)
    assert "k_search_any" in capfd.readouterr().err
    e_n, e_f, e_h, st = OracleIndex64.from_index(*index_io.read_index(INDEX["tiny"])).cal_sa_reg_gap(
        lens, codes, Opt.from_dict(od))
    assert np.array_equal(n64, e_n) and np.array_equal(f64 & 1, e_f & 1)
    got = W.per_read(n64, o64, h64)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(got)) if not np.array_equal(got[i], exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"
