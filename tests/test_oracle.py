"""Pin the CPU restatement (oracle/) against the compiled reference's golden vectors."""
import numpy as np
import pytest

from golden_io import EXTCAP_CASES, GOLD, INDEX, cases, limits_cases, load_case, load_extcap, parse_opts, split_hits
from hsa_amd import index_io
from oracle_ctypes import Opt, OracleIndex, default_opt

_IDX = {}


def oracle_index(name):
    if name not in _IDX:
        _IDX[name] = OracleIndex(*index_io.read_index(INDEX[name]))
    return _IDX[name]


def test_occ_matches_reference_all_positions():
    from golden_io import GOLD
    g = np.load(f"{GOLD}/tiny_occ.npz")
    ix = oracle_index("tiny")
    for d in (0, 1):
        got = np.stack([ix.occ4(d, int(p)) for p in g["pos"]])
        assert np.array_equal(got, g["occ"][d]), f"dir {d}"


def test_occ_is_prefix_count():
    """BWTOccValue == #{p < i - [i > isa0] : code[p] == c} (BWT.c:682-716)."""
    fwd, rev = index_io.read_index(INDEX["rep"])
    ix = oracle_index("rep")
    for d, b in enumerate((fwd, rev)):
        codes = index_io.unpack_codes(b)
        pref = np.zeros((b.T + 1, 4), np.int64)
        for c in range(4):
            pref[1:, c] = np.cumsum(codes == c)
        for i in list(range(0, 400)) + list(range(b.T - 300, b.T + 2)) + [b.isa0, b.isa0 + 1]:
            j = i - (i > b.isa0)
            assert np.array_equal(ix.occ4(d, i), pref[j]), (d, i)


def test_width_matches_reference():
    from golden_io import GOLD
    g = np.load(f"{GOLD}/tiny_width.npz")
    ix = oracle_index("tiny")
    o = 0
    w = g["width"]
    for L in g["lens"]:
        L = int(L)
        seq = g["codes"][o:o + L]
        got = ix.cal_width(seq)
        exp = w[:L + 1]
        w = w[L + 1:]
        o += L
        assert np.array_equal(got, exp)


def test_step_consistency():
    """rev_l - rev_k == l - k for every child of a bidirectional step (2BWT-Interface.c:266-269)."""
    ix = oracle_index("tiny")
    T = ix.fwd.T
    k, l, rk, rl = 0, T, 0, T
    rng = np.random.default_rng(3)
    for _ in range(200):
        ok, ol, ork, orl = ix.step_all(k, l, rk, rl)
        for c in range(4):
            if ok[c] <= ol[c]:
                assert int(orl[c]) - int(ork[c]) == int(ol[c]) - int(ok[c])
        c = int(rng.integers(4))
        if ok[c] > ol[c]:
            k, l, rk, rl = 0, T, 0, T
        else:
            k, l, rk, rl = int(ok[c]), int(ol[c]), int(ork[c]), int(orl[c])


@pytest.mark.parametrize("name", sorted(cases().keys()) + sorted(limits_cases().keys()))
def test_batch_matches_reference(name):
    """bwa_cal_sa_reg_gap restatement vs the reference on every golden case.

    Reads the reference sent to bwt_splice_match (flags bit0) must be flagged the
    same way; their splice hits are out of the oracle's scope, every
    other read's hit list must be identical word for word, order included."""
    g = load_case(name)
    ix = oracle_index(g["index"])
    opt = parse_opts(g["args"], default_opt())
    n_aln, flags, hits, _ = ix.run_batches(g["lens"], g["codes"], opt, g["batch"])
    exp_splice = (g["flags"] & 1).astype(bool)
    assert np.array_equal((flags & 1).astype(bool), exp_splice)
    got = split_hits(n_aln, hits)
    exp = split_hits(g["n_aln"], g["hits"])
    bad = [i for i in range(len(got)) if not exp_splice[i] and not np.array_equal(got[i], exp[i])]
    assert not bad, f"{len(bad)} reads differ, first {bad[:5]}: got {got[bad[0]]} exp {exp[bad[0]]}"


@pytest.mark.parametrize("name", ["mgcap_default", "mgcap_n4o1"])
def test_match_gap_calls_match_reference(name):
    """bwt_match_gap called with caller widths, restated (or_match_gap): every call the
    reference's splice path made (aliased seeds, NULL-seed anchors) and a sample of
    main-path calls -- hits word for word, and the widths after gap_shadow (Q6)."""
    from golden_io import load_mgcap
    from oracle_ctypes import Opt
    ix = oracle_index("tiny")
    calls = load_mgcap(name)
    kinds = {c["seed"] for c in calls}
    assert kinds == {0, 1, 2}, kinds
    bad = []
    for j, c in enumerate(calls):
        opt = Opt.from_buffer_copy(c["opt"].tobytes())
        hits, w = ix.match_gap(opt, c["n_stacks"], c["seq"], c["strand"], c["wb"], c["seed"], c["ws"])
        if not (np.array_equal(hits, c["hits"]) and np.array_equal(w, c["wo"])):
            bad.append(j)
    assert not bad, f"{len(bad)} of {len(calls)} calls differ, first {bad[:5]}"


@pytest.mark.parametrize("name", ["nrun", "tiny"])
def test_sa_position_matches_reference(name):
    """BWTSaValue + BWTRetrievePositionFromSAIndex restated (R11): every SA index of
    a genome with N-runs (blocks with 'ori' offsets) and a sample of the tiny one."""
    g = np.load(f"{GOLD}/{name}_sa.npz")
    fwd, rev = index_io.read_index(INDEX[name])
    ox = OracleIndex(fwd, rev)
    got = ox.sa_positions(index_io.read_sa(INDEX[name]), index_io.read_blocks(INDEX[name]), g["idx"])
    assert np.array_equal(got[:, 0], g["sa"])
    assert np.array_equal(got[:, 1], g["seq_id"])
    assert np.array_equal(got[:, 2], g["ori_pos"])
    assert np.array_equal(got[:, 3], g["occ_pos"])


# ---- the 64-bit restatement (liboracle64.so, -DOR_WIDE): pinned against the 32-bit
# one and the reference's golden vectors on the sub-2^32 indexes
_IDX64 = {}


def oracle_index64(name):
    from oracle_ctypes import OracleIndex64
    if name not in _IDX64:
        _IDX64[name] = OracleIndex64.from_index(*index_io.read_index(INDEX[name]))
    return _IDX64[name]


def test_oracle64_occ_step_width_equal_32():
    fwd, rev = index_io.read_index(INDEX["rep"])
    o32, o64 = oracle_index("rep"), oracle_index64("rep")
    for d, b in enumerate((fwd, rev)):
        for i in list(range(0, 300)) + list(range(b.T - 200, b.T + 2)) + [b.isa0, b.isa0 + 1]:
            assert np.array_equal(o64.occ4(d, i), o32.occ4(d, i).astype(np.uint64)), (d, i)
    T = fwd.T
    k, l, rk, rl = 0, T, 0, T
    rng = np.random.default_rng(11)
    for _ in range(500):
        a = o32.step_all(k, l, rk, rl)
        b = o64.step_all(k, l, rk, rl)
        for x, y in zip(a, b):
            assert np.array_equal(x.astype(np.uint64), y)
        c = int(rng.integers(4))
        if a[0][c] > a[1][c] or rng.random() < 0.05:
            k, l, rk, rl = 0, T, 0, T
        else:
            k, l, rk, rl = (int(v[c]) for v in a)
    g = np.load(f"{GOLD}/tiny_width.npz")
    o32, o64 = oracle_index("tiny"), oracle_index64("tiny")
    o = 0
    for L in g["lens"][:50]:
        seq = g["codes"][o:o + int(L)]
        o += int(L)
        assert np.array_equal(o64.cal_width(seq), o32.cal_width(seq).astype(np.uint64))


@pytest.mark.parametrize("name", sorted(cases().keys()) + sorted(limits_cases().keys()))
def test_oracle64_batch_matches_reference(name):
    """bwa_cal_sa_reg_gap with 64-bit intervals on every golden case: the reference's
    hits, widened to hsa_aln64_t (bwt_aln1_t fields, 64-bit k/l/rev_k/rev_l)."""
    from oracle_ctypes import Opt, aln64_to_aln32
    g = load_case(name)
    ix = oracle_index64(g["index"])
    opt = Opt.from_dict(parse_opts(g["args"], default_opt()))
    offs = np.concatenate([[0], np.cumsum(g["lens"].astype(np.int64))])
    ns, fs, hs = [], [], []
    for b0 in range(0, len(g["lens"]), g["batch"]):      # bwa_aln_core's batches (bwtaln.c:477-506)
        b1 = min(b0 + g["batch"], len(g["lens"]))
        n_aln, flags, hits, _ = ix.cal_sa_reg_gap(g["lens"][b0:b1], g["codes"][offs[b0]:offs[b1]], opt)
        ns.append(n_aln); fs.append(flags); hs.append(aln64_to_aln32(hits))
    n_aln, flags, hits = np.concatenate(ns), np.concatenate(fs), np.concatenate(hs)
    exp_splice = (g["flags"] & 1).astype(bool)
    assert np.array_equal((flags & 1).astype(bool), exp_splice)
    got = split_hits(n_aln, hits)
    exp = split_hits(g["n_aln"], g["hits"])
    bad = [i for i in range(len(got)) if not exp_splice[i] and not np.array_equal(got[i], exp[i])]
    assert not bad, f"{len(bad)} reads differ, first {bad[:5]}"


@pytest.mark.parametrize("name", EXTCAP_CASES)
def test_extension_matches_reference(name):
    """bwt_extend_backward / bwt_extend_foreward (bwtgap.c:640-663, the splice path's
    seed extensions through bwt_backtracing_search :346-511): every call the compiled
    reference made on the splice read set, restated from the recorded window of the
    read alone -- return value, max_pos and every bwt_aln1_t field."""
    fwd, rev = index_io.read_index(INDEX["tiny"])
    ox = OracleIndex(fwd, rev)
    n = bad = 0
    for c in load_extcap(name):
        opt = Opt.from_buffer_copy(np.ascontiguousarray(c["opt"], np.uint32).tobytes())
        ret, mp, a = ox.extend(opt, c["n_stacks"], c["dir"], c["len"], c["seq"], c["bid"], c["lo"], c["aln_in"],
                               c["max_pos"])
        n += 1
        if ret != c["ret"] or mp != c["max_pos_out"] or not np.array_equal(a, c["aln_out"]):
            bad += 1
    assert n > 3000
    assert bad == 0, f"{bad} of {n} extensions differ"


def test_width_type0_matches_reference():
    """bwt_cal_width type 0 (the splice path's width_fore, bwtgap.c:868/:872) against the
    compiled reference's (tests/golden/tiny_width0.npz)."""
    fwd, rev = index_io.read_index(INDEX["tiny"])
    ox = OracleIndex(fwd, rev)
    g = np.load(f"{GOLD}/tiny_width0.npz")
    o = 0
    exp = g["width"]
    for L, off in zip(g["lens"].astype(int), np.concatenate([[0], np.cumsum(g["lens"].astype(int))[:-1]])):
        off = int(off)
        got = ox.cal_width0(g["codes"][off:off + L])
        assert np.array_equal(got, exp[o:o + L + 1]), off
        o += L + 1
