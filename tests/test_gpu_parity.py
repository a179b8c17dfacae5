"""GPU parity: the HIP path (through the C ABI) against the compiled reference's
golden vectors and the CPU restatement (oracle).  Integer work: bit-exact."""
import numpy as np
import pytest

from golden_io import GOLD, INDEX, cases, load_case, parse_opts, split_hits
from hsa_amd import index_io

pytestmark = pytest.mark.gpu

_GPU = {}


def gpu_index(name):
    from hsa_amd._lib import GpuIndex
    if name not in _GPU:
        _GPU[name] = GpuIndex(*index_io.read_index(INDEX[name]))
    return _GPU[name]


def test_rank_matches_reference():
    g = np.load(f"{GOLD}/tiny_occ.npz")
    ix = gpu_index("tiny")
    for d in (0, 1):
        assert np.array_equal(ix.occ4(d, g["pos"]), g["occ"][d]), f"dir {d}"


def test_rank_all_positions_prefix_count():
    fwd, rev = index_io.read_index(INDEX["rep"])
    ix = gpu_index("rep")
    for d, b in enumerate((fwd, rev)):
        codes = index_io.unpack_codes(b)
        pref = np.zeros((b.T + 1, 4), np.int64)
        for c in range(4):
            pref[1:, c] = np.cumsum(codes == c)
        pos = np.arange(b.T + 2, dtype=np.int64)
        exp = pref[pos - (pos > b.isa0)]
        assert np.array_equal(ix.occ4(d, pos.astype(np.uint32)), exp)


def test_width_matches_reference():
    g = np.load(f"{GOLD}/tiny_width.npz")
    ix = gpu_index("tiny")
    assert np.array_equal(ix.widths(g["lens"], g["codes"]), g["width"].reshape(-1))


def test_width_type0_matches_reference():
    """bwt_cal_width type 0 (the splice path's width_fore) on the GPU vs the compiled
    reference's values; entry 0, which the reference never writes, is 0 on both."""
    g = np.load(f"{GOLD}/tiny_width0.npz")
    ix = gpu_index("tiny")
    assert np.array_equal(ix.widths(g["lens"], g["codes"], type=0), g["width"].reshape(-1))


def test_step_matches_oracle():
    from oracle_ctypes import OracleIndex
    fwd, rev = index_io.read_index(INDEX["tiny"])
    ox = OracleIndex(fwd, rev)
    ix = gpu_index("tiny")
    rng = np.random.default_rng(5)
    T = fwd.T
    q = []
    k, l, rk, rl = 0, T, 0, T
    for _ in range(3000):
        q.append((k, l, rk, rl))
        ok, ol, ork, orl = ox.step_all(k, l, rk, rl)
        c = int(rng.integers(4))
        if ok[c] > ol[c] or rng.random() < 0.05:
            k, l, rk, rl = 0, T, 0, T
        else:
            k, l, rk, rl = int(ok[c]), int(ol[c]), int(ork[c]), int(orl[c])
    q = np.array(q, np.uint32)
    got = ix.step_all(q)
    for j in range(0, len(q), 97):
        exp = np.stack(ox.step_all(*[int(x) for x in q[j]]))
        assert np.array_equal(got[j], exp)


def _compare(name, pool_entries=0):
    from hsa_amd._lib import GapOpt, configure
    from oracle_ctypes import default_opt
    g = load_case(name)
    ix = gpu_index(g["index"])
    if pool_entries:
        configure(pool_entries=pool_entries)
    try:
        n_aln, flags, per_read, _ = ix.run_batches(g["lens"], g["codes"], parse_opts(g["args"], default_opt()),
                                                   g["batch"])
    finally:
        if pool_entries:
            configure(pool_entries=-1)
    exp_splice = (g["flags"] & 1).astype(bool)
    got_splice = (flags & 1).astype(bool)
    assert np.array_equal(got_splice, exp_splice), np.nonzero(got_splice != exp_splice)[0][:10]
    exp = split_hits(g["n_aln"], g["hits"])
    bad = [i for i in range(len(exp)) if not exp_splice[i] and not np.array_equal(per_read[i], exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}: got {per_read[bad[0]]} exp {exp[bad[0]]}"


@pytest.mark.parametrize("name", sorted(cases().keys()))
def test_search_matches_reference(name):
    _compare(name)


@pytest.mark.parametrize("name", ["tiny_gap100_n4o1", "rep_gap60_default"])
def test_search_after_scratch_release(name):
    """hsa_index_release_scratch gives the handle's working buffers back between calls;
    the next search allocates them again and its results are the reference's."""
    ix = gpu_index(load_case(name)["index"])
    _compare(name)
    ix.release_scratch()
    _compare(name)
    ix.release_scratch()
    ix.release_scratch()                      # twice in a row: nothing left to free
    _compare(name)


@pytest.mark.parametrize("name", ["tiny_gap100_n4o1", "tiny_edge_default", "rep_gap60_default", "tiny_gap100_n4o1_b400"])
def test_search_matches_reference_one_lane_per_read(name, monkeypatch):
    """Batches smaller than the chip run strand-split (each read's rc and fwd searches on
    two lanes, k_split_finalize choosing, bwtaln.c:343-359); this is the one-read-per-lane
    main pass that large batches use, on the same golden cases."""
    monkeypatch.setenv("HSA_SPLIT", "0")
    _compare(name)


@pytest.mark.parametrize("name", ["tiny_gap100_n4o1", "tiny_mm100_n4o0", "rep_gap60_default", "tiny_edge_default",
                                  "tiny_gap100_n4o1_b400"])
def test_search_matches_reference_cost_order(name, monkeypatch):
    """Batches larger than the chip take their reads in cost order (k_order_*: the lower
    strand bid first-highest), a permutation of the list positions k_search pulls; forced
    here on the golden cases (one read per lane, no strand split)."""
    monkeypatch.setenv("HSA_ORDER", "1")
    monkeypatch.setenv("HSA_SPLIT", "0")
    _compare(name)


@pytest.mark.parametrize("case", ["tiny_mm100_n4o0", "tiny_gap100_n4o1"])
def test_rank_queries_match_oracle_cost_order(case, monkeypatch):
    """The device path in cost order: the same per-read hits and the oracle's rank-query
    and pop counts."""
    monkeypatch.setenv("HSA_ORDER", "1")
    monkeypatch.setenv("HSA_SPLIT", "0")
    got, (e_n, e_f, e_h, st) = _device_run(case)
    assert np.array_equal(got["n"], e_n) and np.array_equal(got["f"] & 1, e_f & 1)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(exp)) if not np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)],
                                                             exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"
    assert int(got["c"][2]) == int(st[0]) and int(got["c"][4]) == int(st[1])


@pytest.mark.parametrize("lazy", ["0", "1"])
@pytest.mark.parametrize("name", ["tiny_gap100_n4o1", "tiny_mm100_n4o0", "rep_gap60_default", "tiny_opts_seed"])
def test_search_matches_reference_lazy_forward_rows(name, lazy, monkeypatch):
    """The main pass of a batch searched one read per lane computes a read's forward
    width row only when its rc search cannot hit (the root is pruned: last bid >
    max_diff); the reads whose rc search finds nothing without one go through the
    forward pass (k_widths_reads mode 2 + a fwd-only k_search).  HSA_LAZY=0: every row
    up front."""
    monkeypatch.setenv("HSA_LAZY", lazy)
    monkeypatch.setenv("HSA_SPLIT", "0")
    _compare(name)


@pytest.mark.parametrize("lazy", ["0", "1"])
@pytest.mark.parametrize("case", ["tiny_mm100_n4o0", "tiny_gap100_n4o1", "rep_mm100_n4o1"])
def test_rank_queries_match_oracle_lazy_forward_rows(case, lazy, monkeypatch):
    """Lazy forward rows keep the reference's rank-query and pop counts: a forward row
    counts when the forward strand is searched, in either pass."""
    monkeypatch.setenv("HSA_LAZY", lazy)
    monkeypatch.setenv("HSA_SPLIT", "0")
    got, (e_n, e_f, e_h, st) = _device_run(case)
    assert np.array_equal(got["n"], e_n) and np.array_equal(got["f"] & 1, e_f & 1)
    assert int(got["c"][2]) == int(st[0]) and int(got["c"][4]) == int(st[1])
    assert got["c"][13] >= got["c"][14]


@pytest.mark.parametrize("name", ["tiny_gap100_n4o1", "rep_mm100_n4o1"])
def test_overflow_rerun_is_exact(name):
    """A tiny per-lane pool forces most reads through the large-capacity re-run."""
    _compare(name, pool_entries=64)


def _device_run(case, pool_entries=0, cap=None, ix=None, args=None):
    """One hsa_search_device call (device-resident batch, bench.py's path) on a golden
    case as a steady-state batch (GAPE already cleared: both regimes coincide), and
    the oracle's bwa_cal_sa_reg_gap on the same reads.  ix: an index of the case's
    genome (default: the cached one); args: options instead of the case's."""
    import torch
    from hsa_amd._lib import JOB_DTYPE, DeviceBatch, GapOpt, configure, pad_codes, regime_of
    from oracle_ctypes import Opt, OracleIndex, default_opt
    g = load_case(case)
    fwd, rev = index_io.read_index(INDEX[g["index"]])
    ix = gpu_index(g["index"]) if ix is None else ix
    od = parse_opts(g["args"] if args is None else args.split(), default_opt())
    od["mode"] &= ~0x01
    # the device path searches every job it is given: keep the reads that pass
    # bwa_cal_sa_reg_gap's filters (bwtaln.c:314-325; the drop-in applies them on the host)
    offs = np.concatenate([[0], np.cumsum(g["lens"].astype(np.int64))])
    keep = []
    for r in range(len(g["lens"])):
        sq = g["codes"][offs[r]:offs[r + 1]]
        polyat = len(sq) >= 15 and ((sq[:15] == 0).all() or (sq[:15] == 3).all())
        keep.append(int((sq > 3).sum()) <= od["max_diff"] and not polyat)
    keep = np.array(keep)
    g = dict(g, lens=g["lens"][keep], codes=np.concatenate([g["codes"][offs[r]:offs[r + 1]]
                                                            for r in np.flatnonzero(keep)]))
    n = len(g["lens"])
    exp = OracleIndex(fwd, rev).cal_sa_reg_gap(g["lens"], g["codes"], Opt.from_dict(od))
    o = GapOpt.from_dict(od)
    n_stacks = (o.max_diff + 1) * o.s_mm + (o.max_gapo + 1) * o.s_gapo + (o.max_gape + 1) * o.s_gape
    rg = regime_of(od, n_stacks, o.max_diff)           # the option bits bwt_match_gap reads (NONSTOP, LOGGAP)
    jobs = np.zeros(n, JOB_DTYPE)
    jobs["off"] = np.concatenate([[0], np.cumsum(g["lens"].astype(np.uint64))[:-1]])
    jobs["len"] = g["lens"]
    jobs["max_diff"] = o.max_diff
    jobs["seed_len"] = np.where(g["lens"] > o.seed_len, o.seed_len, 0x7FFFFFFF)
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).cuda()
    d_codes = torch.from_numpy(pad_codes(g["codes"])).cuda()
    cap = n * 16 if cap is None else cap
    t = dict(n=torch.zeros(n, dtype=torch.int32, device="cuda"), f=torch.zeros(n, dtype=torch.int32, device="cuda"),
             o=torch.zeros(n, dtype=torch.int64, device="cuda"),
             h=torch.zeros(max(cap, 1) * 9, dtype=torch.int32, device="cuda"),
             c=torch.zeros(16, dtype=torch.int64, device="cuda"))
    b = DeviceBatch(d_jobs=d_jobs.data_ptr(), n_jobs=n, d_codes=d_codes.data_ptr(), d_n_aln=t["n"].data_ptr(),
                    d_flags=t["f"].data_ptr(), d_hit_off=t["o"].data_ptr(), d_hits=t["h"].data_ptr(), hit_cap=cap,
                    d_counters=t["c"].data_ptr(), max_len=int(g["lens"].max()), max_seed=o.seed_len)
    if pool_entries:
        configure(pool_entries=pool_entries)
    try:
        ix.search_device([rg], b)
        torch.cuda.synchronize()
    finally:
        if pool_entries:
            configure(pool_entries=-1)
    got = dict(n=t["n"].cpu().numpy(), f=t["f"].cpu().numpy().astype(np.uint32), o=t["o"].cpu().numpy(),
               h=t["h"].cpu().numpy().view(np.uint32).reshape(-1, 9), c=t["c"].cpu().numpy())
    return got, exp


def test_device_path_rerun_is_exact():
    """hsa_search_device re-runs reads that overflow their lane's capacity on the
    device: with a tiny pool most reads of a gapped case take that route, and every
    hit must still equal the oracle's."""
    got, (e_n, e_f, e_h, _) = _device_run("tiny_gap100_n4o1", pool_entries=8)
    assert got["c"][8] > 0, got["c"][8]
    assert got["c"][11] == 0, "reads left unfinished after the re-run"
    assert not (got["f"] & 2).any(), "reads left overflowed after the re-run"
    assert np.array_equal(got["f"] & 1, e_f & 1)
    assert np.array_equal(got["n"], e_n)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(exp)) if not np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)],
                                                             exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"


@pytest.mark.parametrize("case", ["tiny_gap100_n4o1", "rep_mm100_n4o1"])
def test_scratch_cap_shrinks_pool_and_stays_exact(case, monkeypatch, capfd):
    """HSA_SCRATCH_MB caps the search scratch a handle may take (as a co-resident
    process or a third handle would, by leaving little HBM free): the main pass's
    per-lane pool shrinks to fit instead of the call failing, reads that outgrow the
    smaller pool finish in the BIG/HUGE re-runs, and every hit equals the oracle's."""
    from hsa_amd._lib import GpuIndex
    monkeypatch.setenv("HSA_SCRATCH_MB", "4")
    monkeypatch.setenv("HSA_VERBOSE", "1")
    g = load_case(case)
    fresh = GpuIndex(*index_io.read_index(INDEX[g["index"]]))     # no scratch held yet
    try:
        got, (e_n, e_f, e_h, _) = _device_run(case, ix=fresh)
    finally:
        fresh.close()
    assert "search scratch: pool" in capfd.readouterr().err, "the pool was not capped"
    assert got["c"][11] == 0, "reads left unfinished"
    assert np.array_equal(got["f"] & 1, e_f & 1)
    assert np.array_equal(got["n"], e_n)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(exp)) if not np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)],
                                                             exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"


def test_parent_freed_before_its_clone():
    """hsa_index_free on an index whose clone is still live defers the free of the shared
    rank blocks to the clone's own hsa_index_free: the clone still searches exactly."""
    from hsa_amd._lib import GpuIndex, lib
    parent = GpuIndex(*index_io.read_index(INDEX["tiny"]))
    c = parent.clone()
    lib().hsa_index_free(parent.h)            # the C API directly (the wrapper closes clones first)
    parent.h, parent._clones = None, []
    try:
        got, (e_n, e_f, e_h, _) = _device_run("tiny_mm100_n4o0", ix=c)
    finally:
        c.close()                              # frees the clone, then the deferred parent
    assert np.array_equal(got["n"], e_n) and np.array_equal(got["f"] & 1, e_f & 1)


@pytest.mark.parametrize("split", ["0", "1"])
@pytest.mark.parametrize("case", ["tiny_mm100_n4o0", "tiny_gap100_n4o1", "rep_mm100_n4o1"])
def test_rank_queries_match_oracle(case, split, monkeypatch):
    """The roofline numerator: the rank queries the kernels count (d_counters[2]) are
    the ones the reference algorithm issues -- widths only for the strands it
    searches (bwtaln.c:343-359), 2 per bidirectional step -- exactly the oracle's
    count on the same reads (no read overflows at the default capacity) -- also in the
    strand-split main pass, which counts a fwd search only when rc had no hit."""
    monkeypatch.setenv("HSA_SPLIT", split)
    got, (_, _, _, st) = _device_run(case)
    assert got["c"][8] == 0
    assert int(got["c"][2]) == int(st[0]), (int(got["c"][2]), int(st[0]))
    assert int(got["c"][4]) == int(st[1]), "gap_pop count"
    # the speculative forward-strand widths are counted apart: all >= searched ones
    assert got["c"][13] >= got["c"][14]


def test_device_path_hit_buffer_exhausted_is_reported():
    """A caller hit buffer too small for the batch: the reads whose hits do not fit
    stay flagged HSA_F_OVERFLOW with no hits and are counted in d_counters[11]
    (include/hsa_gpu.h); every read that completed is exact."""
    got, (e_n, e_f, e_h, _) = _device_run("tiny_mm100_n4o0", cap=40)
    unfinished = (got["f"] & 2) != 0
    assert unfinished.any()
    assert int(got["c"][11]) == int(unfinished.sum())
    exp = split_hits(e_n, e_h)
    done = np.flatnonzero(~unfinished)
    assert len(done) > 0
    for i in done:
        assert got["n"][i] == e_n[i]
        assert np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)], exp[i])
    assert (got["n"][unfinished] == 0).all()


def test_device_path_huge_pass_is_exact():
    """Reads whose stacks take more than the big pass's 65 535 slots (NONSTOP, -n 6
    -o 2 on the repeat-rich index: ~10^5-10^6 pushes per read) finish in the huge pass
    (reused slots, bwtgap.c:150-151's bound) with the oracle's hits."""
    got, (e_n, e_f, e_h, _) = _device_run("rep_deep_n6o2N")
    assert got["c"][12] > 0, "no read reached the huge pass"
    assert got["c"][11] == 0, "reads left unfinished"
    assert np.array_equal(got["f"] & 1, e_f & 1)
    assert np.array_equal(got["n"], e_n)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(exp)) if not np.array_equal(got["h"][got["o"][i]:got["o"][i] + max(got["n"][i], 0)],
                                                             exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"


def _slot_indexes(name, n):
    from hsa_amd._lib import GpuIndex
    key = f"{name}#slots"
    if key not in _GPU:
        _GPU[key] = [GpuIndex(*index_io.read_index(INDEX[name])) for _ in range(3)]
    return _GPU[key][:n]


@pytest.mark.parametrize("name,slots", [("tiny_gap100_n4o1_b400", 2), ("tiny_edge_default", 3), ("rep_gap60_default", 2)])
def test_device_slots_match_reference(name, slots):
    """bwa_cal_sa_reg_gap split over device slots (hsa_cal_sa_reg_gap_multi: the
    boundary's hsa_gpu_set_devices) gives the golden hits, the option-regime switch
    after the first splice fallback read included (tiny_gap100_n4o1_b400)."""
    from oracle_ctypes import default_opt
    g = load_case(name)
    ix = gpu_index(g["index"])
    n_aln, flags, per_read, _ = ix.run_batches(g["lens"], g["codes"], parse_opts(g["args"], default_opt()), g["batch"],
                                               others=_slot_indexes(g["index"], slots - 1))
    exp_splice = (g["flags"] & 1).astype(bool)
    assert np.array_equal((flags & 1).astype(bool), exp_splice)
    exp = split_hits(g["n_aln"], g["hits"])
    bad = [i for i in range(len(exp)) if not exp_splice[i] and not np.array_equal(per_read[i], exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"


@pytest.mark.parametrize("slots", [1, 2])
def test_regime_switch_after_first_chunk(slots):
    """A gapped batch of 20 000 reads whose first splice-fallback read comes after the
    first 8 192-read chunk (CHUNK0 in bwtaln_gpu.c) and after the first slot's part:
    regime A up to and including that read, regime B after it (bwtaln.c:254-363),
    against the oracle's bwa_cal_sa_reg_gap on the same batch."""
    from hsa_amd._lib import GapOpt
    from oracle_ctypes import Opt, OracleIndex, default_opt
    g = load_case("tiny_gap100_n4o1")
    fwd, rev = index_io.read_index(INDEX["tiny"])
    L = int(g["lens"][0])
    assert (g["lens"] == L).all()
    base = g["codes"].reshape(-1, L)
    reps = np.concatenate([base] * (20000 // len(base) + 1))[:20000].copy()
    flags_seq = OracleIndex(fwd, rev).cal_sa_reg_gap(np.full(len(base), L, np.uint32), base.reshape(-1),
                                                      Opt.from_dict(parse_opts(g["args"], default_opt())))[1]
    # make every read before 12 345 mappable, and an unmappable read at 12 345
    mappable = base[np.flatnonzero((flags_seq & 1) == 0)]
    reps[:12345] = np.concatenate([mappable] * (12345 // len(mappable) + 1))[:12345]
    rng = np.random.default_rng(9)
    reps[12345] = rng.integers(0, 4, L)
    lens = np.full(len(reps), L, np.uint32)
    od = parse_opts(g["args"], default_opt())
    e_n, e_f, e_h, _ = OracleIndex(fwd, rev).cal_sa_reg_gap(lens, reps.reshape(-1), Opt.from_dict(od))
    assert (e_f[:12345] & 1).sum() == 0 and e_f[12345] & 1
    ix = gpu_index("tiny")
    others = _slot_indexes("tiny", slots - 1) if slots > 1 else []
    if others:
        n_aln, flags, hoff, hits, _ = ix.cal_sa_reg_gap_slots(others, lens, reps.reshape(-1), GapOpt.from_dict(od))
    else:
        n_aln, flags, hoff, hits, _ = ix.cal_sa_reg_gap(lens, reps.reshape(-1), GapOpt.from_dict(od))
    assert np.array_equal(flags & 1, e_f & 1)
    assert np.array_equal(n_aln, e_n)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(exp)) if not np.array_equal(hits[int(hoff[i]):int(hoff[i]) + max(int(n_aln[i]), 0)], exp[i])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}"
