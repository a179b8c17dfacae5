"""The 64-bit interval instantiation (config 5: texts of 2^32 characters or more,
which the reference's 32-bit bwtint_t cannot index, 2BWT-Interface.h:26).

* sub-2^32 parity: hsa_search_device64 on indexes built with
  hsa_index_create_device64 from the golden index files equals the reference's
  golden hits, the 32-bit kernels on the same index, and the 64-bit oracle;
* ranks past 2^32: hsa_occ4_batch64 on a 4.3 G-character code string equals the
  64-bit oracle at random positions and at every boundary the layout has (2^32, the
  count-wrap blocks of the wrap table, the '$' row);
* search past 2^32: a device-built BWT of a 4.3 Gbp synthetic text, reads from the
  whole text, -n 4 -o 1 (100 bp) and config 5's own instantiation (250 bp, -n 4 -o 0,
  64-bit intervals with 4-bit pruning rows): every hit equals the 64-bit oracle's (liboracle64.so, the
  same restatement pinned against the 32-bit one in tests/test_oracle.py), and hits
  with SA bounds >= 2^32 occur.  No reference output exists at this size (the
  reference cannot index it): parity is against the restatement only."""
import ctypes as C

import numpy as np
import pytest

from golden_io import INDEX, load_case, parse_opts, split_hits
from hsa_amd import index_io

pytestmark = pytest.mark.gpu

_IX = {}


def _upload_lsb(b):
    import torch
    from oracle_ctypes import msb_to_lsb
    w = msb_to_lsb(b.code, b.T)
    return torch.from_numpy(np.concatenate([w, np.zeros(8, np.uint32)]).view(np.int32)).cuda()


def index64(name):
    """hsa_index_create_device64 over a golden index (T < 2^32: the 32-bit entry
    points serve the same index)."""
    from hsa_amd._lib import GpuIndex
    if name not in _IX:
        fwd, rev = index_io.read_index(INDEX[name])
        d_f, d_r = _upload_lsb(fwd), _upload_lsb(rev)
        gi = GpuIndex.from_device_codes64(fwd.T, fwd.isa0, np.asarray(fwd.C, np.uint64), d_f.data_ptr(), rev.T,
                                          rev.isa0, np.asarray(rev.C, np.uint64), d_r.data_ptr())
        _IX[name] = gi
    return _IX[name]


def _device_jobs(g, od):
    """The reads of a golden case that pass bwa_cal_sa_reg_gap's filters
    (bwtaln.c:314-325) as a steady-state device batch."""
    offs = np.concatenate([[0], np.cumsum(g["lens"].astype(np.int64))])
    keep = []
    for r in range(len(g["lens"])):
        sq = g["codes"][offs[r]:offs[r + 1]]
        polyat = len(sq) >= 15 and ((sq[:15] == 0).all() or (sq[:15] == 3).all())
        keep.append(int((sq > 3).sum()) <= od["max_diff"] and not polyat)
    keep = np.flatnonzero(keep)
    lens = g["lens"][keep]
    codes = np.concatenate([g["codes"][offs[r]:offs[r + 1]] for r in keep])
    return lens, codes


def search(gi, lens, codes, od, wide, cap_per_read=16):
    """One hsa_search_device(64) call; hits as (n_aln, flags, hit_off, hits rows)."""
    import torch
    from hsa_amd._lib import ALN64_WORDS, JOB_DTYPE, DeviceBatch, GapOpt, pad_codes, regime_of
    o = GapOpt.from_dict(od)
    n = len(lens)
    n_stacks = (o.max_diff + 1) * o.s_mm + (o.max_gapo + 1) * o.s_gapo + (o.max_gape + 1) * o.s_gape
    rg = regime_of(od, n_stacks, o.max_diff)
    jobs = np.zeros(n, JOB_DTYPE)
    jobs["off"] = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]])
    jobs["len"] = lens
    jobs["max_diff"] = o.max_diff
    jobs["seed_len"] = np.where(lens > o.seed_len, o.seed_len, 0x7FFFFFFF)
    hw = ALN64_WORDS if wide else 9
    cap = n * cap_per_read
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).cuda()
    d_codes = torch.from_numpy(pad_codes(codes)).cuda()
    t = dict(n=torch.zeros(n, dtype=torch.int32, device="cuda"), f=torch.zeros(n, dtype=torch.int32, device="cuda"),
             o=torch.zeros(n, dtype=torch.int64, device="cuda"),
             h=torch.zeros(cap * hw + 2, dtype=torch.int32, device="cuda"),
             c=torch.zeros(16, dtype=torch.int64, device="cuda"))
    b = DeviceBatch(d_jobs=d_jobs.data_ptr(), n_jobs=n, d_codes=d_codes.data_ptr(), d_n_aln=t["n"].data_ptr(),
                    d_flags=t["f"].data_ptr(), d_hit_off=t["o"].data_ptr(), d_hits=t["h"].data_ptr(), hit_cap=cap,
                    d_counters=t["c"].data_ptr(), max_len=int(lens.max()), max_seed=o.seed_len)
    (gi.search_device64 if wide else gi.search_device)([rg], b)
    torch.cuda.synchronize()
    c = t["c"].cpu().numpy()
    assert c[11] == 0, "reads left unfinished"
    h = t["h"].cpu().numpy().view(np.uint32)[:cap * hw].reshape(-1, hw)
    return t["n"].cpu().numpy(), t["f"].cpu().numpy().astype(np.uint32), t["o"].cpu().numpy(), h, c


def per_read(n_aln, hit_off, hits):
    return [hits[int(hit_off[i]):int(hit_off[i]) + max(int(n_aln[i]), 0)] for i in range(len(n_aln))]


@pytest.mark.parametrize("case", ["tiny_mm100_n4o0", "tiny_gap100_n4o1", "tiny_edge_n3o1e3L", "rep_mm100_n4o1",
                                  "rep_gap60_nonstop", "tiny_opts_scores", "tiny_opts_seed", "rep_deep_n6o2N"])
def test_wide_kernels_match_32bit_and_oracle(case):
    from oracle_ctypes import Opt, OracleIndex64, aln64_to_aln32, default_opt
    g = load_case(case)
    od = parse_opts(g["args"], default_opt())
    od["mode"] &= ~0x01                                  # a steady-state batch (both regimes coincide)
    lens, codes = _device_jobs(g, od)
    gi = index64(g["index"])
    n64, f64, o64, h64, c64 = search(gi, lens, codes, od, True)
    n32, f32, o32, h32, c32 = search(gi, lens, codes, od, False)
    # the same work: rank queries and pops
    assert c64[2] == c32[2] and c64[4] == c32[4]
    assert np.array_equal(n64, n32) and np.array_equal(f64 & 1, f32 & 1)
    got = per_read(n64, o64, h64)
    exp32 = per_read(n32, o32, h32)
    bad = [i for i in range(len(got)) if not np.array_equal(aln64_to_aln32(got[i]), exp32[i])]
    assert not bad, f"{len(bad)} reads differ from the 32-bit kernels; first {bad[0]}"
    # and the 64-bit restatement, record for record
    ox = OracleIndex64.from_index(*index_io.read_index(INDEX[g["index"]]))
    e_n, e_f, e_h, st = ox.cal_sa_reg_gap(lens, codes, Opt.from_dict(od))
    assert np.array_equal(n64, e_n) and np.array_equal(f64 & 1, e_f & 1)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(got)) if not np.array_equal(got[i], exp[i])]
    assert not bad, f"{len(bad)} reads differ from the 64-bit oracle; first {bad[0]}"
    if c64[8] == 0:      # (a read re-run for capacity counts its work twice: include/hsa_gpu.h)
        assert int(c64[2]) == int(st[0])


# golden cases whose two option regimes coincide (no gap opens, or -e given: GAPE is
# off from the start, bwtaln.c:261, :548), so a steady-state device batch reproduces
# the reference's own run read for read
STEADY_CASES = ["tiny_mm100_n4o0", "tiny_opts_seed", "tiny_exact36_n0", "tiny_edge_n3o1e3L", "tiny_opts_bigstack"]


@pytest.mark.parametrize("case", STEADY_CASES)
def test_wide_4bit_rows_match_reference(case, monkeypatch, capfd):
    """hsa_search_device64 with the 4-bit pruning rows forced (HSA_WFMT=nib, exact for
    these bounds) against the compiled reference's golden hits: every read that passes
    the filters and does not fall to the splice path has the reference's bwt_aln1_t
    list (the 64-bit records narrowed), and the fallback flags agree."""
    from oracle_ctypes import aln64_to_aln32, default_opt
    monkeypatch.setenv("HSA_WFMT", "nib")
    monkeypatch.setenv("HSA_VERBOSE", "1")
    g = load_case(case)
    od = parse_opts(g["args"], default_opt())
    od["mode"] &= ~0x01
    offs = np.concatenate([[0], np.cumsum(g["lens"].astype(np.int64))])
    keep = []
    for r in range(len(g["lens"])):
        sq = g["codes"][offs[r]:offs[r + 1]]
        polyat = len(sq) >= 15 and ((sq[:15] == 0).all() or (sq[:15] == 3).all())
        if int((sq > 3).sum()) <= od["max_diff"] and not polyat:
            keep.append(r)
    lens, codes = _device_jobs(g, od)
    assert len(lens) == len(keep)
    n64, f64, o64, h64, _ = search(index64(g["index"]), lens, codes, od, True)
    assert "4-bit rows" in capfd.readouterr().err
    exp = split_hits(g["n_aln"], g["hits"])
    exp_splice = (g["flags"][keep] & 1).astype(bool)
    assert np.array_equal((f64 & 1).astype(bool), exp_splice)
    got = per_read(n64, o64, h64)
    bad = [j for j, r in enumerate(keep) if not exp_splice[j] and not np.array_equal(aln64_to_aln32(got[j]), exp[r])]
    assert not bad, f"{len(bad)} reads differ from the reference; first read {keep[bad[0]]}"


def test_wide_index_serves_32bit_entry_points():
    """A sub-2^32 index made by hsa_index_create_device64 answers the 32-bit rank
    primitive exactly as hsa_index_create's, and the 64-bit one agrees."""
    from hsa_amd._lib import GpuIndex
    fwd, rev = index_io.read_index(INDEX["rep"])
    a = GpuIndex(fwd, rev)
    b = index64("rep")
    assert not b.is64()
    for d, bw in enumerate((fwd, rev)):
        pos = np.arange(bw.T + 2, dtype=np.uint32)
        ref = a.occ4(d, pos)
        assert np.array_equal(b.occ4(d, pos), ref)
        assert np.array_equal(b.occ4_64(d, pos.astype(np.uint64)), ref.astype(np.uint64))


# ---------------------------------------------------------------- past 2^32
BIG_T = (1 << 32) + (1 << 22) + 7


def _counts_lsb(w, T):
    """A, C, G, T counts of LSB-first 2-bit words (trailing codes past T are 0 = A)."""
    lo = w & np.uint32(0x55555555)
    hi = (w >> np.uint32(1)) & np.uint32(0x55555555)
    n3 = int(np.bitwise_count(lo & hi).sum(dtype=np.int64))
    n1 = int(np.bitwise_count(lo).sum(dtype=np.int64)) - n3
    n2 = int(np.bitwise_count(hi).sum(dtype=np.int64)) - n3
    return np.array([T - n1 - n2 - n3, n1, n2, n3], np.int64)


def test_rank_past_2_32_matches_oracle():
    """Occ at 64-bit positions over a 4.3 G-character code string (random codes; the
    rank structure does not need a BWT): random positions plus 2^32 +- 1, multiples of
    2^24 (the old superblock edges, kept as arbitrary far-apart probes), the '$' row and
    T + 1."""
    import torch
    from hsa_amd._lib import GpuIndex, check, lib
    from oracle_ctypes import OracleIndex64
    T = BIG_T
    nw = (T + 15) // 16
    d = []
    for seed in (21, 22):
        t = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
        check(lib().hsa_synth_genome_device(0, T, seed, t.data_ptr()))
        d.append(t)
    torch.cuda.synchronize()
    host = [x[:nw].cpu().numpy().view(np.uint32) for x in d]
    Cs = []
    for w in host:
        cnt = _counts_lsb(w, T)
        Cs.append(np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint64))
    isa0 = (T // 3 + 12345, (1 << 32) + 5)
    gi = GpuIndex.from_device_codes64(T, isa0[0], Cs[0], d[0].data_ptr(), T, isa0[1], Cs[1], d[1].data_ptr())
    assert gi.is64()
    ox = OracleIndex64(T, isa0[0], Cs[0], host[0], T, isa0[1], Cs[1], host[1])
    rng = np.random.default_rng(4)
    edges = [0, 1, 15, 16, 17, (1 << 32) - 1, 1 << 32, (1 << 32) + 1, (1 << 32) + 16, T - 1, T, T + 1]
    edges += [s * (1 << 24) + e for s in (1, 7, 255, 256, T >> 24) for e in (-1, 0, 1)]
    for d_ in (0, 1):
        pos = np.concatenate([rng.integers(0, T + 2, 4000, dtype=np.uint64),
                              np.array(edges + [isa0[d_] - 1, isa0[d_], isa0[d_] + 1, isa0[d_] + 2], np.uint64)])
        got = gi.occ4_64(d_, pos)
        exp = np.stack([ox.occ4(d_, int(p)) for p in pos])
        bad = np.flatnonzero((got != exp).any(axis=1))
        assert len(bad) == 0, f"dir {d_}: {len(bad)} positions differ, first {int(pos[bad[0]])}: {got[bad[0]]} vs {exp[bad[0]]}"
        # and the prefix-count identity: the four counts of a prefix sum to its length
        p = pos.astype(np.int64)
        assert np.array_equal(got.sum(axis=1).astype(np.int64), p - (p > isa0[d_]))
    gi.close()


def test_rank_count_wraps_match_oracle():
    """Occ past a count wrap: base counts above 2^32 (the blocks keep them modulo 2^32 and
    the index's wrap table adds the high words).  Forward: A everywhere but 1 in 2 000
    code words random, so Occ(A) passes 2^32 near the end; reverse: the same with C.
    Positions around each wrap block, random ones and the usual edges."""
    import torch
    from hsa_amd._lib import GpuIndex, check, lib
    from oracle_ctypes import OracleIndex64
    T = BIG_T
    nw = (T + 15) // 16
    d, host, Cs, wraps = [], [], [], []
    for fill, seed in ((0x00000000, 31), (0x55555555, 32)):
        t = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
        check(lib().hsa_synth_genome_device(0, T, seed, t.data_ptr()))
        g = torch.Generator(device="cuda").manual_seed(seed)
        keep = torch.rand(nw + 8, device="cuda", generator=g) < 1.0 / 2000
        t = torch.where(keep, t, torch.tensor(np.int32(np.uint32(fill).view(np.int32)), device="cuda"))
        if T % 16:                                   # no codes past T in the last word
            last = int(np.uint32(t[nw - 1].item() & 0xFFFFFFFF)) & ((1 << (2 * (T % 16))) - 1)
            t[nw - 1] = int(np.uint32(last).view(np.int32))
        t[nw:] = 0
        torch.cuda.synchronize()
        w = t[:nw].cpu().numpy().view(np.uint32)
        cnt = _counts_lsb(w, T)
        Cs.append(np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint64))
        base = 0 if fill == 0 else 1
        assert cnt[base] > (1 << 32)
        # the character position where the count of `base` reaches 2^32
        lo = w & np.uint32(0x55555555)
        hi = (w >> np.uint32(1)) & np.uint32(0x55555555)
        per = (np.bitwise_count(lo & ~hi & np.uint32(0x55555555)) if base == 1 else
               16 - np.bitwise_count((lo | hi) & np.uint32(0x55555555))).astype(np.int64)
        if base == 0:
            per[-1] -= 16 - (T - 16 * (nw - 1))    # padding codes are not characters
        word = int(np.searchsorted(np.cumsum(per), 1 << 32))
        wraps.append(16 * word)
        d.append(t)
        host.append(w)
    isa0 = (T // 5 + 3, (1 << 32) + 77)
    gi = GpuIndex.from_device_codes64(T, isa0[0], Cs[0], d[0].data_ptr(), T, isa0[1], Cs[1], d[1].data_ptr())
    ox = OracleIndex64(T, isa0[0], Cs[0], host[0], T, isa0[1], Cs[1], host[1])
    rng = np.random.default_rng(9)
    for d_ in (0, 1):
        w0 = wraps[d_]
        near = [w0 + e for e in range(-40, 41)] + [w0 + 16 * k for k in (-3, -2, -1, 1, 2, 3, 1000)]
        pos = np.concatenate([rng.integers(0, T + 2, 3000, dtype=np.uint64),
                              rng.integers(w0 - 100000, w0 + 100000, 1000, dtype=np.uint64),
                              np.array(near + [0, 1, 16, (1 << 32) - 1, 1 << 32, T - 1, T, T + 1,
                                               isa0[d_] - 1, isa0[d_], isa0[d_] + 1], np.uint64)])
        got = gi.occ4_64(d_, pos)
        exp = np.stack([ox.occ4(d_, int(p)) for p in pos])
        bad = np.flatnonzero((got != exp).any(axis=1))
        assert len(bad) == 0, f"dir {d_}: {len(bad)} positions differ, first {int(pos[bad[0]])}: {got[bad[0]]} vs {exp[bad[0]]}"
        assert int(exp[:, d_].max()) > (1 << 32)     # the wrap was crossed
    gi.close()


@pytest.fixture(scope="module")
def big_index():
    """A 4.3 Gbp synthetic text, its forward and reverse BWTs built on the device
    (hsa_build_bwt_device64: u64 suffix positions), the 64-bit index over them and the
    64-bit restatement's index over the same code words."""
    import torch
    from hsa_amd import synth
    from hsa_amd._lib import GpuIndex, check, lib
    from oracle_ctypes import OracleIndex64
    T = BIG_T
    nw = (T + 15) // 16
    text = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
    check(lib().hsa_synth_genome_device(0, T, 77, text.data_ptr()))
    res = []
    for rev in (0, 1):
        bw = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
        isa0 = C.c_uint64()
        Cc = np.zeros(5, np.uint64)
        check(lib().hsa_build_bwt_device64(0, T, text.data_ptr(), rev, bw.data_ptr(), C.byref(isa0), Cc))
        res.append((bw, int(isa0.value), Cc))
    del text
    torch.cuda.synchronize()
    assert int(res[0][2][4]) == T and int(res[1][2][4]) == T
    gi = GpuIndex.from_device_codes64(T, res[0][1], res[0][2], res[0][0].data_ptr(), T, res[1][1], res[1][2],
                                      res[1][0].data_ptr())
    host = [r[0][:nw].cpu().numpy().view(np.uint32) for r in res]
    ox = OracleIndex64(T, res[0][1], res[0][2], host[0], T, res[1][1], res[1][2], host[1])
    genome = synth.PackedGenome(T, 77)
    yield gi, ox, genome
    gi.close()


def _check_past_2_32(gi, ox, reads, od, wide_hits=True):
    from oracle_ctypes import Opt
    lens = np.full(len(reads), reads.shape[1], np.uint32)
    codes = reads.reshape(-1)
    g_n, g_f, g_o, g_h, ctr = search(gi, lens, codes, od, True)
    e_n, e_f, e_h, st = ox.cal_sa_reg_gap(lens, codes, Opt.from_dict(od))
    assert np.array_equal(g_n, e_n)
    assert np.array_equal(g_f & 1, e_f & 1)
    got = per_read(g_n, g_o, g_h)
    exp = split_hits(e_n, e_h)
    bad = [i for i in range(len(got)) if not np.array_equal(got[i], exp[i])]
    assert not bad, f"{len(bad)} reads differ from the 64-bit oracle; first {bad[0]}"
    assert int(ctr[2]) == int(st[0]), "rank queries"
    assert int(ctr[4]) == int(st[1]), "gap_pop count"
    hits = np.concatenate([x for x in got if len(x)])
    if wide_hits:
        assert (hits[:, 3] > 0).any(), "no hit with k >= 2^32"
    return e_n


def test_search_past_2_32_matches_oracle(big_index):
    """2 000 reads of 100 bp from the whole 4.3 Gbp text with an indel or
    substitutions, -n 4 -o 1 (8-bit pruning rows, 64-bit intervals)."""
    from hsa_amd import synth
    from oracle_ctypes import default_opt
    gi, ox, genome = big_index
    recs = [(0, BIG_T)]
    r1, _ = synth.make_reads(genome, recs, 1000, 100, 31, max_mm=3)
    r2, _ = synth.make_reads(genome, recs, 1000, 100, 32, indel=True, max_mm_indel=1)
    od = default_opt()
    od.update(max_diff=4, fnr=-1.0, max_gapo=1)
    od["mode"] &= ~0x01
    e_n = _check_past_2_32(gi, ox, np.concatenate([r1, r2]), od)
    assert (e_n > 0).mean() > 0.9


@pytest.mark.parametrize("one_lane", [False, True])
def test_config5_kernel_past_2_32_matches_oracle(big_index, monkeypatch, capfd, one_lane):
    """Config 5's own kernel instantiation: 250 bp reads, -n 4 -o 0, 64-bit intervals
    AND 4-bit pruning rows (the planner picks them by itself for long ungapped reads,
    as in the config-5 bench).  2 000 reads from the whole 4.3 Gbp text with 0-4
    substitutions, half reverse-complemented (make_reads), 1 in 50 with an N; every
    hsa_aln64_t field of every hit, the splice-fallback flags and the rank-query and pop
    counts equal the 64-bit restatement's, and hits with SA bounds past 2^32 occur.
    one_lane: the main pass of a large batch -- one read per lane, the lazy forward
    rows and their forward pass, the cost order -- forced on this small one."""
    from hsa_amd import synth
    from oracle_ctypes import default_opt
    monkeypatch.setenv("HSA_VERBOSE", "1")
    monkeypatch.delenv("HSA_WFMT", raising=False)
    if one_lane:
        monkeypatch.setenv("HSA_SPLIT", "0")
        monkeypatch.setenv("HSA_LAZY", "1")
        monkeypatch.setenv("HSA_ORDER", "1")
    gi, ox, genome = big_index
    reads, _ = synth.make_reads(genome, [(0, BIG_T)], 2000, 250, 8 * 1_000_000 + 77, max_mm=4)
    reads = reads.copy()
    rng = np.random.default_rng(5)
    for r in range(0, len(reads), 50):
        reads[r, int(rng.integers(0, 250))] = 4
    od = default_opt()
    od.update(max_diff=4, fnr=-1.0, max_gapo=0)
    od["mode"] &= ~0x01
    e_n = _check_past_2_32(gi, ox, reads, od)
    err = capfd.readouterr().err
    assert "4-bit rows" in err, "config 5's 4-bit-row instantiation was not the one that ran"
    assert (e_n > 0).mean() > 0.9
