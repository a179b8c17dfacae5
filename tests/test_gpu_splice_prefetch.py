"""The splice path's prefetch on the device (hsa_splice_prefetch_batch, include/hsa_gpu.h):
for every read of the drop-in's splice read set, each width row, seed search, 12-mer
anchor search and SA -> position lookup bwt_splice_match (bwtgap.c:748-1332) can make
before its first extension equals the CPU restatement's (oracle/hsa_oracle.c, pinned
against the reference's recorded bwt_match_gap calls in tests/test_oracle.py):

* rows: bwt_cal_width type 1 of each strand and of its last 12 bases, type 0 of each
  strand (bwtaln.c:73-116);
* the six seed calls (bwtgap.c:797-812: the strand prefix's widths, width_seed aliased)
  and the anchors of the strands whose seed hit pattern is 3 or 6 (bwtgap.c:911-919,
  :1187-1192): hit counts, every word of every hit, width_back after gap_shadow;
* SA -> position of k .. min(l, k + 49) of every hit (bwt_aln_corelate_check,
  bwtgap.c:698, :711).

The end-to-end check -- the reference's HSA aln with these answers inside prints the
reference's SAM byte for byte -- is tests/test_gpu_dropin.py."""
import gzip
import json
import os

import numpy as np
import pytest

from golden_io import GOLD, INDEX, parse_opts
from hsa_amd import index_io

pytestmark = pytest.mark.gpu

NT4 = np.full(256, 4, np.uint8)
for _i, _c in enumerate(b"ACGT"):
    NT4[_c] = NT4[_c + 32] = _i


def fastq_codes(path):
    lines = gzip.open(path, "rt").read().split("\n")
    return [NT4[np.frombuffer(lines[i + 1].encode(), np.uint8)] for i in range(0, len(lines) - 3, 4)]


@pytest.mark.parametrize("args", ["-n 4 -o 1", "-n 4 -o 0", "-n 2 -o 1 -e 3"])
def test_splice_prefetch_matches_oracle(args):
    from hsa_amd._lib import GpuIndex, regime_of
    from oracle_ctypes import Opt, OracleIndex, default_opt
    man = json.load(open(os.path.join(GOLD, "manifest_dropin.json")))
    reads = [r for r in fastq_codes(os.path.join(GOLD, man["splice_reads"])) if len(r) >= 3]
    prefix = INDEX[man["index"]]
    fwd, rev = index_io.read_index(prefix)
    gi = GpuIndex(fwd, rev)
    sa, blocks = index_io.read_sa(prefix), index_io.read_blocks(prefix)
    gi.set_sa(sa, blocks)
    ox = OracleIndex(fwd, rev)
    od = parse_opts(args.split(), default_opt())                 # local_opt as the splice path receives it
    n_stacks = (od["max_diff"] + 1) * od["s_mm"] + (od["max_gapo"] + 1) * od["s_gapo"] + \
        (od["max_gape"] + 1) * od["s_gape"]
    so = dict(od, max_gapo=0, max_gape=0, max_diff=od["max_seed_diff"], mode=od["mode"] & ~0x01)   # bwtgap.c:769-774
    ao = dict(od, max_gape=3)                                                                      # bwtgap.c:777-782
    rng = np.random.default_rng(3)
    amd = rng.integers(0, od["max_diff"] + 1, len(reads)).astype(np.int32)    # per-read max_diff (bwtaln.c:330)
    lens = np.array([len(r) for r in reads], np.uint32)
    got = gi.splice_prefetch(regime_of(so, n_stacks, so["max_diff"]), regime_of(ao, n_stacks, od["max_diff"]),
                             lens, np.concatenate(reads), amd)
    gi.close()
    n_calls = {"seed": 0, "anchor": 0, "hits": 0, "sa": 0}
    for r, seq in enumerate(reads):
        L, sl = len(seq), len(seq) // 3
        ss = [seq, np.where(seq[::-1] < 4, 3 - seq[::-1], seq[::-1]).astype(np.uint8)]
        w1 = [ox.cal_width(x).astype(np.int32) for x in ss]
        for s in range(2):
            assert np.array_equal(got["rows"][r, s, :L + 1], w1[s]), (r, s, "type 1")
            if L >= 12:
                assert np.array_equal(got["rows"][r, 2 + s, :13], ox.cal_width(ss[s][L - 12:]).astype(np.int32))
            assert np.array_equal(got["rows"][r, 4 + s, 1:L + 1], ox.cal_width0(ss[s]).astype(np.int32)[1:]), (r, s)
        calls = []
        for c in range(6):
            s, t = c // 3, c % 3
            la = sl + (L % 3 if t == 2 else 0)
            w = np.concatenate([w1[s][:la], [[0, (w1[s][la - 1, 1] if la else 0) + 1]]]).astype(np.int32)
            calls.append((c, Opt.from_dict(dict(so, seed_len=la)), ss[s][t * sl:t * sl + la], s, w, 2))
        for s in range(2):
            c = 6 + s
            hit = [got["call_n"][r, 3 * s + t] > 0 for t in range(3)]
            mask = hit[0] | hit[1] << 1 | hit[2] << 2
            if L <= 12 or mask not in (3, 6):
                assert got["call_n"][r, c] == -1, (r, c)
                continue
            tail = mask == 3
            w = (ox.cal_width(ss[s][L - 12:]) if tail else w1[s][:13]).astype(np.int32)
            calls.append((c, Opt.from_dict(dict(ao, max_diff=int(amd[r]))), ss[s][L - 12:] if tail else ss[s][:12],
                          s, w, 0))
        for c, o, q, s, w, kind in calls:
            exp, w_after = ox.match_gap(o, n_stacks, q, s, w, kind)
            na = int(got["call_n"][r, c])
            assert na == len(exp), (r, c, na, len(exp))
            h0 = int(got["call_hit"][r, c])
            assert np.array_equal(got["hits"][h0:h0 + na], exp), (r, c)
            assert np.array_equal(got["wafter"][r, c, :len(q) + 1], w_after), (r, c, "width_back after")
            n_calls["seed" if c < 6 else "anchor"] += 1
            n_calls["hits"] += na
            if na:
                idx = np.concatenate([np.arange(int(h[1]), min(int(h[2]), int(h[1]) + 49) + 1, dtype=np.int64)
                                      for h in exp if int(h[1]) <= int(h[2])] or [np.zeros(0, np.int64)])
                s0 = int(got["call_sa"][r, c])
                assert np.array_equal(got["sa"][s0:s0 + len(idx)], ox.sa_positions(sa, blocks, idx)), (r, c, "SA")
                n_calls["sa"] += len(idx)
    assert n_calls["anchor"] > 0 and n_calls["hits"] > 0 and n_calls["sa"] > 0, n_calls
