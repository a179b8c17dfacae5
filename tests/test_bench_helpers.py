"""bench.py's full-batch parity comparison (CPU only): GPU hit lists, allocated in
arbitrary order by the search kernel's atomics, against the oracle's in read order."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _scrambled(rng, n):
    o_n = rng.integers(0, 4, n).astype(np.int32)
    o_f = (o_n == 0).astype(np.uint32)
    tot = int(o_n.sum())
    o_h = rng.integers(0, 2**32, (tot, 9), dtype=np.uint64).astype(np.uint32)
    # the GPU's layout: each read's hits contiguous, reads in a random order
    perm = rng.permutation(n)
    off = np.zeros(n, np.int64)
    g_h = np.zeros_like(o_h)
    o_off = np.concatenate([[0], np.cumsum(o_n.astype(np.int64))])
    pos = 0
    for r in perm:
        off[r] = pos
        g_h[pos:pos + o_n[r]] = o_h[o_off[r]:o_off[r + 1]]
        pos += o_n[r]
    return o_n, o_f, o_h, o_n.copy(), o_f.copy(), off, g_h


def test_compare_batch_identical_and_single_field_change():
    rng = np.random.default_rng(3)
    o_n, o_f, o_h, g_n, g_f, g_o, g_h = _scrambled(rng, 500)
    assert bench.compare_batch(g_n, g_f, g_o, g_h, o_n, o_f, o_h) == (0, None)
    r = int(np.flatnonzero(o_n >= 2)[7])
    g_h2 = g_h.copy()
    g_h2[g_o[r] + 1, 8] ^= 1                          # one score of one hit
    assert bench.compare_batch(g_n, g_f, g_o, g_h2, o_n, o_f, o_h) == (1, r)
    g_f2 = g_f.copy()
    z = int(np.flatnonzero(o_n == 0)[0])
    g_f2[z] ^= 1                                      # the splice-fallback flag
    assert bench.compare_batch(g_n, g_f2, g_o, g_h, o_n, o_f, o_h) == (1, z)
    g_n2 = g_n.copy()
    g_n2[r] -= 1                                      # a missing hit
    assert bench.compare_batch(g_n2, g_f, g_o, g_h, o_n, o_f, o_h)[0] == 1


def test_cpu_info_fields():
    c = bench.cpu_info()
    assert 1 <= c["threads"] <= 16 and c["affinity"] >= 1 and isinstance(c["model"], str)


def test_hits_in_read_order_and_digest():
    rng = np.random.default_rng(5)
    o_n, o_f, o_h, g_n, g_f, g_o, g_h = _scrambled(rng, 300)
    assert np.array_equal(bench.hits_in_read_order(g_n, g_o, g_h), o_h)
    d = bench.batch_digest(o_n, o_f, o_h)
    assert d == bench.batch_digest(g_n, g_f, bench.hits_in_read_order(g_n, g_o, g_h))
    h2 = o_h.copy()
    h2[3, 4] ^= 1
    assert bench.batch_digest(o_n, o_f, h2) != d


def test_shard_pack_roundtrip_scrambled():
    """shard.pack puts each read's hits in read order whatever the kernel's layout."""
    from hsa_amd import shard
    rng = np.random.default_rng(8)
    o_n, o_f, o_h, g_n, g_f, g_o, g_h = _scrambled(rng, 400)
    out = shard.unpack(shard.pack({7: (g_n, g_f, g_o, g_h)}))
    n_aln, flags, hits = out[7]
    assert np.array_equal(n_aln, o_n) and np.array_equal(flags, o_f) and np.array_equal(hits, o_h)


def test_spawn_ranks_sets_rank_env(tmp_path):
    """`bench.py --gpus N` without a launcher starts N ranks with the rendezvous
    environment and relays rank 0's JSON line alone to stdout (a stand-in script here: no GPU)."""
    script = tmp_path / "rank.py"
    script.write_text("import json, os, sys\n"
                      "r = int(os.environ['RANK'])\n"
                      "assert os.environ['LOCAL_RANK'] == str(r) and os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                      "if r == 0: print('[Gloo] Rank 0 is connected to 2 peer ranks.')\n"
                      "if r == 0: print(json.dumps({'world': int(os.environ['WORLD_SIZE']), 'argv': sys.argv[1:]}))\n")
    import contextlib
    import io
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bench.spawn_ranks(3, ["--gpus", "3"], script=str(script))
    assert rc == 0
    import json
    assert json.loads(buf.getvalue()) == {"world": 3, "argv": ["--gpus", "3"]}


def test_spawn_ranks_reports_a_failing_rank(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1': sys.exit(3)\n"
                      "time.sleep(30)\n")
    assert bench.spawn_ranks(2, [], script=str(script)) == 3


@pytest.mark.parametrize("S,nd,warmup", [(1, 3, 1), (2, 3, 1), (2, 3, 5), (3, 3, 2), (2, 2, 0), (4, 3, 1), (3, 1, 1)])
def test_step_plan_never_overlaps_writers_of_one_read_set(S, nd, warmup):
    """bench.py's timed loop over S handles: any two steps writing the same read set's
    outputs are ordered (same handle, or an event wait, transitively)."""
    steps = 40
    plan = bench.step_plan(steps, warmup, nd, S)
    before = [set() for _ in range(steps)]          # steps known to finish before step s starts
    last_on = {}
    for s, (hi, _, after) in enumerate(plan):
        preds = set()
        if hi in last_on:
            preds.add(last_on[hi])
        if after is not None:
            preds.add(after)
        for p in preds:
            before[s] |= before[p] | {p}
        last_on[hi] = s
    for b in range(steps):
        for a in range(b):
            if plan[a][1] == plan[b][1]:
                assert a in before[b], (a, b, plan[a], plan[b])
    assert [h for h, _, _ in plan[:S]] == list(range(S))


def test_parse_batch_stages_sums_the_calls():
    """bench.py's drop-in end-to-end leg: the per-call stage lines the drop-in prints under
    HSA_VERBOSE (bwtaln_gpu.c) -> stage sums, fallback reads, per-call totals."""
    err = "\n".join([
        "[hsa] launch: 256 CUs x 9 workgroups of 64 lanes, LDS 17296 B, 1563 workgroups, 39 buckets",
        "[hsa] batch of 100000 reads: search 0.177 s, splice prefetch 0.269 s, splice path 0.002 s (100000 fallback "
        "reads, 100000 on the device; per-read outputs 0.4 ms beside the device pass, 269.0 ms waited for)",
        "[hsa] splice kernel: 100000 reads, 54255 spliced, 0 to the host's path",
        "[hsa] batch of 100000 reads: search 0.176 s, splice prefetch 0.061 s, splice path 0.004 s (2362 fallback "
        "reads, 2362 on the device; per-read outputs 0.4 ms beside the device pass, 61.0 ms waited for)",
    ])
    splice_s, search_s, prefetch_s, n_fb, calls = bench.parse_batch_stages(err)
    assert n_fb == 102362
    assert abs(search_s - 0.353) < 1e-9 and abs(prefetch_s - 0.330) < 1e-9 and abs(splice_s - 0.006) < 1e-9
    assert len(calls) == 2 and abs(calls[0] - 0.448) < 1e-9 and abs(calls[1] - 0.241) < 1e-9
    assert bench.parse_batch_stages("no stage lines\n") == (0.0, 0.0, 0.0, 0, [])


def test_fixed_total_batch_codes_follow_search_sharded():
    """bench.py --total-reads: shard.search_sharded slices the global codes by batch
    (codes[offs[b0]:offs[b1]]); _BatchCodes holds only this rank's batches and hands each
    slice its batch.  With world 3 and a ragged 7-batch stream, rank 1 searches batches 1
    and 4 with the option state the sequential reference has there."""
    from hsa_amd import shard
    L, B, R, world, rank = 5, 4, 26, 3, 1
    bounds = shard.batch_bounds(R, B)
    mine = shard.my_batches(len(bounds), world, rank)
    assert len(bounds) == 7 and mine == [1, 4]
    reads = {b: np.full((bounds[b][1] - bounds[b][0], L), b, np.uint8) for b in mine}
    codes = bench._BatchCodes(reads, B * L)
    seen = []

    def search(lens, c, o):
        seen.append((int(c[0]), len(lens), len(c), o.mode & 1))
        return np.zeros(len(lens), np.int32), np.zeros(len(lens), np.uint32), np.zeros(len(lens), np.uint64), \
            np.zeros((0, 9), np.uint32)

    opt0 = {"mode": 0x03, "seed_len": 32}
    from types import SimpleNamespace
    out = shard.search_sharded(search, lambda d: SimpleNamespace(**d), opt0, np.full(R, L, np.uint32), codes, B, world, rank, lambda x: x)
    assert sorted(out) == [1, 4]
    assert seen == [(1, 4, 20, 0), (4, 4, 20, 0)]      # batch 1 and 4: GAPE already cleared
