"""bench.py's full-batch parity comparison (CPU only): GPU hit lists, allocated in
arbitrary order by the search kernel's atomics, against the oracle's in read order."""
import os
import sys

import numpy as np

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
