"""Multi-rank path on CPU (gloo, world_size 2): whole batches round-robin over
ranks, the option-state exchange, and the hit-list gather to rank 0 must give
exactly the sequential reference's result (hsa_amd/shard.py).

The search callable here is the oracle (the CPU restatement: no GPU in this
container); on the GPU box bench.py plugs the HIP search into the same driver."""
import multiprocessing as mp
import queue
import socket

import numpy as np
import pytest

from golden_io import INDEX, load_case, parse_opts, split_hits
from shard_worker import _inputs, _worker

CASES = {
    # 1200 reads in 400-read batches, unmappable reads in batch 0: the Q2 regime switch
    "tiny_gap100_n4o1_b400": dict(batch=400),
    # 2000 exact reads in 7 batches of 300: more batches than ranks, a ragged last one
    "tiny_exact36_n0": dict(batch=300),
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sequential(name, batch, short_reads):
    from hsa_amd import index_io
    from oracle_ctypes import OracleIndex, default_opt
    g = load_case(name)
    lens, codes = _inputs(g, short_reads)
    fwd, rev = index_io.read_index(INDEX[g["index"]])
    return OracleIndex(fwd, rev).run_batches(lens, codes, parse_opts(g["args"], default_opt()), batch)[:3]


PARAMS = [("tiny_gap100_n4o1_b400", False), ("tiny_exact36_n0", False), ("tiny_exact36_n0", True)]


@pytest.mark.parametrize("name,short_reads", PARAMS)
def test_two_ranks_equal_sequential(name, short_reads):
    _two_ranks(name, short_reads, use_gpu=False)


@pytest.mark.parametrize("name,short_reads", [("tiny_exact36_n0", False), ("tiny_exact36_n0", True),
                                              ("tiny_gap100_n4o1_b400", False)])
def test_three_ranks_ragged_equal_sequential(name, short_reads):
    """World size 3: 7 batches of 300 reads (the last one 200) give the ranks 3, 2 and 2
    batches; tiny_gap100 has 3 batches, one per rank, its first with the Q2 regime switch.
    The fixed-total mode of bench.py (--total-reads) drives this same sharding."""
    _two_ranks(name, short_reads, use_gpu=False, world=3)


@pytest.mark.gpu
@pytest.mark.parametrize("name,short_reads", PARAMS)
def test_two_ranks_gpu_search_equal_sequential(name, short_reads):
    """Same driver with the HIP search in each rank (both ranks on the box's one GPU)."""
    _two_ranks(name, short_reads, use_gpu=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name,short_reads", [("tiny_gap100_n4o1_b400", False), ("tiny_exact36_n0", True)])
def test_one_rank_rccl_gather_equal_sequential(name, short_reads):
    """The bench's RCCL path (the `nccl` backend: bench.py's all-reduce of the
    option-state flags and its hit-list gather, hsa_amd/shard.py) executed on the box's
    GPU at world size 1, with the HIP search: the gathered lists equal the sequential
    reference's."""
    _two_ranks(name, short_reads, use_gpu=True, world=1, backend="nccl")


def _two_ranks(name, short_reads, use_gpu, world=2, backend="gloo"):
    batch = CASES[name]["batch"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, batch, short_reads, q, use_gpu, backend))
             for r in range(world)]
    for p in procs:
        p.start()
    out = None
    for _ in range(600):
        try:
            out = q.get(timeout=1)
            break
        except queue.Empty:
            assert all(p.exitcode in (None, 0) for p in procs), [p.exitcode for p in procs]
    assert out is not None
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    (n_aln, flags, hits), info = out
    assert info["backend"] == backend
    if world > 1:
        # rank 0 holds batches 0, 2, 4, ...: with the short reads in batch 0, its later
        # batches must have been searched again with the sticky seed_len
        assert info["first_sticky"] == (0 if short_reads else None)
        assert bool(info["rerun"]) == short_reads
    e_n, e_f, e_h = _sequential(name, batch, short_reads)
    assert np.array_equal(n_aln, e_n)
    assert np.array_equal(flags, e_f)
    got, exp = split_hits(n_aln, hits), split_hits(e_n, e_h)
    assert all(np.array_equal(a, b) for a, b in zip(got, exp))
    if not short_reads:
        # and the sequential oracle is the reference itself on these reads (main path)
        g = load_case(name)
        ref = split_hits(g["n_aln"], g["hits"])
        sp = (g["flags"] & 1).astype(bool)
        assert np.array_equal((flags & 1).astype(bool), sp)
        assert all(np.array_equal(got[i], ref[i]) for i in range(len(got)) if not sp[i])
