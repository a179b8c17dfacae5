"""Rank body of tests/test_shard_gloo.py (its own module so that a spawned rank
imports hsa_amd before torch, as the package requires)."""
import os

import hsa_amd  # noqa: F401  (before torch)
import numpy as np

from golden_io import INDEX, load_case, parse_opts


def _worker(rank, world, port, name, batch, short_reads, q, use_gpu=False, backend="gloo"):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":      # RCCL: the collectives on the rank's GPU, as bench.py does
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        comm = torch.device("cuda", 0)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        comm = torch.device("cpu")
    try:
        from hsa_amd import index_io, shard
        from oracle_ctypes import Opt, OracleIndex, default_opt
        g = load_case(name)
        lens, codes = _inputs(g, short_reads)
        fwd, rev = index_io.read_index(INDEX[g["index"]])
        opt0 = parse_opts(g["args"], default_opt())
        if use_gpu:
            # the HIP search (every rank on the one GPU of the box; gloo carries the collectives)
            from hsa_amd import _lib
            gi = _lib.GpuIndex(fwd, rev, device=0)
            make_opt = _lib.GapOpt.from_dict

            def search(l, c, o):
                n_aln, flags, hoff, hits, _ = gi.cal_sa_reg_gap(l, c, o)
                return n_aln, flags, hoff, hits
        else:
            ox = OracleIndex(fwd, rev)
            make_opt = Opt.from_dict

            def search(l, c, o):
                n_aln, flags, hits, _ = ox.cal_sa_reg_gap(l, c, o)
                hoff = np.concatenate([[0], np.cumsum(np.maximum(n_aln, 0))[:-1]]).astype(np.uint64)
                return n_aln, flags, hoff, hits

        def allreduce_max(a):
            t = torch.from_numpy(a.astype(np.int64)).to(comm)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return t.cpu().numpy().astype(np.int32)

        info = {}
        res = shard.search_sharded(search, make_opt, opt0, lens, codes, batch, world, rank, allreduce_max, info)
        out = shard.gather_to_root(res, dist, comm)
        if rank == 0:
            info["backend"] = dist.get_backend()
            q.put((out, info))
    finally:
        dist.destroy_process_group()


def _inputs(g, short_reads):
    lens, codes = g["lens"].copy(), g["codes"].copy()
    if short_reads:
        # shorten two reads of batch 0 to 30 bp (<= seed_len): in the reference this
        # makes opt->seed_len sticky for every later batch (bwtaln.c:332)
        offs = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
        keep = np.ones(len(codes), bool)
        for i in (5, 17):
            keep[offs[i] + 30:offs[i + 1]] = False
            lens[i] = 30
        codes = codes[keep]
    return lens, codes
