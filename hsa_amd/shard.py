"""Read sharding over ranks: one process per GPU, whole reference batches per rank.

The reference's host loop calls bwa_cal_sa_reg_gap once per 100 000-read batch
(bwtaln.c:477, :506).  Reads are independent, so ranks take whole batches round-robin
and search them without any communication: every GPU holds the whole index.

Batches are NOT quite independent in the reference, because the call mutates the
caller's option block:
  * the first call clears BWA_MODE_GAPE in *opt before searching (bwtaln.c:261), so
    every later batch starts with GAPE cleared, while batch 0's local_opt keeps it;
  * in the part of a batch searched with the caller's block (reads up to the first
    splice-fallback read, bwtaln.c:363), a read of length <= seed_len sets
    opt->seed_len = 0x7fffffff (bwtaln.c:332), and it never changes back.
So a rank that starts at batch b > 0 enters with GAPE cleared.  Whether seed_len is
already "sticky" depends on earlier batches searched elsewhere.  That is the one real
exchange the sharded path has: after the first pass every rank all-reduces
(MAX) a per-batch "turned sticky" flag.  Batches after the first such batch that were
searched with the non-sticky block are then searched again.  (No configuration of
BASELINE.json has reads that short, so the second pass is normally empty.)

Then the per-batch results are gathered to rank 0 (RCCL over xGMI for GPU tensors,
gloo in the CPU tests): the final hit-list gather of SURVEY §8e.
"""
from __future__ import annotations

import numpy as np

GAPE = 0x01
SEED_NONE = 0x7FFFFFFF


def batch_bounds(n_reads: int, batch: int):
    return [(b0, min(b0 + batch, n_reads)) for b0 in range(0, n_reads, batch)]


def my_batches(n_batches: int, world: int, rank: int):
    return list(range(rank, n_batches, world))


def opt_entering_batch(opt0: dict, b: int, sticky_seed: bool) -> dict:
    """The caller's option block as the sequential reference has it when batch b starts."""
    o = dict(opt0)
    if b > 0:
        o["mode"] &= ~GAPE
    if sticky_seed:
        o["seed_len"] = SEED_NONE
    return o


def search_sharded(search, make_opt, opt0: dict, lens, codes, batch: int, world: int, rank: int, allreduce_max,
                   info: dict | None = None):
    """Search this rank's batches with the sequential reference's option state.

    search(lens, codes, opt) -> (n_aln, flags, hit_off, hits) mutates opt like
    bwa_cal_sa_reg_gap; make_opt(dict) builds the option object it takes.
    allreduce_max(np.int32 array) -> elementwise max over ranks.
    Returns {batch index: (n_aln, flags, hit_off, hits)}; `info` (optional) receives
    the first batch that made seed_len sticky and the batches searched again."""
    lens = np.asarray(lens, np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    bounds = batch_bounds(len(lens), batch)
    mine = my_batches(len(bounds), world, rank)
    res = {}
    turned = np.zeros(len(bounds), np.int32)

    def run(b, sticky):
        b0, b1 = bounds[b]
        o = make_opt(opt_entering_batch(opt0, b, sticky))
        r = search(lens[b0:b1], codes[offs[b0]:offs[b1]], o)
        return r, int(o.seed_len) == SEED_NONE

    for b in mine:
        res[b], sticky_out = run(b, False)
        turned[b] = int(sticky_out and opt0["seed_len"] != SEED_NONE)
    turned = allreduce_max(turned)
    hit = np.flatnonzero(turned)
    rerun = []
    if len(hit):
        first = int(hit[0])
        for b in mine:
            if b > first:
                res[b], _ = run(b, True)
                rerun.append(b)
    if info is not None:
        info["first_sticky"] = int(hit[0]) if len(hit) else None
        info["rerun"] = rerun
    return res


def pack(res: dict) -> np.ndarray:
    """Per-batch results as one int32 stream: [b, n, nh, hw] + n_aln + flags + hits
    (hw = words per hit record: 9 for bwt_aln1_t, 14 for hsa_aln64_t)."""
    parts = []
    for b in sorted(res):
        n_aln, flags, hoff, hits = res[b]
        n = len(n_aln)
        hits = np.asarray(hits, np.uint32)
        hw = int(hits.shape[1]) if hits.ndim == 2 else 9
        hits = hits.reshape(-1, hw)
        # hits in read order (hit_off may point anywhere in the batch's hit array)
        cnt = np.maximum(np.asarray(n_aln, np.int64), 0)
        tot = int(cnt.sum())
        if tot:
            idx = np.repeat(np.asarray(hoff, np.int64) - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt) + \
                np.arange(tot)
            h = hits[idx]
        else:
            h = np.zeros((0, hw), np.uint32)
        parts += [np.array([b, n, tot, hw], np.int32), np.asarray(n_aln, np.int32),
                  np.asarray(flags, np.uint32).view(np.int32), np.ascontiguousarray(h).reshape(-1).view(np.int32)]
    return np.concatenate(parts) if parts else np.zeros(0, np.int32)


def unpack(buf: np.ndarray) -> dict:
    out, i = {}, 0
    while i < len(buf):
        b, n, nh, hw = (int(x) for x in buf[i:i + 4])
        i += 4
        n_aln = buf[i:i + n].copy()
        i += n
        flags = buf[i:i + n].view(np.uint32).copy()
        i += n
        hits = buf[i:i + hw * nh].view(np.uint32).reshape(nh, hw).copy()
        i += hw * nh
        out[b] = (n_aln, flags, hits)
    return out


def gather_to_root(res: dict, dist, device, root: int = 0, per_batch: bool = False):
    """Gather every rank's packed results to `root` (sizes first, then one padded
    gather).  Returns (n_aln, flags, hits) over all reads in global order on root (or,
    with per_batch, {batch: (n_aln, flags, hits)}), None elsewhere."""
    import torch
    mine = torch.from_numpy(pack(res)).to(device)
    world = dist.get_world_size()
    n = torch.tensor([mine.numel()], dtype=torch.int64, device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    m = int(max(int(s.item()) for s in sizes))
    buf = torch.zeros(max(m, 1), dtype=torch.int32, device=device)
    buf[:mine.numel()] = mine
    rank = dist.get_rank()
    bufs = [torch.zeros_like(buf) for _ in range(world)] if rank == root else None
    dist.gather(buf, bufs, dst=root)
    if rank != root:
        return None
    allres = {}
    for r in range(world):
        allres.update(unpack(bufs[r][:int(sizes[r].item())].cpu().numpy()))
    if per_batch:
        return allres
    bs = sorted(allres)
    n_aln = np.concatenate([allres[b][0] for b in bs]) if bs else np.zeros(0, np.int32)
    flags = np.concatenate([allres[b][1] for b in bs]) if bs else np.zeros(0, np.uint32)
    hits = np.concatenate([allres[b][2] for b in bs]) if bs else np.zeros((0, 9), np.uint32)
    return n_aln, flags, hits
