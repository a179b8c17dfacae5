"""Parity at the size north_star names: the hg19-sized (3 000 000 005 bp) index the
bench uses, built on the device, with >= 20 000 reads of each of the config-2 and
config-3 workloads through the device path, compared field by field (and in hit
order) with the C restatement run on the same reads -- so the u32 interval
arithmetic near T = 3e9 (l + 1, rev_l = rev_k + (l - k), the oCount subtractions;
SURVEY Q8) is exercised by the GPU suite.  The rank-query count is checked too."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

N_READS = 20000
_IX = {}


def _index():
    import bench
    if not _IX:
        import torch
        gi, res, _ = bench.build_index(bench.GENOME_T, bench.GENOME_SEED, torch.cuda.current_device())
        _IX["gi"], _IX["ox"] = gi, bench.host_oracle_index(res, bench.GENOME_T)
        del res
    return _IX["gi"], _IX["ox"]


@pytest.mark.parametrize("config", [2, 3])
def test_hg19_sized_batch_matches_oracle(config):
    import torch

    import bench
    from hsa_amd import _lib, synth
    from hsa_amd._lib import DeviceBatch, GapOpt, Regime
    from oracle_ctypes import default_opt
    gi, ox = _index()
    T = bench.GENOME_T
    genome = synth.PackedGenome(T, bench.GENOME_SEED)
    recs = synth.record_layout(T, bench.RECORDS)
    if config == 2:
        reads, _ = synth.make_reads(genome, recs, N_READS, 100, 5 * 1_000_000 + 77, max_mm=4)
    else:
        reads, _ = synth.make_reads(genome, recs, N_READS, 100, 6 * 1_000_000 + 77, indel=True, max_mm_indel=2)
    max_gapo = 0 if config == 2 else 1
    opt = GapOpt.default()
    opt.max_diff, opt.fnr, opt.max_gapo = 4, -1.0, max_gapo
    opt.mode &= ~0x01
    n_stacks = (opt.max_diff + 1) * opt.s_mm + (opt.max_gapo + 1) * opt.s_gapo + (opt.max_gape + 1) * opt.s_gape
    rg = Regime(s_mm=opt.s_mm, s_gapo=opt.s_gapo, s_gape=opt.s_gape, mode=0, indel_end_skip=opt.indel_end_skip,
                max_del_occ=opt.max_del_occ, max_entries=opt.max_entries, max_gapo=max_gapo, max_gape=opt.max_gape,
                max_seed_diff=opt.max_seed_diff, max_top2=opt.max_top2, n_stacks=n_stacks, max_diff=opt.max_diff)
    jobs = np.zeros(N_READS, _lib.JOB_DTYPE)
    jobs["off"] = np.arange(N_READS, dtype=np.uint64) * 100
    jobs["len"] = 100
    jobs["max_diff"] = opt.max_diff
    jobs["seed_len"] = opt.seed_len
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).cuda()
    d_codes = torch.from_numpy(_lib.pad_codes(reads.reshape(-1))).cuda()
    cap = N_READS * 8
    t = dict(n=torch.zeros(N_READS, dtype=torch.int32, device="cuda"),
             f=torch.zeros(N_READS, dtype=torch.int32, device="cuda"),
             o=torch.zeros(N_READS, dtype=torch.int64, device="cuda"),
             h=torch.zeros(cap * 9, dtype=torch.int32, device="cuda"),
             c=torch.zeros(16, dtype=torch.int64, device="cuda"))
    gi.search_device([rg], DeviceBatch(d_jobs=d_jobs.data_ptr(), n_jobs=N_READS, d_codes=d_codes.data_ptr(),
                                       d_n_aln=t["n"].data_ptr(), d_flags=t["f"].data_ptr(),
                                       d_hit_off=t["o"].data_ptr(), d_hits=t["h"].data_ptr(), hit_cap=cap,
                                       d_counters=t["c"].data_ptr(), max_len=100, max_seed=opt.seed_len))
    torch.cuda.synchronize()
    c = t["c"].cpu().numpy()
    assert c[11] == 0
    od = default_opt()
    od.update(max_diff=4, fnr=-1.0, max_gapo=max_gapo, mode=od["mode"] & ~0x01)
    o_n, o_f, o_h, o_q = bench.oracle_threaded(ox, reads, 100, od, bench.cpu_info()["threads"])
    bad, first = bench.compare_batch(t["n"].cpu().numpy(), t["f"].cpu().numpy().astype(np.uint32),
                                     t["o"].cpu().numpy(), t["h"].cpu().numpy().view(np.uint32).reshape(-1, 9),
                                     o_n, o_f, o_h)
    assert bad == 0, f"{bad} of {N_READS} reads differ; first {first}"
    assert (o_n > 0).mean() > 0.9                     # the batch really maps (not a vacuous pass)
    if c[8] == 0:                                     # no capacity re-run: every query counted once
        assert int(c[2]) == int(o_q), (int(c[2]), int(o_q))


def _device_batch(reads, max_gapo):
    """Jobs, outputs and the DeviceBatch of one fixed-length 100 bp batch (bench.py's layout)."""
    import torch

    from hsa_amd import _lib
    from hsa_amd._lib import DeviceBatch, GapOpt, Regime
    n = len(reads)
    opt = GapOpt.default()
    opt.max_diff, opt.fnr, opt.max_gapo = 4, -1.0, max_gapo
    opt.mode &= ~0x01
    n_stacks = (opt.max_diff + 1) * opt.s_mm + (opt.max_gapo + 1) * opt.s_gapo + (opt.max_gape + 1) * opt.s_gape
    rg = Regime(s_mm=opt.s_mm, s_gapo=opt.s_gapo, s_gape=opt.s_gape, mode=0, indel_end_skip=opt.indel_end_skip,
                max_del_occ=opt.max_del_occ, max_entries=opt.max_entries, max_gapo=max_gapo, max_gape=opt.max_gape,
                max_seed_diff=opt.max_seed_diff, max_top2=opt.max_top2, n_stacks=n_stacks, max_diff=opt.max_diff)
    jobs = np.zeros(n, _lib.JOB_DTYPE)
    jobs["off"] = np.arange(n, dtype=np.uint64) * 100
    jobs["len"] = 100
    jobs["max_diff"] = opt.max_diff
    jobs["seed_len"] = opt.seed_len
    t = dict(j=torch.from_numpy(jobs.view(np.uint8).copy()).cuda(),
             r=torch.from_numpy(_lib.pad_codes(reads.reshape(-1))).cuda(),
             n=torch.zeros(n, dtype=torch.int32, device="cuda"), f=torch.zeros(n, dtype=torch.int32, device="cuda"),
             o=torch.zeros(n, dtype=torch.int64, device="cuda"), h=torch.zeros(n * 8 * 9, dtype=torch.int32, device="cuda"),
             c=torch.zeros(16, dtype=torch.int64, device="cuda"))
    b = DeviceBatch(d_jobs=t["j"].data_ptr(), n_jobs=n, d_codes=t["r"].data_ptr(), d_n_aln=t["n"].data_ptr(),
                    d_flags=t["f"].data_ptr(), d_hit_off=t["o"].data_ptr(), d_hits=t["h"].data_ptr(), hit_cap=n * 8,
                    d_counters=t["c"].data_ptr(), max_len=100, max_seed=opt.seed_len)
    return rg, b, t


def test_hg19_sized_clones_search_concurrently():
    """hsa_index_clone: three batches of 100 000 reads issued back to back on two handles
    of the same resident index without a synchronisation between them (bench.py
    --streams 2), so the second handle's launches overlap the first's.  Every batch is
    compared with the restatement, and its counters with a serialized run on one handle."""
    import torch

    import bench
    from hsa_amd import synth
    from hsa_amd._lib import HsaError
    from oracle_ctypes import default_opt
    gi, ox = _index()
    cl = gi.clone()
    genome = synth.PackedGenome(bench.GENOME_T, bench.GENOME_SEED)
    recs = synth.record_layout(bench.GENOME_T, bench.RECORDS)
    n = 100_000
    sets = [synth.make_reads(genome, recs, n, 100, 5 * 1_000_000 + 91 + i, max_mm=4)[0] for i in range(3)]
    bat = [_device_batch(r, 0) for r in sets]
    for i, (rg, b, _) in enumerate(bat):
        (gi if i % 2 == 0 else cl).search_device([rg], b)
    torch.cuda.synchronize()
    conc = [{k: t[k].cpu().numpy().copy() for k in "nfohc"} for _, _, t in bat]
    od = default_opt()
    od.update(max_diff=4, fnr=-1.0, max_gapo=0, mode=od["mode"] & ~0x01)
    for i, (rg, b, t) in enumerate(bat):
        o_n, o_f, o_h, o_q = bench.oracle_threaded(ox, sets[i], 100, od, bench.cpu_info()["threads"])
        g = conc[i]
        assert g["c"][11] == 0
        bad, first = bench.compare_batch(g["n"], g["f"].astype(np.uint32), g["o"], g["h"].view(np.uint32).reshape(-1, 9),
                                         o_n, o_f, o_h)
        assert bad == 0, f"batch {i}: {bad} of {n} reads differ; first {first}"
        if g["c"][8] == 0:
            assert int(g["c"][2]) == int(o_q)
        cl.search_device([rg], b)                     # serialized, on the clone alone
        torch.cuda.synchronize()
        np.testing.assert_array_equal(t["c"].cpu().numpy()[[1, 2, 4, 7, 8, 11]], g["c"][[1, 2, 4, 7, 8, 11]])
    # the shared arrays cannot be replaced under a clone
    from hsa_amd import index_io
    one = index_io.SaFile(interval=8, values=np.zeros(1, np.uint32))
    with pytest.raises(HsaError, match="clone"):
        cl.set_sa(one, np.zeros((0, 4), np.uint32))
    with pytest.raises(HsaError, match="clone"):
        gi.set_sa(one, np.zeros((0, 4), np.uint32))
    cl.close()
