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
