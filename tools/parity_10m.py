"""Bit-exact parity at the size north_star names: 10 M x 100 bp synthetic reads against
the hg19-sized (3 000 000 005 bp) index, searched on the GPU in 1 M-read batches
(the bench's device path: hsa_search_device = k_widths + k_search + capacity
re-runs) and every batch compared with the C restatement (oracle/, threaded over
disjoint chunks on the host cores) field by field: n_aln, the splice-fallback flag,
every bwt_aln1_t field of every hit and the hit order (bwtaln.c:303-373), plus the
rank-query count of each batch.

The read stream is the bench's (hsa_amd.synth, seeds 5e6 + j for config 2 and
6e6 + j for config 3), so batch j is the bench's global batch j.  Test
infrastructure: the oracle is the checker, never the thing measured.

    python tools/parity_10m.py --config 2 --batches 10 --out gpurun_out/parity10m_c2.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import hsa_amd  # noqa: E402,F401  (loads libhsa_gpu.so before torch)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2, choices=(2, 3))
    ap.add_argument("--batches", type=int, default=10)
    ap.add_argument("--first", type=int, default=0, help="global index of the first batch (a run split over calls)")
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--max-seconds", type=float, default=0, help="stop after the batch that passes this wall time")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch

    import bench
    from hsa_amd import _lib, synth
    from hsa_amd._lib import DeviceBatch, GapOpt, Regime
    from oracle_ctypes import default_opt

    t_start = time.perf_counter()
    T, RL, N = bench.GENOME_T, bench.READ_LEN, a.batch
    gi, res, _ = bench.build_index(T, bench.GENOME_SEED, torch.cuda.current_device())
    ox = bench.host_oracle_index(res, T)
    del res
    genome = synth.PackedGenome(T, bench.GENOME_SEED)
    recs = synth.record_layout(T, bench.RECORDS)
    max_gapo = 0 if a.config == 2 else 1
    opt = GapOpt.default()
    opt.max_diff, opt.fnr, opt.max_gapo = 4, -1.0, max_gapo
    opt.mode &= ~0x01
    n_stacks = (opt.max_diff + 1) * opt.s_mm + (opt.max_gapo + 1) * opt.s_gapo + (opt.max_gape + 1) * opt.s_gape
    rg = Regime(s_mm=opt.s_mm, s_gapo=opt.s_gapo, s_gape=opt.s_gape, mode=0, indel_end_skip=opt.indel_end_skip,
                max_del_occ=opt.max_del_occ, max_entries=opt.max_entries, max_gapo=max_gapo, max_gape=opt.max_gape,
                max_seed_diff=opt.max_seed_diff, max_top2=opt.max_top2, n_stacks=n_stacks, max_diff=opt.max_diff)
    od = default_opt()
    od.update(max_diff=4, fnr=-1.0, max_gapo=max_gapo, mode=od["mode"] & ~0x01)
    threads = bench.cpu_info()["threads"]

    jobs = np.zeros(N, _lib.JOB_DTYPE)
    jobs["off"] = np.arange(N, dtype=np.uint64) * RL
    jobs["len"] = RL
    jobs["max_diff"] = opt.max_diff
    jobs["seed_len"] = opt.seed_len
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).cuda()
    cap = N * 8
    t = dict(n=torch.zeros(N, dtype=torch.int32, device="cuda"), f=torch.zeros(N, dtype=torch.int32, device="cuda"),
             o=torch.zeros(N, dtype=torch.int64, device="cuda"), h=torch.zeros(cap * 9, dtype=torch.int32, device="cuda"),
             c=torch.zeros(16, dtype=torch.int64, device="cuda"))

    per = []
    tot = dict(reads=0, mismatching_reads=0, mapped=0, fallback=0, hits=0, rank_queries_gpu=0, rank_queries_oracle=0,
               gpu_s=0.0, oracle_s=0.0)
    for j in range(a.first, a.first + a.batches):
        t0 = time.perf_counter()
        if a.config == 2:
            reads, _ = synth.make_reads(genome, recs, N, RL, 5 * 1_000_000 + j, max_mm=4)
        else:
            reads, _ = synth.make_reads(genome, recs, N, RL, 6 * 1_000_000 + j, indel=True, max_mm_indel=2)
        d_codes = torch.from_numpy(_lib.pad_codes(reads.reshape(-1))).cuda()
        t1 = time.perf_counter()
        gi.search_device([rg], DeviceBatch(d_jobs=d_jobs.data_ptr(), n_jobs=N, d_codes=d_codes.data_ptr(),
                                           d_n_aln=t["n"].data_ptr(), d_flags=t["f"].data_ptr(),
                                           d_hit_off=t["o"].data_ptr(), d_hits=t["h"].data_ptr(), hit_cap=cap,
                                           d_counters=t["c"].data_ptr(), max_len=RL, max_seed=opt.seed_len))
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        c = t["c"].cpu().numpy()
        g_n, g_f = t["n"].cpu().numpy(), t["f"].cpu().numpy().astype(np.uint32)
        g_o, g_h = t["o"].cpu().numpy(), t["h"].cpu().numpy().view(np.uint32).reshape(-1, 9)
        o_n, o_f, o_h, o_q = bench.oracle_threaded(ox, reads, RL, od, threads)
        t3 = time.perf_counter()
        bad, first = bench.compare_batch(g_n, g_f, g_o, g_h, o_n, o_f, o_h)
        rec = dict(batch=j, reads=N, mismatching_reads=bad, first_mismatch=first, unfinished=int(c[11]),
                   mapped=int((o_n > 0).sum()), fallback=int((o_f & 1).sum()), hits=int(o_n.sum()),
                   rank_queries_gpu=int(c[2]), rank_queries_oracle=int(o_q), overflow_reruns=int(c[8]),
                   gpu_s=round(t2 - t1, 3), oracle_s=round(t3 - t2, 1))
        per.append(rec)
        for k in tot:
            tot[k] += rec[k] if k in rec else 0
        tot["gpu_s"] = round(tot["gpu_s"], 3)
        tot["oracle_s"] = round(tot["oracle_s"], 1)
        print(f"[parity10m] config {a.config} batch {j}: {N} reads, {bad} differ (first {first}), "
              f"unfinished {rec['unfinished']}, mapped {rec['mapped']}, hits {rec['hits']}, Q gpu {rec['rank_queries_gpu']} "
              f"oracle {rec['rank_queries_oracle']}; reads {t1 - t0:.1f} s, GPU {t2 - t1:.2f} s, oracle {t3 - t2:.1f} s "
              f"({threads} threads)", flush=True)
        del d_codes, reads
        if a.max_seconds and time.perf_counter() - t_start > a.max_seconds:
            break
    out = {"config": a.config, "options": f"-n 4 -o {max_gapo}", "genome_bp": T, "read_len": RL,
           "batches": len(per), "total": tot, "per_batch": per,
           "q_equal_every_batch": all(p["rank_queries_gpu"] == p["rank_queries_oracle"] for p in per
                                      if p["overflow_reruns"] == 0),
           "against": "oracle/hsa_oracle.c (C restatement, pinned to the compiled reference's golden vectors)",
           "fields": "n_aln, splice-fallback flag, every bwt_aln1_t field of every hit, hit order",
           "oracle_threads": threads, "wall_s": round(time.perf_counter() - t_start, 1)}
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    sys.exit(0 if tot["mismatching_reads"] == 0 else 1)


if __name__ == "__main__":
    main()
