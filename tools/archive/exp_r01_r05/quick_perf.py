#!/usr/bin/env python3
"""Quick throughput probe on one GPU: synthetic genome -> device BWT build ->
index -> search of synthetic reads.  Development aid (bench.py is the contract)."""
import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from hsa_amd import _lib, index_io, synth  # noqa: E402


def build_index_device(T, seed, n_records=1):
    import torch
    L = _lib.lib()
    nw = (T + 15) // 16
    text = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
    _lib.check(L.hsa_synth_genome_device(0, T, seed, text.data_ptr()))
    bw = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
    rbw = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
    isa0, risa0 = C.c_uint32(), C.c_uint32()
    Cf, Cr = np.zeros(5, np.uint32), np.zeros(5, np.uint32)
    t0 = time.time()
    _lib.check(L.hsa_build_bwt_device(0, T, text.data_ptr(), 0, bw.data_ptr(), C.byref(isa0), Cf))
    _lib.check(L.hsa_build_bwt_device(0, T, text.data_ptr(), 1, rbw.data_ptr(), C.byref(risa0), Cr))
    t1 = time.time()
    gi = _lib.GpuIndex.from_device_codes(T, isa0.value, Cf, bw.data_ptr(), T, risa0.value, Cr, rbw.data_ptr())
    t2 = time.time()
    del bw, rbw, text
    torch.cuda.empty_cache()
    return gi, t1 - t0, t2 - t1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=4641652)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--n", type=int, default=200000)
    ap.add_argument("--L", type=int, default=100)
    ap.add_argument("--mm", type=int, default=4)
    ap.add_argument("--args", default="-n 4 -o 0")
    ap.add_argument("--indel", action="store_true")
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--pool", type=int, default=0)
    a = ap.parse_args()
    _lib.configure(a.waves, a.pool, 0)
    gi, tb, ti = build_index_device(a.T, a.seed)
    print(f"index: T={a.T} build {tb:.2f}s relayout {ti:.2f}s bytes={gi.nbytes()}", flush=True)
    genome = synth.genome_codes(a.T, a.seed)
    rec = synth.record_layout(a.T, 1)
    reads, _ = synth.make_reads(genome, rec, a.n, a.L, 5, max_mm=a.mm, indel=a.indel)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_io import parse_opts
    opt = parse_opts(a.args.split(), _lib.GapOpt.default().as_dict())
    lens = np.full(a.n, a.L, np.uint32)
    codes = reads.reshape(-1)
    for rep in range(3):
        o = _lib.GapOpt.from_dict(opt)
        t0 = time.time()
        n_aln, flags, hoff, hits, st = gi.cal_sa_reg_gap(lens, codes, o)
        dt = time.time() - t0
        print(f"rep {rep}: wall {dt*1e3:.1f} ms kernel {st['kernel_ms']:.1f} ms main {st['main_kernel_ms']:.1f} ms "
              f"reads/s(kernel) {a.n / (st['kernel_ms'] / 1e3):.0f} hits {hits.shape[0]} "
              f"fallback {int((flags & 1).sum())} Q/read {st['rank_queries'] / a.n:.1f} "
              f"blocks/query {st['blocks_loaded'] / max(st['rank_queries'], 1):.3f} pops/read {st['pops'] / a.n:.1f} "
              f"reruns {st['overflow_reruns']}", flush=True)


if __name__ == "__main__":
    main()
