"""Where the drop-in's time goes: hsa_cal_sa_reg_gap_flat on host arrays (what a host
`HSA aln` calls through bwa_cal_sa_reg_gap) over 1 M config-2 reads on the hg19-sized
index, with the library's HSA_VERBOSE stage timings and the Python-side wall time.

    HSA_VERBOSE=1 python tools/dropin_time.py [--reads 1000000] [--config 2|3]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import hsa_amd  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--config", type=int, default=2, choices=(2, 3))
    a = ap.parse_args()
    import torch

    import bench
    from hsa_amd import synth
    from hsa_amd._lib import GapOpt
    gi, res, _ = bench.build_index(bench.GENOME_T, bench.GENOME_SEED, torch.cuda.current_device())
    del res
    genome = synth.PackedGenome(bench.GENOME_T, bench.GENOME_SEED)
    recs = synth.record_layout(bench.GENOME_T, bench.RECORDS)
    if a.config == 2:
        reads, _ = synth.make_reads(genome, recs, a.reads, 100, 5 * 1_000_000, max_mm=4)
    else:
        reads, _ = synth.make_reads(genome, recs, a.reads, 100, 6 * 1_000_000, indel=True, max_mm_indel=2)
    opt = GapOpt.default()
    opt.max_diff, opt.fnr, opt.max_gapo = 4, -1.0, 0 if a.config == 2 else 1
    opt.mode &= ~0x01
    lens = np.full(a.reads, 100, np.uint32)
    codes = np.ascontiguousarray(reads.reshape(-1))
    for it in range(4):
        t0 = time.perf_counter()
        n_aln, flags, hoff, hits, st = gi.cal_sa_reg_gap(lens, codes, opt)
        dt = time.perf_counter() - t0
        print(f"[dropin_time] call {it}: {a.reads} reads in {dt * 1e3:.1f} ms ({a.reads / dt:.0f} reads/s), "
              f"kernels {st['kernel_ms']:.1f} ms, {len(hits)} hits", flush=True)


if __name__ == "__main__":
    main()
