"""The tail of a 100 000-read drop-in call (the reference's batch, bwtaln.c:477), measured
with the diagnostic build's per-read maxima (libhsa_gpu_diag.so, tools/build_diag.sh:
-DHSA_DIAG, never the product).

A 100 000-read call has fewer reads than the 262 144 lanes k_search keeps resident, so
every read gets its own lane at once and the kernel lasts as long as its slowest read's
chain of dependent rank steps (both strands).  This prints, for one call on the
hg19-sized index (bench.py's config-2 or config-3 reads): the kernels' time, the largest
number of rank steps and pops one read took, the longest wall time one read held its
lane (s_memrealtime, 100 MHz), and that time per rank step -- the latency of one step of
a dependent chain at this load.

    HSA_GPU_LIB=libhsa_gpu_diag.so python tools/tail_diag.py --config 2 --out gpurun_out/r06_tail_c2.json
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2, choices=(2, 3))
    ap.add_argument("--reads", type=int, default=100_000)
    ap.add_argument("--calls", type=int, default=5)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    assert "diag" in os.environ.get("HSA_GPU_LIB", ""), "run with HSA_GPU_LIB=libhsa_gpu_diag.so"
    import hsa_amd  # noqa: F401  (before torch)
    import numpy as np
    import torch

    import bench
    from hsa_amd import _lib, synth
    from hsa_amd._lib import GapOpt
    L = _lib.lib()
    gi, _, _ = bench.build_index(bench.GENOME_T, bench.GENOME_SEED, torch.cuda.current_device())
    genome = synth.PackedGenome(bench.GENOME_T, bench.GENOME_SEED)
    recs = synth.record_layout(bench.GENOME_T, bench.RECORDS)
    if a.config == 3:
        reads, _ = synth.make_reads(genome, recs, a.reads, 100, 6 * 1_000_000, indel=True, max_mm_indel=2)
    else:
        reads, _ = synth.make_reads(genome, recs, a.reads, 100, 5 * 1_000_000, max_mm=4)
    lens = np.full(a.reads, 100, np.uint32)
    codes = reads.reshape(-1)
    opt0 = GapOpt.default()
    opt0.max_diff, opt0.fnr, opt0.max_gapo = 4, -1.0, 0 if a.config == 2 else 1
    opt0.mode &= ~0x01                                  # a steady-state batch
    out = {"config": a.config, "reads": a.reads, "calls": []}
    buf = (C.c_ulonglong * 32)()
    for c in range(a.calls):
        L.hsa_diag_counters(buf, 1)                     # reset
        o = GapOpt.from_dict(opt0.as_dict())
        t0 = time.perf_counter()
        n_aln, flags, hoff, hits, st = gi.cal_sa_reg_gap(lens, codes, o)
        wall = time.perf_counter() - t0
        L.hsa_diag_counters(buf, 0)
        steps, ticks, pops = int(buf[21]), int(buf[22]), int(buf[23])
        steps_hit, steps_nohit = int(buf[24]), int(buf[25])
        rec = {"call_wall_ms": round(wall * 1e3, 2), "kernels_ms": round(st["kernel_ms"], 3),
               "main_pass_ms": round(st["main_kernel_ms"], 3),
               "slowest_read_steps": steps, "slowest_read_pops": pops,
               "slowest_item_with_hits_steps": steps_hit, "slowest_item_without_hits_steps": steps_nohit, "slowest_read_us": round(ticks / 100.0, 1),
               "ns_per_step_on_the_longest_read": round(ticks * 10.0 / max(steps, 1), 1),
               "rank_steps_mean_per_read": round(st["rank_queries"] / 2 / a.reads, 1),
               "mapped": int((n_aln > 0).sum())}
        out["calls"].append(rec)
        print(json.dumps(rec), flush=True)
    out["note"] = ("maxima over the call's reads: steps / pops / lane time of the read that took the most of each "
                   "(not necessarily one read); ns per step = the longest lane time / the most steps")
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    gi.close()


if __name__ == "__main__":
    main()
