#!/usr/bin/env python3
"""Experiment: where in the search trie the rank steps fall.  Runs the instrumented
restatement (oracle/liboracle_hist.so, -DOR_DEPTH_HIST) on a sample of the bench's
reads against the device-built hg19-sized index and prints, per string length d, the
search steps and the width steps whose string is d characters long, and the share of
each whose two rank queries fall in different 16-character blocks (two sectors).
Sizes a table of all strings up to length D (its steps become one table load)."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_ctypes  # noqa: E402

oracle_ctypes.LIB = os.path.join(ROOT, "oracle", "liboracle_hist.so")
import bench  # noqa: E402
from hsa_amd import synth  # noqa: E402
from oracle_ctypes import Opt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=bench.GENOME_T)
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--out", default="gpurun_out/depth_hist.json")
    a = ap.parse_args()
    gi, res, _ = bench.build_index(a.T, bench.GENOME_SEED, 0)
    ox = bench.host_oracle_index(res, a.T)
    del gi
    L = oracle_ctypes.lib()
    L.or_depth_hist.argtypes = [np.ctypeslib.ndpointer(np.uint64, flags="C"), C.c_int]
    genome = synth.PackedGenome(a.T, bench.GENOME_SEED)
    recs = synth.record_layout(a.T, bench.RECORDS)
    out = {}
    for name, RL, kw, mg in (("config2", 100, dict(max_mm=4), 0), ("config3", 100, dict(indel=True, max_mm_indel=2), 1),
                             ("config5_on_3g", 250, dict(max_mm=4), 0)):
        n = a.n if name != "config3" else a.n // 4
        reads, _ = synth.make_reads(genome, recs, n, RL, 5 * 1_000_000, **kw)
        from hsa_amd._lib import GapOpt
        opt = GapOpt.default()
        opt.max_diff, opt.fnr, opt.max_gapo = 4, -1.0, mg
        opt.mode &= ~0x01
        h = np.zeros(4 * 64, np.uint64)
        L.or_depth_hist(h, 1)
        o = ox.cal_sa_reg_gap(np.full(n, RL, np.uint32), np.ascontiguousarray(reads).reshape(-1),
                              Opt.from_dict(opt.as_dict()))
        L.or_depth_hist(h, 1)
        h = h.reshape(4, 64).astype(np.float64) / n
        q = int(o[3][0]) / n
        print(f"== {name}: {n} reads, {q:.1f} rank queries per read")
        cs, cw = np.cumsum(h[0]), np.cumsum(h[2])
        cs2, cw2 = np.cumsum(h[1]), np.cumsum(h[3])
        for d in range(1, 24):
            print(f"  d={d:2d}  search steps {h[0][d]:8.2f} (2 blocks {h[1][d]:7.2f})  cum {cs[d]:8.1f}"
                  f"   width steps {h[2][d]:7.2f} (2 blocks {h[3][d]:6.2f})  cum {cw[d]:7.1f}")
        print(f"  total: search steps {cs[-1]:.1f} ({cs2[-1]:.1f} on 2 blocks), width steps {cw[-1]:.1f} "
              f"({cw2[-1]:.1f} on 2 blocks)")
        out[name] = dict(reads=n, queries_per_read=q, hist=h.tolist())
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(out, open(a.out, "w"))


if __name__ == "__main__":
    main()
