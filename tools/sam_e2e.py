"""`HSA aln` end to end, FASTQ -> SAM, at hg19 size: the reference's own program
(oracle/_ref/HSA, built here from its sources: single-threaded C) against the same
program with every drop-in entry point of ours linked in (oracle/_ref/HSA_gpu_all: the
search, the splice path, and the SAM stage -- generate_sam_se_core on host threads,
hsa_amd/csrc/bwtsam_gpu.c, with its SA -> position lookups on the GPU).

* Index: the hg19-sized synthetic genome of bench.py (3 000 000 005 bp, 24 records),
  its BWTs built on the device, written as the reference's index files (bench.py
  reference_files: .bwt/.fmv/.rev.* /.sa/.pac/.ann).
* Config 2: 1 M x 100 bp reads with 0-4 substitutions (bench.py's first batch), random
  quality strings, `-n 4 -o 0`, one process each.
* Config 4: 200 000 x 150 bp spliced reads, default options.  The reference needs about
  4 ms per read here (12+ minutes in one process), so both programs run on the same 8
  FASTQ pieces of 25 000 reads -- the reference's 8 processes side by side, ours one
  after another -- and the SAM of every piece is compared; ours also runs the whole
  200 000 reads in one process (the speed a user sees).
* Each GPU run is repeated with HSA_SAM_THREADS=1 (same binary, same box): the SAM
  stage's own thread speed-up.

Reported per run: wall seconds (the program, index load included), the program's own
per-batch stage lines (bwtaln.c:511, :521: CPU seconds from clock(); ours adds
"[hsa] SAM stage" wall lines), the SAM's SHA-256.  Writes one JSON file.

    python tools/sam_e2e.py --out gpurun_out/r06_sam_e2e.json
"""
import argparse
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = os.path.join(ROOT, "oracle", "_ref")


def say(*a):
    print(*a, flush=True)


def prepare(d):
    """(child process: the only one that touches the GPU) the index files under d/g.index.*"""
    import hsa_amd  # noqa: F401  (libhsa_gpu.so before torch)
    import bench
    import torch
    t0 = time.time()
    gi, res, extra = bench.build_index(bench.GENOME_T, bench.GENOME_SEED, 0, with_files=True)
    gi.close()
    prefix = bench.reference_files(d, bench.GENOME_T, res, extra)
    del res, extra
    torch.cuda.empty_cache()
    say(f"[sam_e2e] index files at {prefix} in {time.time() - t0:.1f} s")


def run(binary, args, prefix, fq, sam, env=None, tag=""):
    """One `HSA aln` process; prints a heartbeat every 30 s while it runs."""
    e = dict(os.environ, HSA_VERBOSE="1", **(env or {}))
    t0 = time.perf_counter()
    with open(sam, "wb") as fo, open(sam + ".err", "wb") as fe:
        p = subprocess.Popen([binary, "aln", *args, prefix, fq], stdout=fo, stderr=fe, env=e)
        while True:
            try:
                p.wait(timeout=30)
                break
            except subprocess.TimeoutExpired:
                say(f"[sam_e2e]   {tag} running, {time.perf_counter() - t0:.0f} s")
    wall = time.perf_counter() - t0
    err = open(sam + ".err", errors="replace").read()
    if p.returncode:
        raise SystemExit(f"{binary} exit {p.returncode}:\n{err[-3000:]}")
    return summarise(wall, err, sam)


def summarise(wall, err, sam):
    secs = [float(x) for x in re.findall(r"^([0-9.]+) sec$", err, re.M)]
    sam_wall = [float(x) for x in re.findall(r"\[hsa\] SAM stage of \d+ reads on \d+ threads: .* total ([0-9.]+) ms",
                                              err)]
    thr = re.findall(r"\[hsa\] SAM stage of \d+ reads on (\d+) threads", err)
    search = [float(x) for x in re.findall(r"\[hsa\] batch of \d+ reads: search ([0-9.]+) s", err)]
    real = re.findall(r"Real time: ([0-9.]+) sec; CPU: ([0-9.]+) sec", err)
    h = hashlib.sha256()
    lines = 0
    with open(sam, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
            lines += blk.count(b"\n")
    r = {"wall_s": round(wall, 3), "sam_lines": lines, "sha256": h.hexdigest(),
         "batches": len(secs) // 2,
         "search_clock_s": round(sum(secs[0::2]), 3),           # bwtaln.c:511 (process CPU seconds)
         "sam_clock_s": round(sum(secs[1::2]), 3)}              # bwtaln.c:521 (process CPU seconds)
    if real:
        r["main_real_s"], r["main_cpu_s"] = float(real[-1][0]), float(real[-1][1])
    if sam_wall:
        r["sam_stage_wall_s"] = round(sum(sam_wall) / 1e3, 3)
        r["sam_threads"] = int(thr[0])
    if search:
        r["search_wall_s"] = round(sum(search), 3)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--c2-reads", type=int, default=1_000_000)
    ap.add_argument("--c4-reads", type=int, default=200_000)
    ap.add_argument("--c4-pieces", type=int, default=8)
    ap.add_argument("--prepare", default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.prepare:
        prepare(a.prepare)
        return
    import numpy as np

    import bench
    from hsa_amd import synth
    d = a.workdir or tempfile.mkdtemp(prefix="sam_e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
    os.makedirs(d, exist_ok=True)
    t0 = time.time()
    subprocess.run([sys.executable, os.path.abspath(__file__), "--out", a.out, "--prepare", d], check=True)
    prefix = os.path.join(d, "g")
    T = bench.GENOME_T
    genome = synth.PackedGenome(T, bench.GENOME_SEED)
    recs = synth.record_layout(T, bench.RECORDS)
    fq2 = os.path.join(d, "c2.fq")
    r2, _ = synth.make_reads(genome, recs, a.c2_reads, 100, 5 * 1_000_000, max_mm=4)
    synth.write_fastq(fq2, r2, qual_seed=2)
    del r2
    r4, _ = synth.make_spliced_reads(genome, recs, a.c4_reads, 150, 7 * 1_000_000)
    fq4 = os.path.join(d, "c4.fq")
    synth.write_fastq(fq4, r4, qual_seed=4)
    per = a.c4_reads // a.c4_pieces
    pieces = []
    for k in range(a.c4_pieces):
        pk = os.path.join(d, f"c4_{k}.fq")
        synth.write_fastq(pk, r4[k * per:(k + 1) * per], prefix=f"p{k}_", qual_seed=40 + k)
        pieces.append(pk)
    del r4, genome
    say(f"[sam_e2e] inputs ready in {time.time() - t0:.1f} s: {a.c2_reads} config-2 reads, {a.c4_reads} config-4 reads")

    hsa, gpu = os.path.join(REF, "HSA"), os.path.join(REF, "HSA_gpu_all")
    res = {"genome_bp": T, "workdir_note": "index files written from the device-built BWTs (bench.reference_files)",
           "cpu": bench.cpu_info(), "config2": {}, "config4": {}}

    def save():
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)

    # ---- config 2: one process each
    c2 = res["config2"]
    c2["reads"], c2["args"] = a.c2_reads, "-n 4 -o 0"
    c2["gpu_all"] = run(gpu, ["-n", "4", "-o", "0"], prefix, fq2, os.path.join(d, "c2_gpu.sam"), tag="c2 HSA_gpu_all")
    say(f"[sam_e2e] config 2 HSA_gpu_all: {c2['gpu_all']}")
    c2["gpu_all_sam1"] = run(gpu, ["-n", "4", "-o", "0"], prefix, fq2, os.path.join(d, "c2_gpu1.sam"),
                             {"HSA_SAM_THREADS": "1"}, tag="c2 HSA_gpu_all 1 SAM thread")
    say(f"[sam_e2e] config 2 HSA_gpu_all, 1 SAM thread: {c2['gpu_all_sam1']}")
    save()
    c2["reference"] = run(hsa, ["-n", "4", "-o", "0"], prefix, fq2, os.path.join(d, "c2_ref.sam"), tag="c2 HSA")
    say(f"[sam_e2e] config 2 reference HSA: {c2['reference']}")
    c2["sam_identical"] = c2["reference"]["sha256"] == c2["gpu_all"]["sha256"] == c2["gpu_all_sam1"]["sha256"]
    ref, ours, one = c2["reference"], c2["gpu_all"], c2["gpu_all_sam1"]
    c2["speedup_whole_program"] = round(ref["wall_s"] / ours["wall_s"], 2)
    c2["sam_stage_speedup_vs_reference"] = round(ref["sam_clock_s"] / ours["sam_stage_wall_s"], 2)
    c2["sam_stage_speedup_vs_1_thread"] = round(one["sam_stage_wall_s"] / ours["sam_stage_wall_s"], 2)
    save()
    for f in ("c2_gpu.sam", "c2_gpu1.sam", "c2_ref.sam"):
        os.remove(os.path.join(d, f))

    # ---- config 4: the pieces (reference side by side, ours in turn), then ours on all
    c4 = res["config4"]
    c4["reads"], c4["pieces"], c4["args"] = a.c4_reads, a.c4_pieces, "(defaults: -n 0.04 -o 1)"
    t1 = time.perf_counter()
    procs = []
    for k, pk in enumerate(pieces):
        sam = os.path.join(d, f"c4_ref_{k}.sam")
        fo, fe = open(sam, "wb"), open(sam + ".err", "wb")
        procs.append((subprocess.Popen([hsa, "aln", prefix, pk], stdout=fo, stderr=fe), sam, fo, fe, time.perf_counter()))
    walls = [None] * len(procs)
    while any(w is None for w in walls):
        for k, (p, sam, fo, fe, ts) in enumerate(procs):
            if walls[k] is None and p.poll() is not None:
                walls[k] = time.perf_counter() - ts
                fo.close(); fe.close()
                if p.returncode:
                    raise SystemExit(f"reference piece {k} exit {p.returncode}")
        if any(w is None for w in walls):
            time.sleep(2)
            if int(time.perf_counter() - t1) % 30 < 2:
                say(f"[sam_e2e]   config-4 reference pieces: {sum(w is not None for w in walls)} of {len(walls)} done, "
                    f"{time.perf_counter() - t1:.0f} s")
    refp = [summarise(walls[k], open(procs[k][1] + ".err", errors="replace").read(), procs[k][1])
            for k in range(len(procs))]
    say(f"[sam_e2e] config 4 reference pieces: {time.perf_counter() - t1:.0f} s side by side")
    gp = []
    for k, pk in enumerate(pieces):
        gp.append(run(gpu, [], prefix, pk, os.path.join(d, f"c4_gpu_{k}.sam"), tag=f"c4 piece {k}"))
    same = [refp[k]["sha256"] == gp[k]["sha256"] for k in range(len(pieces))]
    c4["pieces_reference"], c4["pieces_gpu_all"], c4["pieces_sam_identical"] = refp, gp, same
    say(f"[sam_e2e] config 4 pieces: SAM identical {same}")
    save()
    c4["gpu_all_whole"] = run(gpu, [], prefix, fq4, os.path.join(d, "c4_gpu.sam"), tag="c4 whole")
    c4["gpu_all_whole_sam1"] = run(gpu, [], prefix, fq4, os.path.join(d, "c4_gpu1.sam"), {"HSA_SAM_THREADS": "1"},
                                   tag="c4 whole, 1 SAM thread")
    c4["whole_sam_identical_1_vs_n_threads"] = c4["gpu_all_whole"]["sha256"] == c4["gpu_all_whole_sam1"]["sha256"]
    ref_reads_per_s = sum(a.c4_reads // a.c4_pieces / p["wall_s"] for p in refp) / len(refp)
    c4["reference_reads_per_s_per_process"] = round(ref_reads_per_s, 1)
    c4["gpu_all_whole_reads_per_s"] = round(a.c4_reads / c4["gpu_all_whole"]["wall_s"], 1)
    c4["sam_stage_speedup_vs_reference"] = round(sum(p["sam_clock_s"] for p in refp) /
                                                 c4["gpu_all_whole"]["sam_stage_wall_s"], 2)
    c4["sam_stage_speedup_vs_1_thread"] = round(c4["gpu_all_whole_sam1"]["sam_stage_wall_s"] /
                                                c4["gpu_all_whole"]["sam_stage_wall_s"], 2)
    save()
    say(json.dumps({"config2": {k: v for k, v in c2.items() if not isinstance(v, dict)},
                    "config4": {k: v for k, v in c4.items() if not isinstance(v, (dict, list))}}))
    ok = c2["sam_identical"] and all(same) and c4["whole_sam_identical_1_vs_n_threads"]
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
