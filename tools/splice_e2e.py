"""End-to-end timing of the spliced-read workload (BASELINE config 4 shape) through the
reference's own `HSA aln` program: the reference as built from its sources
(oracle/_ref/HSA, CPU, single-threaded: its pthread path is commented out,
bwtaln.c:481-504) against the same program with the drop-in entry points linked in
(oracle/ref.mk HSA_gpu_mg: bwa_cal_sa_reg_gap + bwt_match_gap; HSA_gpu_all: + the SAM
stage's bwa_cal_pac_pos).  Same synthetic genome, same index files (written by
hsa_amd.index_build on the device, byte-identical to `HSA index`), same FASTQ; the
SAM outputs must be byte-identical.  Reports wall seconds per program and the
per-batch clock() lines the program prints (bwtaln.c:511, :521: CPU seconds of the
search+splice stage and of the SAM stage).

    python tools/splice_e2e.py --genome 50000005 --reads 20000 [--bins HSA HSA_gpu_mg]
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


def run(binary, args, prefix, fq, out, env=None, timeout=1800, err_path=None):
    t0 = time.perf_counter()
    with open(out, "wb") as f:
        r = subprocess.run([binary, "aln", *args, prefix, fq], stdout=f, stderr=subprocess.PIPE, timeout=timeout,
                           env=env)
    wall = time.perf_counter() - t0
    err = r.stderr.decode(errors="replace")
    if err_path:
        with open(err_path, "w") as f:
            f.write(err)
    if r.returncode:
        raise SystemExit(f"{binary} failed ({r.returncode}):\n{err[-2000:]}")
    secs = [float(x) for x in re.findall(r"^([0-9.]+) sec$", err, re.M)]
    with open(out, "rb") as f:
        digest = hashlib.sha256(f.read()).hexdigest()
    with open(out, "rb") as f:
        lines = sum(1 for _ in f)
    if lines == 0:
        raise SystemExit(f"{binary} printed no SAM lines:\n{err[-2000:]}")
    return {"wall_s": round(wall, 3), "sam_lines": lines, "search_cpu_s": round(sum(secs[0::2]), 3),
            "sam_cpu_s": round(sum(secs[1::2]), 3), "sha256": digest,
            "log": [l for l in err.splitlines() if l.startswith("[hsa]") and "launch:" not in l][-6:]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome", type=int, default=50_000_005,
                    help="genome length; not a multiple of 16 (the reference loses the last 16 characters of the reversed text then, SURVEY Q9)")
    ap.add_argument("--records", type=int, default=4)
    ap.add_argument("--reads", type=int, default=5000)
    ap.add_argument("--len", type=int, default=150)
    ap.add_argument("--args", default="-n 4 -o 1")
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--bins", nargs="+", default=["HSA", "HSA_gpu_mg", "HSA_gpu_all"])
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--out", default=None, help="JSON result file")
    ap.add_argument("--stderr-dir", default=None, help="keep each program's stderr here")
    a = ap.parse_args()

    from hsa_amd import index_build, synth
    wd = a.workdir or tempfile.mkdtemp(prefix="splice_e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
    os.makedirs(wd, exist_ok=True)
    fa = os.path.join(wd, "genome.fa")
    fq = os.path.join(wd, "reads.fq")
    t0 = time.perf_counter()
    codes = synth.genome_codes(a.genome, a.seed)
    recs = synth.record_layout(a.genome, a.records)
    synth.write_fasta(fa, codes, recs)
    reads, _ = synth.make_spliced_reads(codes, recs, a.reads, a.len, a.seed + 1)
    synth.write_fastq(fq, reads)
    del codes
    t1 = time.perf_counter()
    info = index_build.build_index(fa)
    t2 = time.perf_counter()
    print(f"[e2e] genome {a.genome} bp, {a.reads} x {a.len} bp spliced reads: inputs {t1 - t0:.1f} s, "
          f"index on the device {t2 - t1:.1f} s", flush=True)

    res = {"genome_bp": a.genome, "records": a.records, "reads": a.reads, "read_len": a.len, "args": a.args,
           "index": info, "index_build_s": round(t2 - t1, 2), "runs": {}}
    env = dict(os.environ, HSA_VERBOSE="1")
    for b in a.bins:
        path = os.path.join(ROOT, "oracle", "_ref", b)
        r = run(path, a.args.split(), fa, fq, os.path.join(wd, f"{b}.sam"), env=env,
                err_path=os.path.join(a.stderr_dir, f"{b}.err") if a.stderr_dir else None)
        r["reads_per_s"] = round(a.reads / r["wall_s"], 1)
        res["runs"][b] = r
        print(f"[e2e] {b}: wall {r['wall_s']} s ({r['reads_per_s']} reads/s), search+splice {r['search_cpu_s']} "
              f"CPU-s, SAM {r['sam_cpu_s']} CPU-s, sam {r['sha256'][:16]} {' | '.join(r['log'])}", flush=True)
    shas = {r["sha256"] for r in res["runs"].values()}
    res["sam_identical"] = len(shas) == 1
    print(f"[e2e] SAM byte-identical across {len(res['runs'])} programs: {res['sam_identical']}", flush=True)
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    if not res["sam_identical"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
