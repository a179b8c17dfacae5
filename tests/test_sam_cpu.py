"""The drop-in SAM stage (hsa_amd/csrc/bwtsam_gpu.c: generate_sam_se_core, bwtse.c:884,
on host threads) inside the reference's own `HSA aln`, on CPU.

oracle/_ref/HSA_sam is the reference program (built here from /root/reference by
oracle/ref.mk) with only generate_sam_se_core replaced: its search and its SA -> position
step are the reference's own, so any byte that differs from the unmodified reference's
SAM comes from the SAM stage -- the drand48 jump-ahead of the hit choice (bwtse.c:44,
:51, :97), the chunked bwa_refine_gapped calls, the restated bwa_print_sam1, or the
order the chunks are written in.

* the recorded golden SAM of the drop-in fixtures (tests/golden, the reference's `HSA aln`
  output), with 1 and 8 threads and chunks of 1, 7 and 2048 reads;
* reads generated here, run through both programs: 230 000 36 bp reads of the 50 kbp
  repeat genome (three 100 000-read batches: most reads have several equal-best hits, so
  the drand48 sequence has to continue across reads, chunks and batches), and
  gapped 100 bp reads of the tiny genome with -n 4 -o 1 (the CIGAR DP of
  bwa_refine_gapped and MD tags), each with random quality strings (reverse-strand
  reads print theirs reversed);
* the printing guard: with a host bwa_print_sam1 that prints other bytes (a shim linked
  in place of the reference's), the stage prints every line with the host's function.

Skips where the reference binaries were not built (the GPU box)."""
import gzip
import hashlib
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF = os.path.join(ROOT, "oracle", "_ref")
OBJ = os.path.join(REF, "obj")
HSA, HSA_SAM = os.path.join(REF, "HSA"), os.path.join(REF, "HSA_sam")
MAN = json.load(open(os.path.join(GOLD, "manifest_dropin.json")))

needs_bins = pytest.mark.skipif(not (os.path.exists(HSA) and os.path.exists(HSA_SAM)),
                                reason="oracle/_ref/HSA(_sam) not built (make -C oracle)")


def run(binary, args, prefix, fq, env=None):
    e = dict(os.environ, **(env or {}))
    r = subprocess.run([binary, "aln", *args, prefix, fq], capture_output=True, timeout=600, env=e)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    return r.stdout, r.stderr.decode()


def first_diff(a, b):
    la, lb = a.splitlines(), b.splitlines()
    for i, (x, y) in enumerate(zip(la, lb)):
        if x != y:
            return i, x[:200], y[:200]
    return len(la), len(lb)


@needs_bins
@pytest.mark.parametrize("threads,chunk", [(1, 2048), (8, 1), (8, 7), (3, 2048)])
@pytest.mark.parametrize("name,reads", [("default", "reads"), ("n4o0", "reads"), ("splice_default", "splice_reads"),
                                        ("splice_n4o1", "splice_reads")])
def test_golden_sam(name, reads, threads, chunk):
    out, _ = run(HSA_SAM, MAN[name]["args"], os.path.join(GOLD, "index", "tiny.fa"), os.path.join(GOLD, MAN[reads]),
                 {"HSA_SAM_THREADS": str(threads), "HSA_SAM_CHUNK": str(chunk)})
    if hashlib.sha256(out).hexdigest() != MAN[name]["sam_sha256"]:
        ref = gzip.open(os.path.join(GOLD, f"dropin_ref_{name}.sam.gz")).read()
        pytest.fail(f"SAM differs from the reference's: {first_diff(ref, out)}")


def write_fastq_q(path, reads, seed):
    """FASTQ with a random quality string per read (Phred+33 in '#'..'J')."""
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    q = rng.integers(35, 75, size=reads.shape, dtype=np.uint8)
    with open(path, "wb") as f:
        for i in range(len(reads)):
            f.write(b"@q%d\n%s\n+\n%s\n" % (i, acgt[reads[i]].tobytes(), q[i].tobytes()))


@pytest.fixture(scope="module")
def generated(tmp_path_factory):
    from hsa_amd import index_io, synth
    d = tmp_path_factory.mktemp("sam_cpu")
    out = {}
    rep = index_io.read_pac(os.path.join(GOLD, "index", "rep.fa"))
    r, _ = synth.make_reads(rep, [(0, len(rep))], 230_000, 36, 611, max_mm=2)
    out["rep"] = str(d / "rep.fq")
    write_fastq_q(out["rep"], r, 1)
    tiny = index_io.read_pac(os.path.join(GOLD, "index", "tiny.fa"))
    recs = [(0, 66667), (66667, 66667), (133334, 66669)]
    r, _ = synth.make_reads(tiny, recs, 6_000, 100, 612, indel=True, max_mm_indel=2)
    out["gap"] = str(d / "gap.fq")
    write_fastq_q(out["gap"], r, 2)
    return out


@needs_bins
@pytest.mark.parametrize("case,index,args,threads,chunk", [
    ("rep", "rep.fa", [], 8, 2048),
    ("rep", "rep.fa", [], 5, 333),
    ("gap", "tiny.fa", ["-n", "4", "-o", "1"], 8, 64),
])
def test_generated_sam_matches_reference(generated, case, index, args, threads, chunk):
    prefix = os.path.join(GOLD, "index", index)
    ref, _ = run(HSA, args, prefix, generated[case])
    got, err = run(HSA_SAM, args, prefix, generated[case],
                   {"HSA_SAM_THREADS": str(threads), "HSA_SAM_CHUNK": str(chunk), "HSA_VERBOSE": "1"})
    assert ref.count(b"\n") > 1000
    assert got == ref, f"SAM differs from the reference's: {first_diff(ref, got)}"
    if case == "rep":       # several equal-best hits per read: the random choice and XA lists are exercised
        assert ref.count(b"XT:A:R") > 10_000 and ref.count(b"XA:Z:") > 1_000
        assert err.count("[hsa] SAM stage of") == 3            # three batches of <= 100 000 reads
    else:
        assert b"I\t" in ref or b"D\t" in ref or any(c in ref for c in (b"1I", b"2D", b"3I"))


SHIM = r'''
#include <stdio.h>
typedef struct { char *name; } seq_head_t;
/* a host whose bwa_print_sam1 is not bwtse.c:677's: prints one marker line per read */
void bwa_print_sam1(const void *hsp, seq_head_t *p, const void *mate, int mode, int max_top2)
{
    printf("SHIM\t%s\n", p->name);
}
'''


@needs_bins
@pytest.mark.skipif(not shutil.which("gcc"), reason="gcc")
def test_print_guard_follows_a_different_host_function(tmp_path):
    """A host bwa_print_sam1 that prints other bytes: the guard sees the difference on the
    first batch and every SAM line comes from the host's function (in read order)."""
    objs = [os.path.join(OBJ, f) for f in os.listdir(OBJ)
            if f.endswith(".o") and f in {o + ".o" for o in (
                "BWT", "BWTConstruct", "utils", "dictionary", "DNACount", "HSP", "iniparser", "inistrlib", "MemManager",
                "MiscUtilities", "QSufSort", "2BWT-Builder", "TextConverter", "Timing", "bamlite", "2BWT-Interface",
                "bwaseqio", "r250", "cs2nt", "kstring", "stdaln", "bwt_array", "main", "bwtaln", "bwtgap",
                "bwtse_weak_sam_print")}]
    if len(objs) != 26:
        pytest.skip("reference objects not built")
    shim = tmp_path / "shim.c"
    shim.write_text(SHIM)
    sam_o = tmp_path / "bwtsam.o"
    subprocess.run(["gcc", "-O2", "-c", "-std=gnu11", os.path.join(ROOT, "hsa_amd", "csrc", "bwtsam_gpu.c"), "-o",
                    str(sam_o)], check=True)
    exe = tmp_path / "HSA_shim"
    subprocess.run(["gcc", *objs, str(sam_o), str(shim), "-lm", "-lz", "-lpthread", "-o", str(exe)], check=True)
    out, err = run(str(exe), [], os.path.join(GOLD, "index", "tiny.fa"), os.path.join(GOLD, MAN["reads"]),
                   {"HSA_SAM_THREADS": "4", "HSA_SAM_CHUNK": "100"})
    ref = gzip.open(os.path.join(GOLD, "dropin_ref_default.sam.gz")).read()
    want = b"".join(b"SHIM\t" + ln.split(b"\t")[0] + b"\n" for ln in ref.splitlines())
    assert out == want
    assert "prints other bytes" in err
