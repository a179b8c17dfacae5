"""The whole drop-in host C inside the reference's own `HSA aln`, on CPU, under
AddressSanitizer + UndefinedBehaviorSanitizer.

The program is the reference's objects (built here from /root/reference by
oracle/ref.mk, with bwa_cal_sa_reg_gap and bwt_match_gap weakened as in HSA_gpu_mg --
and, variant "all", bwt_extend_backward / bwt_extend_foreward too, as in HSA_gpu_all)
plus OUR bwtaln_gpu.c, bwtgap_gpu.c (and bwtext_gpu.c), and the core's device calls
answered by the C restatement (tests/san/san_core.c + oracle/hsa_oracle.c: test
infrastructure, never the product).  So the reference's splice path (bwt_splice_match,
bwtgap.c:748) calls our bwt_match_gap for every seed and 12-mer anchor search, answered
from the table the drop-in prefetches in batches (hsa_splice_prefetch), and in variant
"all" runs for all fallback reads of a batch as coroutines whose seed extensions are
answered in batches -- and the SAM it prints must be byte-identical to the unmodified
reference's (the recorded tests/golden SAM digests).  With HSA_VERBOSE the drop-in
reports how many of those calls the table answered: the seed and anchor prefetch must
answer every one (none runs alone).

Skips where the reference objects were not built (the GPU box: oracle/_ref/obj is not
sent there)."""
import gzip
import json
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
OBJ = os.path.join(ROOT, "oracle", "_ref", "obj")
MAN = json.load(open(os.path.join(GOLD, "manifest_dropin.json")))
COMMON = ["BWT", "BWTConstruct", "utils", "dictionary", "DNACount", "HSP", "iniparser", "inistrlib", "MemManager",
          "MiscUtilities", "QSufSort", "2BWT-Builder", "TextConverter", "Timing", "bamlite", "2BWT-Interface",
          "bwaseqio", "r250", "cs2nt", "bwtse", "kstring", "stdaln", "bwt_array", "main"]
# "mg": bwt_match_gap replaced (seeds and anchors from the prefetch table); "all": the
# seed extensions too (bwtext_gpu.c: the splice path of the batch's fallback reads as
# coroutines, their extensions batched)
VARIANTS = {"mg": (COMMON + ["bwtaln_weak", "bwtgap_weak"], ["hsa_amd/csrc/bwtaln_gpu.c",
                                                                "hsa_amd/csrc/bwtgap_gpu.c"]),
            "all": (COMMON + ["bwtaln_weak_all", "bwtgap_weak_all"], ["hsa_amd/csrc/bwtaln_gpu.c", "hsa_amd/csrc/bwtgap_gpu.c",
                                                   "hsa_amd/csrc/bwtext_gpu.c"])}
CORE = ["tests/san/san_core.c", "oracle/hsa_oracle.c"]
FLAGS = ["-O1", "-g", "-std=gnu11", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
         "-fno-omit-frame-pointer"]

needs_ref = pytest.mark.skipif(not all(os.path.exists(os.path.join(OBJ, o + ".o"))
                                   for o in COMMON + ["bwtaln_weak", "bwtgap_weak", "bwtaln_weak_all", "bwtgap_weak_all"])
                               or not shutil.which("gcc"),
                               reason="reference objects not built here (make -C oracle)")
_BINS = {}


def hsa_san(tmp_path_factory, variant):
    if variant in _BINS:
        return _BINS[variant]
    d = tmp_path_factory.mktemp("hsa_san_" + variant)
    refobjs, ours = VARIANTS[variant]
    objs = []
    for src in ours + CORE:
        o = str(d / (os.path.basename(src) + ".o"))
        r = subprocess.run(["gcc", "-c", *FLAGS, os.path.join(ROOT, src), "-o", o], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
        objs.append(o)
    out = str(d / ("HSA_san_" + variant))
    r = subprocess.run(["gcc", *FLAGS, *[os.path.join(OBJ, o + ".o") for o in refobjs], *objs,
                        "-lm", "-lz", "-lpthread", "-o", out], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    _BINS[variant] = out
    return out


@needs_ref
@pytest.mark.parametrize("variant", ["mg", "all"])
@pytest.mark.parametrize("name,reads", [("splice_default", "splice_reads"), ("splice_n4o1", "splice_reads"),
                                        ("n4o0", "reads")])
def test_reference_hsa_with_dropin_host_c_prints_reference_sam(tmp_path_factory, variant, name, reads):
    hsa_bin = hsa_san(tmp_path_factory, variant)
    idx = os.path.join(GOLD, "index", "tiny.fa")
    fq = os.path.join(GOLD, MAN[reads])
    env = dict(os.environ, HSA_VERBOSE="1", ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([hsa_bin, "aln", *MAN[name]["args"], idx, fq], capture_output=True, timeout=600, env=env)
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0, err[-4000:]
    assert "runtime error" not in err, err[-4000:]
    ref = gzip.open(os.path.join(GOLD, f"dropin_ref_{name}.sam.gz")).read()
    if r.stdout != ref:
        got, exp = r.stdout.splitlines(), ref.splitlines()
        diff = [(i, a, b) for i, (a, b) in enumerate(zip(exp, got)) if a != b][:3]
        pytest.fail(f"SAM differs: {len(got)} vs {len(exp)} lines; first differences {diff}")
    stats = [(int(a), int(b)) for a, b in
             re.findall(r"splice prefetch: (\d+) bwt_match_gap calls answered from the batch, (\d+) run alone", err)]
    if name.startswith("splice"):
        assert stats, err[-2000:]
        answered = sum(a for a, _ in stats)
        alone = sum(b for _, b in stats)
        assert answered > 0
        assert alone == 0, f"{alone} splice-path calls missed the prefetch table ({answered} answered)"
        if variant == "all":   # the extensions ran batched, from the coroutine runner
            m = re.findall(r"splice path: (\d+) reads as coroutines, seed extensions in (\d+) GPU launches", err)
            assert m and sum(int(a) for a, _ in m) > 0, err[-2000:]
            # ... and every width the splice path computed came from the batched table
            w = [(int(a), int(b)) for a, b in
                 re.findall(r"(\d+) bwt_cal_width calls from the batch, (\d+) alone", err)]
            assert w and sum(a for a, _ in w) > 0 and sum(b for _, b in w) == 0, w


@needs_ref
@pytest.mark.parametrize("name", ["splice_default", "splice_n4o1"])
def test_splice_guard_follows_the_host(tmp_path_factory, name):
    """A device whose splice answers disagree with the host's bwt_splice_match (the
    sanitized core's SAN_SPLICE_FAKE=1: every fallback read answered with no hit): on the
    first batch the drop-in runs the host's function for its first 64 device-answered
    reads too, sees the difference, and from then on takes the host's function for every
    fallback read, this batch's included -- so the SAM is the reference's, and the log
    says so once."""
    hsa_bin = hsa_san(tmp_path_factory, "all")
    idx = os.path.join(GOLD, "index", "tiny.fa")
    fq = os.path.join(GOLD, MAN["splice_reads"])
    env = dict(os.environ, HSA_VERBOSE="1", SAN_SPLICE_FAKE="1",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=23", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([hsa_bin, "aln", *MAN[name]["args"], idx, fq], capture_output=True, timeout=600, env=env)
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0, err[-4000:]
    assert "runtime error" not in err, err[-4000:]
    assert err.count("answers read") == 1 and "differently from the splice kernel" in err, err[-3000:]
    ref = gzip.open(os.path.join(GOLD, f"dropin_ref_{name}.sam.gz")).read()
    assert r.stdout == ref
