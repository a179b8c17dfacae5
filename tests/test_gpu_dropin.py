"""Drop-in test: the reference's own `HSA aln` binary with OUR
bwa_cal_sa_reg_gap linked in place of its definition (oracle/ref.mk target HSA_gpu:
reference objects, bwtaln.o with the symbol weakened, hsa_amd/csrc/bwtaln_gpu.o,
libhsa_gpu.so) must print byte-identical SAM to the unmodified reference binary on
the same FASTQ.  The reference's SAM was recorded in this container by
tools/make_golden.py --dropin (tests/golden/dropin_ref_*.sam.gz).

This covers the whole boundary at once: FASTQ batches through bwa_aln_core, the
option-block side effects (Q2/Q3), strand order and start/end (Q4), the filters
(Q13), the calloc'd hit arrays SAM generation consumes, and the host splice
fallback (bwt_splice_match) fed with the option state our side reports.

HSA_gpu lives under oracle/_ref (built here from /root/reference, git-ignored, travels
to the GPU box with the tree); the test skips when it has not been built.
"""
import gzip
import hashlib
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
HSA_GPU = os.path.join(ROOT, "oracle", "_ref", "HSA_gpu")
MAN = json.load(open(os.path.join(GOLD, "manifest_dropin.json")))

needs_bin = pytest.mark.skipif(not os.path.exists(HSA_GPU), reason="oracle/_ref/HSA_gpu not built (make -C oracle)")


def run_hsa_gpu(args, reads="reads", slots=1):
    idx = os.path.join(GOLD, "index", "tiny.fa")
    fq = os.path.join(GOLD, MAN[reads])
    env = dict(os.environ, HSA_GPU_DEVICES=str(slots))
    return subprocess.run([HSA_GPU, "aln", *args, idx, fq], capture_output=True, timeout=120, env=env)


@needs_bin
@pytest.mark.gpu
@pytest.mark.parametrize("name,reads,slots", [("default", "reads", 1), ("n4o0", "reads", 1),
                                              ("splice_default", "splice_reads", 1), ("splice_n4o1", "splice_reads", 1),
                                              ("default", "reads", 2), ("splice_n4o1", "splice_reads", 3)])
def test_dropin_sam_identical(name, reads, slots):
    """The reference HSA aln with our bwa_cal_sa_reg_gap / bwt_match_gap linked in prints
    the reference's SAM byte for byte -- also with each call split over 2 or 3 device
    slots (hsa_gpu_set_devices via HSA_GPU_DEVICES; slots share the one GPU here)."""
    r = run_hsa_gpu(MAN[name]["args"], reads, slots)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    sam = r.stdout
    if hashlib.sha256(sam).hexdigest() != MAN[name]["sam_sha256"]:
        ref = gzip.open(os.path.join(GOLD, f"dropin_ref_{name}.sam.gz")).read().splitlines()
        got = sam.splitlines()
        diff = [(i, a, b) for i, (a, b) in enumerate(zip(ref, got)) if a != b][:5]
        pytest.fail(f"SAM differs: {len(got)} vs {len(ref)} lines; first differences {diff}")


@needs_bin
def test_dropin_fails_loudly_without_gpu():
    """No CPU fallback: without a visible GPU the drop-in exits 1 with a message
    (the reference's error convention), it never silently computes on the host."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    idx = os.path.join(GOLD, "index", "tiny.fa")
    fq = os.path.join(GOLD, MAN["reads"])
    r = subprocess.run([HSA_GPU, "aln", idx, fq], capture_output=True, timeout=120, env=env)
    assert r.returncode == 1
    assert b"[bwa_cal_sa_reg_gap]" in r.stderr
    assert r.stdout == b""


HSA_GPU_ALL = os.path.join(ROOT, "oracle", "_ref", "HSA_gpu_all")


@pytest.mark.skipif(not os.path.exists(HSA_GPU_ALL), reason="oracle/_ref/HSA_gpu_all not built (make -C oracle)")
@pytest.mark.gpu
@pytest.mark.parametrize("name,reads,env", [("default", "reads", {}), ("n4o0", "reads", {}),
                                            ("splice_default", "splice_reads", {}), ("splice_n4o1", "splice_reads", {}),
                                            ("splice_n4o1O120", "splice_reads", {}),
                                            ("splice_n4o1", "splice_reads",
                                             {"HSA_SPLICE_PREFETCH": "0", "HSA_SPLICE_THREADS": "4",
                                              "HSA_SPLICE_DEVICE": "0"}),
                                            ("splice_default", "splice_reads", {"HSA_SPLICE_DEVICE": "0"}),
                                            ("splice_n4o1", "splice_reads", {"HSA_SPLICE_CAP": "6"}),
                                            ("default", "reads", {"HSA_SAM_THREADS": "8", "HSA_SAM_CHUNK": "7"}),
                                            ("splice_n4o1", "splice_reads", {"HSA_SAM_THREADS": "1"})])
def test_dropin_all_entry_points_sam_identical(name, reads, env):
    """Every drop-in entry point replaced at once (oracle/ref.mk HSA_gpu_all):
    bwa_cal_sa_reg_gap, bwt_match_gap, and the SAM stage's bwa_cal_pac_pos, whose SA ->
    position lookups (seq_id, position and the duplicate filter of the extra hits in
    every SAM line) run as one GPU batch per read batch (hsa_amd/csrc/bwtse_gpu.c).
    By default the splice path runs on the device (hsa_splice.hip).
    splice_n4o1O120 (-O 120): n_stacks 283, more score buckets than the splice kernel and
    an extension slice slot hold, so the host's bwt_splice_match runs with its extensions
    through hsa_extend_batch.
    HSA_SPLICE_DEVICE=0: the host's bwt_splice_match for every fallback read (coroutine
    runner); with HSA_SPLICE_PREFETCH=0 and 4 runner threads there are no splice tables,
    so every seed and anchor search and every width of the splice path is a direct GPU
    call, made from four host threads at once (the calls serialise on slot 0's index).
    HSA_SPLICE_CAP=6: the splice kernel's per-lane stack holds 6 entries, so most reads
    outgrow it and go to the host's path while the rest are answered on the device.
    The SAM stage is ours too (generate_sam_se_core, hsa_amd/csrc/bwtsam_gpu.c: drand48 by
    jump-ahead, refine + print on host threads, spliced reads' positions on the GPU);
    HSA_SAM_THREADS / HSA_SAM_CHUNK vary its threads and chunks."""
    idx = os.path.join(GOLD, "index", "tiny.fa")
    fq = os.path.join(GOLD, MAN[reads])
    r = subprocess.run([HSA_GPU_ALL, "aln", *MAN[name]["args"], idx, fq], capture_output=True, timeout=120,
                       env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    if hashlib.sha256(r.stdout).hexdigest() != MAN[name]["sam_sha256"]:
        ref = gzip.open(os.path.join(GOLD, f"dropin_ref_{name}.sam.gz")).read().splitlines()
        got = r.stdout.splitlines()
        diff = [(i, a, b) for i, (a, b) in enumerate(zip(ref, got)) if a != b][:5]
        pytest.fail(f"SAM differs: {len(got)} vs {len(ref)} lines; first differences {diff}")
