"""The splice path on the device (hsa_splice_match_batch, hsa_amd/csrc/hsa_splice.hip):
bwt_splice_match (bwtgap.c:748-1332) of every read the reference sends to it, against
the compiled reference itself (oracle/_ref/ref_probe: bwa_cal_sa_reg_gap batch by batch,
bit 0 of a read's flags = bwt_splice_match was called, its hits are that call's).

Every read the kernel answers (status 0) must carry the reference's n_aln and every
word of its spliced hits; reads it hands back (status > 0: the reference's code is
undefined there, or the read outgrew the kernel's stack) are counted and must be few --
the drop-in runs the host's own bwt_splice_match for them (tests/test_gpu_dropin.py
covers that mix end to end)."""
import gzip
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

from golden_io import GOLD, INDEX, parse_opts
from hsa_amd import index_io

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "oracle", "_ref", "ref_probe")

NT4 = np.full(256, 4, np.uint8)
for _i, _c in enumerate(b"ACGT"):
    NT4[_c] = NT4[_c + 32] = _i


def fastq_codes(path):
    lines = gzip.open(path, "rt").read().split("\n")
    return [NT4[np.frombuffer(lines[i + 1].encode(), np.uint8)] for i in range(0, len(lines) - 3, 4)]


def write_reads(path, reads):
    with open(path, "wb") as f:
        f.write(np.array([len(reads)], np.uint32).tobytes())
        f.write(np.array([len(r) for r in reads], np.uint32).tobytes())
        for r in reads:
            f.write(np.ascontiguousarray(r, np.uint8).tobytes())


def read_out(path):
    """ref_probe's out.bin -> per read (n_aln, flags, hits (n, 9))."""
    b = np.fromfile(path, np.uint32)
    assert b[0] == 0x48415348
    n, i, out = int(b[1]), 2, []
    for _ in range(n):
        na, fl = int(np.int32(b[i])), int(b[i + 1])
        i += 2
        h = b[i:i + 9 * max(na, 0)].reshape(-1, 9)
        i += 9 * max(na, 0)
        out.append((na, fl, h))
    return out


def regimes(od):
    """aux_seed (bwtgap.c:769-774), aux_ext (:776-782) of local_opt od."""
    from hsa_amd._lib import regime_of
    n_stacks = (od["max_diff"] + 1) * od["s_mm"] + (od["max_gapo"] + 1) * od["s_gapo"] + \
        (od["max_gape"] + 1) * od["s_gape"]
    so = dict(od, max_gapo=0, max_gape=0, max_diff=od["max_seed_diff"], mode=od["mode"] & ~0x01)
    ao = dict(od, max_gape=3)
    srg = regime_of(so, n_stacks, so["max_diff"])
    arg = regime_of(ao, n_stacks, od["max_diff"])
    erg = regime_of(ao, n_stacks, od["max_diff"])
    erg.mode = ao["mode"] & (0x01 | 0x04 | 0x10)          # the extension reads GAPE / LOGGAP as given
    return srg, arg, erg


def device_index(prefix):
    from hsa_amd._lib import GpuIndex
    fwd, rev = index_io.read_index(prefix)
    gi = GpuIndex(fwd, rev)
    gi.set_sa(index_io.read_sa(prefix), index_io.read_blocks(prefix))
    words, dna_len = index_io.read_packed_dna(prefix)
    gi.set_text(words, dna_len)
    return gi


@pytest.mark.skipif(not os.path.exists(PROBE), reason="oracle/_ref/ref_probe not built (make -C oracle)")
@pytest.mark.parametrize("args", [["-n", "4", "-o", "1"], ["-n", "4", "-o", "0"], ["-n", "3", "-o", "1", "-e", "2"]])
def test_splice_kernel_matches_reference(args):
    from oracle_ctypes import default_opt
    man = json.load(open(os.path.join(GOLD, "manifest_dropin.json")))
    reads = fastq_codes(os.path.join(GOLD, man["splice_reads"]))
    prefix = INDEX[man["index"]]
    with tempfile.TemporaryDirectory() as d:
        write_reads(os.path.join(d, "r.bin"), reads)
        subprocess.run([PROBE, "aln", prefix, os.path.join(d, "r.bin"), os.path.join(d, "o.bin"), *args], check=True,
                       capture_output=True, timeout=300)
        ref = read_out(os.path.join(d, "o.bin"))
    od = parse_opts(args, default_opt())                    # local_opt: max_diff fixed by -n, GAPE as given
    fb = [i for i, (na, fl, h) in enumerate(ref) if fl & 1]
    assert len(fb) >= 100
    gi = device_index(prefix)
    srg, arg, erg = regimes(od)
    sub = [reads[i] for i in fb]
    res, st = gi.splice_match(srg, arg, erg, [len(r) for r in sub], np.concatenate(sub),
                              np.full(len(sub), od["max_diff"], np.int32))
    gi.close()
    answered = bad = spliced = 0
    for k, i in enumerate(fb):
        status, n_out = int(res[k, 0]), int(res[k, 1])
        if status:
            continue
        answered += 1
        na, _, h = ref[i]
        got = res[k, 2:2 + 9 * n_out].reshape(-1, 9)
        spliced += n_out > 0
        if n_out != na or not np.array_equal(got, h):
            bad += 1
    assert bad == 0, f"{bad} of {answered} answered reads differ from the reference"
    assert answered >= 0.95 * len(fb), f"only {answered} of {len(fb)} answered ({st})"
    assert spliced > 0 and st["extensions"] > 0


@pytest.mark.skipif(not os.path.exists(PROBE), reason="oracle/_ref/ref_probe not built (make -C oracle)")
def test_device_batch_bounds_and_scratch_release():
    """hsa_splice_device on a device batch of the fixture's fallback reads, two jobs of it
    out of range: one 5 bases longer than the batch's max_len, one of 2 bases.  Those two
    are not taken (HSA_SP_WIN: the caller runs the host's path); every other read is
    answered as the reference answers it.  The batch runs twice on one handle with
    hsa_index_release_scratch between the runs (its buffers freed and grown again):
    the same answers."""
    import torch

    from hsa_amd._lib import JOB_DTYPE, SP_RES_WORDS, SpliceBatch, pad_codes
    from oracle_ctypes import default_opt
    args = ["-n", "4", "-o", "1"]
    man = json.load(open(os.path.join(GOLD, "manifest_dropin.json")))
    reads = fastq_codes(os.path.join(GOLD, man["splice_reads"]))
    prefix = INDEX[man["index"]]
    with tempfile.TemporaryDirectory() as d:
        write_reads(os.path.join(d, "r.bin"), reads)
        subprocess.run([PROBE, "aln", prefix, os.path.join(d, "r.bin"), os.path.join(d, "o.bin"), *args], check=True,
                       capture_output=True, timeout=300)
        ref = read_out(os.path.join(d, "o.bin"))
    od = parse_opts(args, default_opt())
    fb = [i for i, (na, fl, h) in enumerate(ref) if fl & 1]
    sub = [reads[i] for i in fb]
    max_len = max(len(r) for r in sub)
    long_read = np.concatenate([sub[0], sub[0][:5]])            # max_len + 5 bases when sub[0] is the longest
    long_read = np.concatenate([long_read, np.zeros(max_len + 5 - len(long_read), np.uint8)])
    sub = [long_read, sub[1][:2]] + sub[2:]
    lens = np.array([len(r) for r in sub], np.uint32)
    jobs = np.zeros(len(sub), JOB_DTYPE)
    jobs["off"] = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]])
    jobs["len"] = lens
    jobs["max_diff"] = od["max_diff"]
    jobs["seed_len"] = od["seed_len"]
    gi = device_index(prefix)
    srg, arg, erg = regimes(od)
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).cuda()
    d_codes = torch.from_numpy(pad_codes(np.concatenate(sub))).cuda()
    d_flags = torch.ones(len(sub), dtype=torch.int32, device="cuda")      # HSA_F_FALLBACK
    d_n = torch.zeros(len(sub), dtype=torch.int32, device="cuda")
    answers = []
    for run in range(2):
        d_res = torch.full((len(sub) * SP_RES_WORDS,), -1, dtype=torch.int32, device="cuda")
        d_ctr = torch.zeros(8, dtype=torch.int64, device="cuda")
        gi.splice_device(srg, arg, erg, SpliceBatch(
            d_jobs=d_jobs.data_ptr(), n_jobs=len(sub), d_codes=d_codes.data_ptr(), d_flags=d_flags.data_ptr(),
            d_n_aln=d_n.data_ptr(), d_res=d_res.data_ptr(), d_counters=d_ctr.data_ptr(), max_len=max_len))
        torch.cuda.synchronize()
        answers.append(d_res.cpu().numpy().view(np.uint32).reshape(len(sub), SP_RES_WORDS).copy())
        assert int(d_ctr[0]) == len(sub) - 2                    # the two out-of-range jobs were not taken
        if run == 0:
            gi.release_scratch()
    gi.close()
    res = answers[0]
    assert np.array_equal(answers[0], answers[1])
    assert res[0, 0] == 5 and res[1, 0] == 5 and res[0, 1] == 0 and res[1, 1] == 0      # HSA_SP_WIN
    answered = bad = 0
    for k in range(2, len(sub)):
        status, n_out = int(res[k, 0]), int(res[k, 1])
        if status:
            continue
        answered += 1
        na, _, h = ref[fb[k]]
        if n_out != na or not np.array_equal(res[k, 2:2 + 9 * n_out].reshape(-1, 9), h):
            bad += 1
    assert bad == 0 and answered >= 0.95 * (len(sub) - 2)
