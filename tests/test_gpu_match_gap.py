"""bwt_match_gap called directly with the caller's widths, on the GPU:
every call the reference's splice path made on the splice read set -- seed searches
with width_seed aliased to width_back (bwtgap.c:809-812), 12-mer anchors with
width_seed NULL (bwtgap.c:1192) -- and a sample of main-path calls (own width_seed,
bwtaln.c:350), recorded from the compiled reference (tools/make_golden.py --mgcap).
Hits must be identical word for word, and width_back after the call must equal the
reference's (gap_shadow, bwtgap.c:94-105).  Then the whole host program: the
reference's HSA binary with our bwa_cal_sa_reg_gap AND bwt_match_gap linked in
(oracle/ref.mk HSA_gpu_mg) prints byte-identical SAM, splice reads included."""
import gzip
import hashlib
import json
import os
import re
import subprocess

import numpy as np
import pytest

from golden_io import GOLD, INDEX, MGCAP_CASES, load_mgcap
from hsa_amd import index_io

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPT_NAMES = ["s_mm", "s_gapo", "s_gape", "mode", "indel_end_skip", "max_del_occ", "max_entries", "fnr", "max_diff",
             "max_gapo", "max_gape", "max_seed_diff", "seed_len", "n_threads", "max_top2", "trim_qual"]


def opt_dict(words):
    d = {k: int(np.int32(np.uint32(w))) for k, w in zip(OPT_NAMES, words)}
    d["fnr"] = float(np.uint32(words[7]).view(np.float32))
    return d


def run_calls(gi, calls, pool_entries=0):
    """Group the calls by option regime (two per launch), run hsa_match_gap_batch."""
    from hsa_amd import _lib
    from hsa_amd._lib import JOB_DTYPE, MG_DTYPE, regime_of
    keys = {}
    for c in calls:
        o = opt_dict(c["opt"])
        k = (tuple(sorted((n, v) for n, v in o.items() if n not in ("max_diff", "seed_len", "fnr", "n_threads"))),
             c["n_stacks"])
        keys.setdefault(k, []).append(c)
    out = {}
    groups = list(keys.items())
    if pool_entries:
        _lib.configure(pool_entries=pool_entries)
    try:
        for g0 in range(0, len(groups), 2):
            part = groups[g0:g0 + 2]
            sel = [(r, c) for r, (_, cs) in enumerate(part) for c in cs]
            regimes = []
            for _, cs in part:
                o = opt_dict(cs[0]["opt"])
                regimes.append(regime_of(o, cs[0]["n_stacks"], max(opt_dict(c["opt"])["max_diff"] for c in cs)))
            jobs = np.zeros(len(sel), JOB_DTYPE)
            mg = np.zeros(len(sel), MG_DTYPE)
            codes, widths = [], []
            co = wo = 0
            for j, (r, c) in enumerate(sel):
                o = opt_dict(c["opt"])
                jobs[j] = (co, c["len"], o["max_diff"], o["seed_len"], r)
                codes.append(c["seq"])
                co += c["len"]
                mg[j]["wb_off"], mg[j]["strand"], mg[j]["seed"] = wo, c["strand"], c["seed"]
                widths.append(c["wb"])
                wo += c["len"] + 1
                if c["seed"] == 1:
                    mg[j]["ws_off"] = wo
                    widths.append(c["ws"])
                    wo += len(c["ws"])
            n_aln, hoff, hits, wout, _ = gi.match_gap(regimes, jobs, mg, np.concatenate(codes),
                                                      np.concatenate(widths))
            for j, (r, c) in enumerate(sel):
                out[id(c)] = (hits[int(hoff[j]):int(hoff[j]) + n_aln[j]],
                              wout[int(mg[j]["wb_off"]):int(mg[j]["wb_off"]) + c["len"] + 1])
    finally:
        if pool_entries:
            _lib.configure(pool_entries=-1)
    return out


@pytest.fixture(scope="module")
def tiny():
    from hsa_amd._lib import GpuIndex
    return GpuIndex(*index_io.read_index(INDEX["tiny"]))


@pytest.mark.parametrize("name", MGCAP_CASES)
def test_match_gap_calls_match_reference(tiny, name):
    calls = load_mgcap(name)
    assert {c["seed"] for c in calls} == {0, 1, 2}
    got = run_calls(tiny, calls)
    bad = [j for j, c in enumerate(calls)
           if not (np.array_equal(got[id(c)][0], c["hits"]) and np.array_equal(got[id(c)][1], c["wo"]))]
    assert not bad, f"{len(bad)} of {len(calls)} calls differ; first {bad[:5]}"


def test_match_gap_overflow_rerun_is_exact(tiny):
    """A tiny per-lane pool sends the calls through the large-capacity re-run, whose
    width rows are rebuilt from the caller's widths (not from the first pass's)."""
    calls = load_mgcap("mgcap_n4o1")[:600]
    got = run_calls(tiny, calls, pool_entries=16)
    bad = [j for j, c in enumerate(calls)
           if not (np.array_equal(got[id(c)][0], c["hits"]) and np.array_equal(got[id(c)][1], c["wo"]))]
    assert not bad, f"{len(bad)} of {len(calls)} calls differ; first {bad[:5]}"


HSA_GPU_MG = os.path.join(ROOT, "oracle", "_ref", "HSA_gpu_mg")
MAN = json.load(open(os.path.join(GOLD, "manifest_dropin.json")))


@pytest.mark.skipif(not os.path.exists(HSA_GPU_MG), reason="oracle/_ref/HSA_gpu_mg not built (make -C oracle)")
@pytest.mark.parametrize("name,reads", [("splice_default", "splice_reads"), ("splice_n4o1", "splice_reads"),
                                        ("default", "reads"), ("n4o0", "reads")])
def test_dropin_both_entry_points_sam_identical(name, reads):
    fq = os.path.join(GOLD, MAN[reads])
    # the host's bwt_splice_match (HSA_SPLICE_DEVICE=0), so that its bwt_match_gap calls
    # reach our entry point; the device's splice path has its own tests (test_gpu_dropin.py,
    # test_gpu_splice_device.py)
    env = dict(os.environ, HSA_VERBOSE="1", HSA_SPLICE_DEVICE="0")
    r = subprocess.run([HSA_GPU_MG, "aln", *MAN[name]["args"], INDEX["tiny"], fq], capture_output=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    # the splice path's seed searches were answered from the batched prefetch
    m = re.findall(rb"splice prefetch: (\d+) bwt_match_gap calls answered from the batch, (\d+) run alone", r.stderr)
    assert m and sum(int(a) for a, _ in m) > 0, r.stderr.decode()[-2000:]
    if hashlib.sha256(r.stdout).hexdigest() != MAN[name]["sam_sha256"]:
        ref = gzip.open(os.path.join(GOLD, f"dropin_ref_{name}.sam.gz")).read().splitlines()
        got = r.stdout.splitlines()
        diff = [(i, a, b) for i, (a, b) in enumerate(zip(ref, got)) if a != b][:5]
        pytest.fail(f"SAM differs: {len(got)} vs {len(ref)} lines; first differences {diff}")


def test_splice_seeds_device_match_oracle(tiny):
    """hsa_splice_seeds_device: after a device main pass over the splice read set
    (-n 4 -o 1, steady state), the six seed searches of every fallback read -- prefix
    widths, calls and searches all on the device -- equal the restated bwt_match_gap on
    the calls hsa_amd/splice.py builds (which test_splice_seeds.py pins to the
    reference's own seed calls)."""
    import torch
    from hsa_amd import splice
    from hsa_amd._lib import JOB_DTYPE, DeviceBatch, SeedBatch, pad_codes, regime_of
    from oracle_ctypes import Opt, OracleIndex, default_opt
    from test_splice_seeds import read_fastq
    lens, codes = read_fastq(os.path.join(GOLD, MAN["splice_reads"]))
    n = len(lens)
    opt = dict(default_opt(), max_diff=4, fnr=-1.0, max_gapo=1)
    opt["mode"] &= ~0x01
    ox = OracleIndex(*index_io.read_index(INDEX["tiny"]))
    e_n, e_f, _, _ = ox.cal_sa_reg_gap(lens, codes, Opt.from_dict(opt))
    n_stacks = splice.n_stacks_of(opt)
    rg = regime_of(opt, n_stacks, opt["max_diff"])
    jobs = np.zeros(n, JOB_DTYPE)
    jobs["off"] = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]])
    jobs["len"] = lens
    jobs["max_diff"] = opt["max_diff"]
    jobs["seed_len"] = np.where(lens > opt["seed_len"], opt["seed_len"], 0x7FFFFFFF)

    def dev(a):
        return torch.from_numpy(np.ascontiguousarray(a)).cuda()

    d_jobs, d_codes = dev(jobs.view(np.uint8)), dev(pad_codes(codes))
    cap = n * 64
    m = dict(n=torch.zeros(n, dtype=torch.int32, device="cuda"), f=torch.zeros(n, dtype=torch.int32, device="cuda"),
             o=torch.zeros(n, dtype=torch.int64, device="cuda"), h=torch.zeros(cap * 9, dtype=torch.int32, device="cuda"),
             c=torch.zeros(16, dtype=torch.int64, device="cuda"))
    b = DeviceBatch(d_jobs=d_jobs.data_ptr(), n_jobs=n, d_codes=d_codes.data_ptr(), d_n_aln=m["n"].data_ptr(),
                    d_flags=m["f"].data_ptr(), d_hit_off=m["o"].data_ptr(), d_hits=m["h"].data_ptr(), hit_cap=cap,
                    d_counters=m["c"].data_ptr(), max_len=int(lens.max()), max_seed=opt["seed_len"])
    tiny.search_device([rg], b)
    torch.cuda.synchronize()
    g_f = m["f"].cpu().numpy().astype(np.uint32)
    assert np.array_equal(g_f & 1, e_f & 1)
    # the seeds on the device
    so = splice.seed_options(opt)
    srg = regime_of(so, n_stacks, so["max_diff"])
    sn = torch.full((6 * n,), -7, dtype=torch.int32, device="cuda")
    so_ = torch.zeros(6 * n, dtype=torch.int64, device="cuda")
    sh = torch.zeros(cap * 9, dtype=torch.int32, device="cuda")
    sc = torch.zeros(16, dtype=torch.int64, device="cuda")
    sb = SeedBatch(d_jobs=d_jobs.data_ptr(), n_jobs=n, d_codes=d_codes.data_ptr(), d_flags=m["f"].data_ptr(),
                   d_n_aln=sn.data_ptr(), d_hit_off=so_.data_ptr(), d_hits=sh.data_ptr(), hit_cap=cap,
                   d_counters=sc.data_ptr(), max_len=int(lens.max()))
    tiny.splice_seeds_device(srg, sb)
    torch.cuda.synchronize()
    g_n = sn.cpu().numpy()
    g_o = so_.cpu().numpy()
    g_h = sh.cpu().numpy().view(np.uint32).reshape(-1, 9)
    fb = np.flatnonzero(e_f & 1)
    fb = fb[lens[fb] >= 3]
    assert len(fb) > 100
    # records of reads that did not fall back stay untouched
    others = np.setdiff1d(np.arange(n), fb)
    assert (g_n.reshape(n, 6)[others] == -7).all()

    def width_fn(wl, wc):
        out, o = [], 0
        for L in wl:
            out.append(ox.cal_width(wc[o:o + int(L)]).reshape(-1))
            o += int(L)
        return np.concatenate(out).astype(np.uint32)

    hb = splice.seed_calls(lens, codes, fb, opt, width_fn)
    bad = 0
    for c in hb["calls"]:
        o = Opt.from_dict(dict(so, seed_len=int(c["len"])))
        seq = hb["codes"][c["off"]:c["off"] + c["len"]]
        w = hb["widths"][c["wb_off"]:c["wb_off"] + c["len"] + 1]
        exp, _ = ox.match_gap(o, n_stacks, seq, c["strand"], w, 2)
        r = 6 * int(c["read"]) + int(c["i"])
        got = g_h[g_o[r]:g_o[r] + g_n[r]]
        bad += not np.array_equal(got, exp)
    assert bad == 0, f"{bad} of {len(hb['calls'])} seed calls differ"
    assert int(sc[7].item()) > 0     # prefix-width rank queries were counted
