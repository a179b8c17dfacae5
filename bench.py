#!/usr/bin/env python3
"""Throughput of the HSA inexact-alignment path on MI355X (the driver's contract).

Workload (BASELINE.json configs[1]): 100 bp synthetic reads with 0-4 substitutions,
50 % reverse-complemented, searched with `-n 4 -o 0` against a synthetic
hg19-sized bidirectional index (3 000 000 005 bp in 24 records).  A "step" is one
search of the whole 1 M-read workload (configs[1]) as ONE bwa_cal_sa_reg_gap
batch -- a single launch of the persistent search kernel.  (The reference's host
loop feeds 100 000 reads per call, bwtaln.c:477; that is fewer reads than the
262 144 lanes the kernel keeps resident, so the drop-in should be fed larger
batches: INTEGRATION.md.)  Reads, job table and outputs are resident in HBM for
the timed region; steps cycle over a few distinct read sets.

--config 5 (BASELINE configs[4], the HBM-capacity stress): 250 bp reads against a
synthetic ~15 Gbp plant-scale text, which the reference's 32-bit bwtint_t cannot
index: the 64-bit interval instantiation (hsa_search_device64, hsa_aln64_t hits) over
a device-built 64-bit index, parity against the 64-bit restatement (liboracle64.so).

Multi-GPU (one rank per GPU): under torch.distributed.run (WORLD_SIZE set), or with
`--gpus N` alone, which starts the N ranks itself (before anything touches the GPU).
Every rank holds the whole index, searches its own K batches of reads (weak scaling,
no collective on the data path), checks a sample of its timed reads against the CPU
restatement, and the per-rank hit lists of every timed read set are gathered to rank 0
over RCCL after timing; rank 0 re-checks the gathered lists against per-rank digests.

Baselines beside the GPU figure (rank 0 at N=1, configs 2 and 3): the restatement on
the box's CPU share (the whole timed batch, also the parity check), and the
REFERENCE's own bwa_cal_sa_reg_gap (oracle/_ref/ref_probe, compiled from its sources
in the build container) on index files written from the device-built BWTs, one process
per core of the share.  The drop-in end to end: the reference's driver linked with
every drop-in entry point of ours (oracle/_ref/ref_probe_gpu) on bwa_seq_t batches of
100 000 reads, splice fallback included, its hits compared with the reference's.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time
from datetime import timedelta

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
# hsa_amd (which loads libhsa_gpu.so, before torch: hsa_amd/_lib.py) is imported in
# main(), after `--gpus N` has started its ranks: the parent never loads the library.
REF_DIR = os.path.join(ROOT, "oracle", "_ref")

GENOME_T = 3_000_000_005
GENOME5_T = 15_000_000_003  # config 5: plant-scale, past 2^32
GENOME_SEED = 1234
RECORDS = 24
READ_LEN = 100
BATCH = 1_000_000
DISTINCT = 3            # distinct read sets the steps cycle over
METRIC = "aligned reads/sec, 100bp synthetic vs hg19-sized 2BWT, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_QUERY = 64    # one 64-byte HBM sector per Occ query
SA_INTERVAL = 8         # the .sa sampling of `HSA index` (2BWT-Builder.c:97)
REF_BATCH = 100_000     # bwa_aln_core's batch (bwtaln.c:477)
PASS_RING = 1024        # per-pass kernel events the library keeps (hsa_index::PASS_RING)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_index(T, seed, device, with_files=False):
    """The hg19-sized index on the device.  with_files: also keep the text (packed) and
    the forward direction's every-8th SA values (hsa_build_bwt_index_device, the same
    sort: the .sa of `HSA index`), for the reference's index files (reference_files)."""
    import torch
    from hsa_amd import _lib
    L = _lib.lib()
    nw = (T + 15) // 16
    text = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
    _lib.check(L.hsa_synth_genome_device(device, T, seed, text.data_ptr()))
    res = {}
    extra = {}
    sa = None
    for rev in (0, 1):
        bw = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
        isa0 = C.c_uint32()
        Cc = np.zeros(5, np.uint32)
        t0 = time.time()
        if rev == 0:
            # the forward BWT and (with_files) every SA_INTERVAL-th suffix-array value of
            # the same sort, for the reference's .sa
            i64 = C.c_uint64()
            C64 = np.zeros(5, np.uint64)
            sa = torch.zeros(T // SA_INTERVAL + 2 if with_files else 1, dtype=torch.int32, device="cuda")
            _lib.check(L.hsa_build_bwt_index_device(device, T, text.data_ptr(), bw.data_ptr(), C.byref(i64), C64,
                                                    SA_INTERVAL if with_files else 0,
                                                    sa.data_ptr() if with_files else None))
            isa0.value = int(i64.value)
            Cc[:] = C64.astype(np.uint32)
            if with_files:
                extra["sa"] = sa[:T // SA_INTERVAL + 1].cpu().numpy().view(np.uint32)
        else:
            _lib.check(L.hsa_build_bwt_device(device, T, text.data_ptr(), rev, bw.data_ptr(), C.byref(isa0), Cc))
        log(f"[bench] BWT{' (reverse)' if rev else ''} of {T} bp built on the device in {time.time() - t0:.1f} s")
        res[rev] = (bw, int(isa0.value), Cc)
    if with_files:
        extra["text"] = text[:nw].cpu().numpy().view(np.uint32)
    gi = _lib.GpuIndex.from_device_codes(T, res[0][1], res[0][2], res[0][0].data_ptr(), T, res[1][1], res[1][2],
                                         res[1][0].data_ptr(), device=device)
    del text, sa
    torch.cuda.empty_cache()
    return gi, res, extra


def build_index64(T, seed, device):
    """config 5: the 64-bit index (hsa_build_bwt_device64 + hsa_index_create_device64)."""
    import torch
    from hsa_amd import _lib
    L = _lib.lib()
    nw = (T + 15) // 16
    text = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
    _lib.check(L.hsa_synth_genome_device(device, T, seed, text.data_ptr()))
    res = {}
    for rev in (0, 1):
        bw = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
        isa0 = C.c_uint64()
        Cc = np.zeros(5, np.uint64)
        t0 = time.time()
        _lib.check(L.hsa_build_bwt_device64(device, T, text.data_ptr(), rev, bw.data_ptr(), C.byref(isa0), Cc))
        log(f"[bench] BWT{' (reverse)' if rev else ''} of {T} bp built on the device in {time.time() - t0:.1f} s "
            f"(64-bit)")
        res[rev] = (bw, int(isa0.value), Cc)
    del text
    torch.cuda.empty_cache()
    gi = _lib.GpuIndex.from_device_codes64(T, res[0][1], res[0][2], res[0][0].data_ptr(), T, res[1][1], res[1][2],
                                           res[1][0].data_ptr(), device=device)
    return gi, res, {}


def msb_words(lsb):
    """16 two-bit codes per u32: LSB-first (code j at bits 2j) <-> MSB-first (code j at
    bits 30 - 2j, the .bwt / HSP packedDNA order)."""
    x = lsb.astype(np.uint32, copy=True)
    x = (x >> 16) | (x << 16)
    x = ((x & 0xFF00FF00) >> 8) | ((x & 0x00FF00FF) << 8)
    x = ((x & 0xF0F0F0F0) >> 4) | ((x & 0x0F0F0F0F) << 4)
    x = ((x & 0xCCCCCCCC) >> 2) | ((x & 0x33333333) << 2)
    return x


def attach_splice_arrays(gi, T, extra):
    """What the splice kernel reads besides the rank blocks, as the reference's loaded
    index holds it: the sampled SA (BWTLoad: values[0] = -1, BWT.c:222) with the record
    blocks of the synthetic genome's .ann, and the packed text as the HSP holds it
    ((T + 15) / 16 + 1 words, first code in the high bits; DNALoadPacked)."""
    from hsa_amd import synth
    vals = np.ascontiguousarray(extra["sa"], np.uint32).copy()
    vals[0] = 0xFFFFFFFF
    blocks = np.array([[r, s0, s0 + n - 1, 0] for r, (s0, n) in enumerate(synth.record_layout(T, RECORDS))],
                      np.int64).astype(np.uint32)
    gi.set_sa(index_io_sa(vals), blocks)
    nw = (T + 15) // 16
    words = np.zeros(nw + 1, np.uint32)
    words[:nw] = msb_words(extra["text"][:nw])
    if T % 16:                  # the .pac holds zero bits past the text (its last byte masked)
        words[nw - 1] &= np.uint32((0xFFFFFFFF << (32 - 2 * (T % 16))) & 0xFFFFFFFF)
    gi.set_text(words, T)


def index_io_sa(vals):
    from hsa_amd import index_io
    return index_io.SaFile(interval=SA_INTERVAL, values=vals)


def host_oracle_index64(res, T):
    """The 64-bit restatement's index (liboracle64.so) from the device-built BWTs."""
    from oracle_ctypes import OracleIndex64
    nw = (T + 15) // 16
    w = [res[r][0][:nw].cpu().numpy().view(np.uint32) for r in (0, 1)]
    return OracleIndex64(T, res[0][1], res[0][2], w[0], T, res[1][1], res[1][2], w[1])


def host_oracle_index(res, T):
    """The CPU restatement's index, from the device-built BWT (MSB-first .bwt words)."""
    from hsa_amd import index_io
    from oracle_ctypes import OracleIndex
    metas = []
    for rev in (0, 1):
        bw, isa0, Cc = res[rev]
        lsb = bw.cpu().numpy().view(np.uint32)[:(T + 15) // 16]
        x = lsb.copy()
        x = (x >> 16) | (x << 16)
        x = ((x & 0xFF00FF00) >> 8) | ((x & 0x00FF00FF) << 8)
        x = ((x & 0xF0F0F0F0) >> 4) | ((x & 0x0F0F0F0F) << 4)
        x = ((x & 0xCCCCCCCC) >> 2) | ((x & 0x33333333) << 2)
        metas.append(index_io.BwtFile(T=T, isa0=isa0, C=Cc.astype(np.uint32), code=x.astype(np.uint32)))
    return OracleIndex(metas[0], metas[1])


# per-config PMC summaries (tools/profile_run.sh + tools/pmc_summary.py; config 4's in
# its "step" mode, which sums the main path's and the splice seeds' kernels); the
# kernel-trace summaries next to them (tools/trace_summary.py) give the same runs'
# per-launch durations
TRAFFIC_SRCS = {2: "profiles/r06_pmc_summary_config2.json", 3: "profiles/r05_pmc_summary_config3.json",
                4: "profiles/r05_pmc_summary_config4.json", 5: "profiles/r06_pmc_summary_config5.json"}


def traffic_per_kernel(config):
    """HBM read+write bytes per launch of each kernel from the committed PMC pass
    (FETCH_SIZE calibrated on random 64-B gathers + WRITE_SIZE; tools/profile_run.sh,
    tools/pmc_summary.py) -- counters cannot be read in the timed run itself."""
    try:
        with open(os.path.join(ROOT, TRAFFIC_SRCS[config])) as f:
            d = json.load(f)
        return {k: round(v["fetch_bytes"] + v["write_bytes"]) for k, v in d["per_kernel"].items()}
    except (OSError, KeyError, ValueError, TypeError):
        return {}


def diag_dump(path):
    """Diagnostic builds only (libhsa_gpu_diag.so): per-workgroup clock stamps of
    the last launch -> in-kernel clock and workgroup-duration spread."""
    from hsa_amd import _lib
    L = _lib.lib()
    nb = 8192
    buf = np.zeros(nb * 4, np.uint64)
    _lib.check(L.hsa_diag_read(buf.ctypes.data_as(C.c_void_p), nb))
    d = buf.reshape(nb, 4).astype(np.int64)
    d = d[d[:, 3] > 0]
    t0 = d[:, 1].min()
    dur_ms = (d[:, 3] - d[:, 1]) / 100e3          # s_memrealtime: 100 MHz
    clk = (d[:, 2] - d[:, 0]) / np.maximum(d[:, 3] - d[:, 1], 1) * 100.0
    out = {"blocks": int(len(d)), "clock_mhz_median": float(np.median(clk)),
           "start_spread_ms": float((d[:, 1].max() - t0) / 100e3),
           "dur_ms_pct": [float(np.percentile(dur_ms, q)) for q in (0, 10, 50, 90, 99, 100)],
           "end_ms_pct": [float(np.percentile((d[:, 3] - t0) / 100e3, q)) for q in (0, 10, 50, 90, 99, 100)]}
    ev = (C.c_ulonglong * 32)()
    _lib.check(L.hsa_diag_counters(ev, 0))
    names = ["width_steps", "exact_steps", "expand_steps", "vt_pops", "pool_pops", "outer_iters_per_wave",
             "lanes_stepping", "control_iters_per_wave", "pool_flushes", "cyc_acquire", "cyc_control",
             "cyc_rank_wait", "cyc_apply", "gap_shadows", "gap_shadow_ldp_sum", "strand_starts",
             "exact_steps_unique", "expand_steps_unique", "pruned_pops", "doomed_pushes", "hits"]
    out["events_total"] = {n: int(ev[i]) for i, n in enumerate(names)}
    log(f"[bench] diag: {json.dumps(out)}")
    with open(path, "w") as f:
        json.dump(out, f)


def cpu_widths(ox, wl, wc):
    """bwt_cal_width type 1 of each sequence on the CPU restatement (flat pairs)."""
    out, o = [], 0
    for L in wl:
        out.append(ox.cal_width(wc[o:o + int(L)]).reshape(-1))
        o += int(L)
    return np.concatenate(out).astype(np.uint32)



def cpu_info():
    """The host CPU the baseline ran on: model, physical cores visible, and the
    threads used (the CPUs this process may run on, at most 16: the GPU box's share)."""
    model, phys = "unknown", set()
    try:
        pid = cid = None
        for ln in open("/proc/cpuinfo"):
            k, _, v = ln.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name":
                model = v
            elif k == "physical id":
                pid = v
            elif k == "core id":
                cid = v
                phys.add((pid, cid))
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0))
    return {"model": model, "physical_cores": len(phys) or None, "affinity": aff,
            "threads": max(1, min(aff, int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16))}


def oracle_threaded(ox, reads, RL, od, threads):
    """bwa_cal_sa_reg_gap on the C restatement over disjoint chunks, one thread each
    (ctypes releases the GIL; a steady-state batch: chunking does not change results).
    Returns n_aln, flags, hits in read order, and the rank queries."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle_ctypes import Opt
    n = len(reads)
    edges = np.linspace(0, n, threads + 1).astype(np.int64)

    def one(i):
        ch = reads[edges[i]:edges[i + 1]]
        return ox.cal_sa_reg_gap(np.full(len(ch), RL, np.uint32), np.ascontiguousarray(ch).reshape(-1),
                                 Opt.from_dict(od))
    with ThreadPoolExecutor(threads) as ex:
        outs = list(ex.map(one, range(threads)))
    return (np.concatenate([o[0] for o in outs]), np.concatenate([o[1] for o in outs]),
            np.concatenate([o[2] for o in outs]), sum(int(o[3][0]) for o in outs))


def compare_batch(g_n, g_f, g_o, g_h, o_n, o_f, o_h):
    """Reads whose n_aln, fallback flag or hit records (every field, in order) differ."""
    g_n = np.maximum(g_n.astype(np.int64), 0)
    bad = (g_n != o_n) | ((g_f & 1) != (o_f & 1))
    same = np.flatnonzero(~bad & (g_n > 0))
    # GPU hits of those reads, gathered into read order
    cnt = g_n[same]
    idx = np.repeat(g_o[same].astype(np.int64) - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt) + \
        np.arange(int(cnt.sum()))
    o_off = np.concatenate([[0], np.cumsum(o_n.astype(np.int64))])
    oidx = np.repeat(o_off[same] - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt) + np.arange(int(cnt.sum()))
    diff = (g_h[idx] != o_h[oidx]).any(axis=1)
    if diff.any():
        owner = np.repeat(same, cnt)
        bad[np.unique(owner[diff])] = True
    nb = int(bad.sum())
    return nb, (int(np.flatnonzero(bad)[0]) if nb else None)

def step_plan(steps, warmup, nd, S):
    """The timed loop's schedule: per step (handle, read set, step whose end it waits
    for).  Steps on one handle run in issue order; a step that reuses a read set's
    output buffers on another handle waits for that set's previous step, so no two
    steps that may run at once write the same outputs (tests/test_bench_helpers.py)."""
    return [(s % S, (warmup + s) % nd, s - nd if S > 1 and s >= nd else None) for s in range(steps)]


# ---------------------------------------------------------------- N ranks from --gpus N
def spawn_ranks(n, argv, script=None):
    """`bench.py --gpus N` without a launcher: start N ranks of this script (RANK,
    LOCAL_RANK = GPU, WORLD_SIZE, MASTER_* on 127.0.0.1), relay rank 0's JSON line and
    return the worst exit status.  The parent imports neither torch nor hsa_amd, so no
    process here has touched the GPU before its ranks start."""
    import socket
    import subprocess
    import tempfile
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs, outs = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = tempfile.TemporaryFile() if r == 0 else subprocess.DEVNULL
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=out))
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0:
                rc = rc or c
                log(f"[bench] rank {r} exited with {c}: stopping the others")
                for q in live:
                    procs[q].terminate()
        time.sleep(0.2)
    outs[0].seek(0)
    for line in outs[0].read().decode().splitlines(keepends=True):   # the JSON line; the rest to stderr
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
    sys.stdout.flush()
    return rc


def hits_in_read_order(n_aln, hit_off, hits):
    """A batch's hit records in read order (the kernel appends each read's hits
    wherever its atomic lands): the gather's and the digests' layout."""
    cnt = np.maximum(np.asarray(n_aln, np.int64), 0)
    if cnt.sum() == 0:
        return np.zeros((0, hits.shape[1]), np.uint32)
    starts = np.asarray(hit_off, np.int64)
    idx = np.repeat(starts - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt) + np.arange(int(cnt.sum()))
    return np.ascontiguousarray(hits[idx], np.uint32)


def batch_digest(n_aln, flags, hits_ordered):
    """SHA-256 of one batch's results (n_aln, fallback flags, hits in read order)."""
    import hashlib
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(n_aln, np.int32).tobytes())
    h.update((np.asarray(flags, np.uint32) & 1).astype(np.uint32).tobytes())
    h.update(np.ascontiguousarray(hits_ordered, np.uint32).tobytes())
    return h.hexdigest()


# ---------------------------------------------------------------- the reference's own path
def write_reads_bin(path, reads):
    """ref_probe's reads.bin: u32 n, u32 len[n], then the codes."""
    reads = np.ascontiguousarray(reads, np.uint8)
    with open(path, "wb") as f:
        f.write(np.array([len(reads)], np.uint32).tobytes())
        f.write(np.full(len(reads), reads.shape[1], np.uint32).tobytes())
        f.write(reads.tobytes())


def read_probe_out(path):
    """ref_probe's out.bin -> (n_aln, hits of every read concatenated (n, 9))."""
    b = np.fromfile(path, np.uint32)
    assert b[0] == 0x48415348, "bad ref_probe output"
    n = int(b[1])
    n_aln = np.zeros(n, np.int32)
    hits = []
    i = 2
    for r in range(n):
        na = int(np.int32(b[i]))
        i += 2
        n_aln[r] = na
        if na > 0:
            hits.append(b[i:i + 9 * na].reshape(na, 9))
            i += 9 * na
    return n_aln, (np.concatenate(hits) if hits else np.zeros((0, 9), np.uint32))


def reference_files(d, T, res, extra):
    """The hg19-sized index as `HSA index` files under d (prefix d/g): .bwt / .rev.bwt
    from the device-built BWTs (MSB-first words, BWTConstruct.c:1209-1224), .fmv /
    .rev.fmv by the reference's own BWTGenerateOccValueFromBwt (ref_probe mkfmv), .sa
    from the device sort's samples (BWTConstruct.c:1373-1392), .pac / .ann from the
    synthetic text and its record layout (HSP.c:313-337)."""
    import subprocess

    from hsa_amd import index_build, synth
    prefix = os.path.join(d, "g")
    nw = (T + 15) // 16
    for rev, suf in ((0, ""), (1, ".rev")):
        bw, isa0, Cc = res[rev]
        x = bw[:nw].cpu().numpy().view(np.uint32).copy()       # LSB-first -> MSB-first codes
        x = (x >> 16) | (x << 16)
        x = ((x & 0xFF00FF00) >> 8) | ((x & 0x00FF00FF) << 8)
        x = ((x & 0xF0F0F0F0) >> 4) | ((x & 0x0F0F0F0F) << 4)
        x = ((x & 0xCCCCCCCC) >> 2) | ((x & 0x33333333) << 2)
        with open(f"{prefix}.index{suf}.bwt", "wb") as f:
            f.write(np.concatenate([[isa0], np.asarray(Cc, np.uint32)[1:5]]).astype(np.uint32).tobytes())
            f.write(x.astype(np.uint32).tobytes())
        del x
        subprocess.run([os.path.join(REF_DIR, "ref_probe"), "mkfmv", f"{prefix}.index{suf}.bwt",
                        f"{prefix}.index{suf}.fmv"], check=True, timeout=600)
    index_build.write_sa(prefix, T, res[0][1], res[0][2], SA_INTERVAL, extra["sa"])
    # .pac: 4 codes per byte, first code in the high bits (text words are LSB-first)
    b = extra["text"].view(np.uint8)
    b = ((b & 3) << 6) | ((b & 12) << 2) | ((b >> 2) & 12) | (b >> 6)
    nb = (T + 3) // 4
    body = b[:nb].copy()
    if T % 4:
        body[-1] &= np.uint8((0xFF << (8 - 2 * (T % 4))) & 0xFF)
    with open(f"{prefix}.index.pac", "wb") as f:
        f.write(body.tobytes())
        f.write((b"\x00" if T % 4 == 0 else b"") + bytes([T % 4]))
    recs = synth.record_layout(T, RECORDS)
    ann = [(f"chr{r + 1}", [(s0, s0 + n - 1, 0)]) for r, (s0, n) in enumerate(recs)]
    with open(f"{prefix}.index.ann", "w") as f:
        f.write(index_build.ann_text(ann, T))
    return prefix


def parse_batch_stages(err):
    """The drop-in's per-call stage lines (HSA_VERBOSE, bwtaln_gpu.c: "[hsa] batch of N reads:
    search S s, splice prefetch P s, splice path H s (F fallback reads, ...") -> the sums of
    the three stages, the fallback reads and each call's total."""
    splice_s, search_s, prefetch_s, n_fb, calls = 0.0, 0.0, 0.0, 0, []
    for ln in err.splitlines():
        if ln.startswith("[hsa] batch of"):
            parts = ln.replace(",", "").split()
            c_path = float(parts[parts.index("path") + 1])
            c_search = float(parts[parts.index("search") + 1])
            c_pf = float(parts[parts.index("prefetch") + 1])
            splice_s += c_path
            search_s += c_search
            prefetch_s += c_pf
            calls.append(c_path + c_search + c_pf)
            n_fb += int(ln.split("(")[-1].split()[0])
    return splice_s, search_s, prefetch_s, n_fb, calls


def reference_legs(T, res, extra, reads_all, opt_args, n_ref, procs, e2e_reads):
    """The reference's own bwa_cal_sa_reg_gap on the box's cores, and the drop-in end to
    end (ref_probe_gpu), on the same index files; returns the bench fields."""
    import shutil
    import subprocess
    import tempfile
    probe, probe_gpu = os.path.join(REF_DIR, "ref_probe"), os.path.join(REF_DIR, "ref_probe_gpu")
    if not (os.path.exists(probe) and os.path.exists(probe_gpu)):
        return {"skipped": "oracle/_ref/ref_probe(_gpu) not built"}
    d = tempfile.mkdtemp(prefix="hsa_ref_")
    try:
        t0 = time.time()
        prefix = reference_files(d, T, res, extra)
        log(f"[bench] reference index files written in {time.time() - t0:.1f} s")
        # the reference: `procs` processes (one core each; it is single-threaded,
        # bwtaln.c:307-311), each one batch of n_ref / procs reads
        per = max(1, n_ref // procs)
        jobs = []
        for k in range(procs):
            rb = os.path.join(d, f"ref_reads{k}.bin")
            write_reads_bin(rb, reads_all[k * per:(k + 1) * per])
            jobs.append(subprocess.Popen([probe, "aln", prefix, rb, os.path.join(d, f"ref_out{k}.bin"), *opt_args,
                                          "-B", str(REF_BATCH)], stdout=subprocess.PIPE, stderr=subprocess.PIPE))
        ts = []
        for k, j in enumerate(jobs):
            o, e = j.communicate(timeout=900)
            if j.returncode != 0:
                raise RuntimeError(f"ref_probe rank {k}: {e.decode()[-500:]}")
            ts.append(float(o.decode().split()[-1]))
        ref = {"value": round(per * procs / max(ts), 1), "unit": "reads/s", "cores": procs, "kind": "reference",
               "value_1core": round(per / float(np.median(ts)), 1),
               "sample": f"the reference's own bwa_cal_sa_reg_gap (oracle/_ref/ref_probe, gcc -O3 from its sources) "
                         f"on {procs} processes x {per} reads of the timed batch, one core each (the reference is "
                         f"single-threaded), index files from the device-built BWTs; search seconds per process "
                         f"{min(ts):.1f}-{max(ts):.1f} (index load excluded)"}
        log(f"[bench] reference CPU path: {ref['value']:.0f} reads/s on {procs} cores ({ref['value_1core']:.0f} per core)")
        r_n, r_h = read_probe_out(os.path.join(d, "ref_out0.bin"))      # process 0: the first `per` reads
        if e2e_reads <= 0:
            return {"reference": ref, "dropin_e2e": None, "ref0": (r_n, r_h)}
        # the drop-in end to end on the same files: bwa_seq_t batches of 100 000 reads
        rb = os.path.join(d, "e2e_reads.bin")
        write_reads_bin(rb, reads_all[:e2e_reads])
        env = dict(os.environ, HSA_VERBOSE="1", HSA_MALLOC_TUNE="1")    # the host's heap kept
        j = subprocess.run([probe_gpu, "aln", prefix, rb, os.path.join(d, "gpu_out.bin"), *opt_args, "-B",
                            str(REF_BATCH)], capture_output=True, timeout=900, env=env)
        err = j.stderr.decode(errors="replace")
        if os.environ.get("HSA_E2E_LOG"):                  # the drop-in's stage timings, whole
            with open(os.environ["HSA_E2E_LOG"], "w") as f:
                f.write(err)
        if j.returncode != 0:                              # the reference leg above still counts
            tail = [ln for ln in err.splitlines() if not ln.startswith("[hsa] ")][-6:]
            log(f"[bench] drop-in end to end failed (exit {j.returncode}): {' | '.join(tail)}")
            return {"reference": ref, "dropin_e2e": {"error": f"ref_probe_gpu exit {j.returncode}",
                                                     "stderr_tail": tail}}
        t_gpu = float(j.stdout.decode().split()[-1])
        splice_s, search_s, prefetch_s, n_fb, calls = parse_batch_stages(err)
        # parity through the real entry point: rank 0's reads are a prefix of the first
        # 100 000-read batch in both runs, so their hits (splice path's included) agree
        g_n, g_h = read_probe_out(os.path.join(d, "gpu_out.bin"))
        m = len(r_n)
        go = np.concatenate([[0], np.cumsum(np.maximum(g_n, 0).astype(np.int64))])
        ro = np.concatenate([[0], np.cumsum(np.maximum(r_n, 0).astype(np.int64))])
        bad = [i for i in range(m) if g_n[i] != r_n[i] or not np.array_equal(g_h[go[i]:go[i + 1]], r_h[ro[i]:ro[i + 1]])]
        e2e = {"reads": e2e_reads, "reads_per_call": REF_BATCH, "value": round(e2e_reads / t_gpu, 1), "unit": "reads/s",
               "seconds": round(t_gpu, 3), "splice_fallback_reads": n_fb, "splice_path_s": round(splice_s, 3),
               "main_search_s": round(search_s, 3), "splice_prefetch_s": round(prefetch_s, 3),
               "splice_path_us_per_fallback_read": round(1e6 * splice_s / n_fb, 1) if n_fb else None,
               "first_call_s": round(calls[0], 3) if calls else None,
               "median_later_call_s": round(float(np.median(calls[1:])), 3) if len(calls) > 1 else None,
               "what": "the reference's driver (ref_probe.c) linked with every drop-in entry point of ours "
                       "(oracle/_ref/ref_probe_gpu, as HSA_gpu_all): bwa_cal_sa_reg_gap on bwa_seq_t batches from "
                       "host memory, bwt_splice_match of the fallback reads on the device (the prefetch pass and the "
                       "splice kernel; the host's own for reads the kernel hands back); wall time of the calls",
               "parity_vs_reference": {"reads": m, "mismatching_reads": len(bad), "first_mismatch": bad[0] if bad else None,
                                       "fields": "n_aln and every bwt_aln1_t field of every hit, splice-path hits "
                                                 "included, hit order"}}
        log(f"[bench] drop-in end to end: {e2e['value']:.0f} reads/s ({e2e_reads} reads in calls of {REF_BATCH}, "
            f"{n_fb} fallback reads; main search {search_s:.3f} s, splice prefetch {prefetch_s:.3f} s, splice path "
            f"{splice_s:.3f} s); {len(bad)} of {m} reads differ from the reference")
        return {"reference": ref, "dropin_e2e": e2e, "ref0": (r_n, r_h)}
    finally:
        shutil.rmtree(d, ignore_errors=True)


class _BatchCodes:
    """The global read stream's codes as hsa_amd.shard.search_sharded slices them
    (codes[offs[b0]:offs[b1]]), holding only this rank's batches (fixed_total)."""

    def __init__(self, batches: dict, per_batch_codes: int):
        self.d, self.m = batches, per_batch_codes

    def __getitem__(self, sl):
        return self.d[sl.start // self.m].reshape(-1)


def fixed_total(a):
    """--total-reads R: BASELINE configs[2] as it is stated -- R reads in the reference's
    100 000-read batches (bwtaln.c:477), the batches dealt round-robin to the ranks
    (hsa_amd.shard.search_sharded: each batch searched with the option state the
    sequential reference has when it reaches that batch, SURVEY Q2/Q3, plus the one
    all-reduce), through the drop-in's bwa_cal_sa_reg_gap semantics on host arrays
    (hsa_cal_sa_reg_gap_flat: H2D reads, search, D2H hits, per-read unpacking), then the
    hit lists gathered to rank 0 (timed apart: `gather.ms`).  Total work is fixed, so
    `scaling` is "strong"; `value` = R / the slowest rank's time.  Each rank checks a
    sample of one steady-state batch (GAPE already cleared) against the restatement."""
    import hsa_amd  # noqa: F401  (libhsa_gpu.so before torch)
    import torch
    import torch.distributed as dist
    from hsa_amd import _lib, shard, synth
    from hsa_amd._lib import GapOpt
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("HSA_BENCH_BACKEND", "nccl")
    comm = torch.device("cpu")
    if world > 1:
        gpu = local % torch.cuda.device_count() if backend == "gloo" else local
        torch.cuda.set_device(gpu)
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
            comm = torch.device("cuda", gpu)
    device = torch.cuda.current_device()
    T = a.genome or GENOME_T
    R = a.total_reads
    max_gapo = 0 if a.config == 2 else 1
    t0 = time.time()
    gi, res, _ = build_index(T, GENOME_SEED, device)
    genome = synth.PackedGenome(T, GENOME_SEED)
    recs = synth.record_layout(T, RECORDS)
    bounds = shard.batch_bounds(R, REF_BATCH)
    mine = shard.my_batches(len(bounds), world, rank)
    seed0 = (6 if a.config == 3 else 5) * 10_000_000            # not the weak mode's read sets
    reads = {}
    for b in mine:
        n = bounds[b][1] - bounds[b][0]
        if a.config == 3:
            reads[b], _ = synth.make_reads(genome, recs, n, READ_LEN, seed0 + b, indel=True, max_mm_indel=2)
        else:
            reads[b], _ = synth.make_reads(genome, recs, n, READ_LEN, seed0 + b, max_mm=4)
    log(f"[bench] rank {rank}: index and {len(mine)} batches of {REF_BATCH} reads ready in {time.time() - t0:.1f} s")
    opt = GapOpt.default()                      # the process's first batch: GAPE still set
    opt.max_diff, opt.fnr, opt.max_gapo = 4, -1.0, max_gapo
    opt0 = opt.as_dict()
    lens = np.full(R, READ_LEN, np.uint32)
    codes = _BatchCodes(reads, REF_BATCH * READ_LEN)
    stats = []

    def search(l, c, o):
        n_aln, flags, hoff, hits, st = gi.cal_sa_reg_gap(l, c, o)
        stats.append(st)
        return n_aln, flags, hoff, hits

    def allreduce_max(x):
        t = torch.from_numpy(x.astype(np.int64)).to(comm)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.cpu().numpy().astype(np.int32)

    # warm-up (untimed): one steady-state call, kernels loaded and scratch grown
    wb = mine[0] if mine else 0
    if mine:
        gi.cal_sa_reg_gap(lens[:REF_BATCH], reads[wb].reshape(-1), GapOpt.from_dict(shard.opt_entering_batch(opt0, 1,
                                                                                                              False)))
    stats.clear()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    info = {}
    out = shard.search_sharded(search, GapOpt.from_dict, opt0, lens, codes, REF_BATCH, world, rank, allreduce_max, info)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    mine_s = elapsed
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=comm)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    q = sum(s["rank_queries"] for s in stats)
    kms = sum(s["kernel_ms"] for s in stats)
    t1 = time.perf_counter()
    g = shard.gather_to_root(out, dist, comm, per_batch=True) if world > 1 else \
        {b: (v[0], v[1], v[3]) for b, v in out.items()}
    t_gather = time.perf_counter() - t1
    # parity: a sample of one steady-state batch of this rank against the restatement
    pb = next((b for b in mine if b > 0), None)
    par = (rank, 0, 0, None)
    if pb is not None and a.rank_parity:
        from oracle_ctypes import default_opt
        ox = host_oracle_index(res, T)
        od = default_opt()
        od.update(max_diff=4, fnr=-1.0, max_gapo=max_gapo, mode=od["mode"] & ~0x01)
        n = min(a.rank_parity, bounds[pb][1] - bounds[pb][0])
        o_n, o_f, o_h, _ = oracle_threaded(ox, reads[pb][:n], READ_LEN, od, cpu_info()["threads"])
        n_aln, flags, hoff, hits = out[pb]
        bad, first = compare_batch(n_aln[:n], flags[:n], hoff, np.asarray(hits, np.uint32).reshape(-1, 9), o_n, o_f,
                                   o_h)
        par = (rank, n, bad, first)
        del ox
        log(f"[bench] rank {rank}: parity batch {pb}: {n} reads, {bad} differ from the restatement")
    pr = [par]
    roof = [(rank, q, kms, mine_s)]
    if world > 1:
        pr, roof = [None] * world, [None] * world
        dist.all_gather_object(pr, par)
        dist.all_gather_object(roof, (rank, q, kms, mine_s))
    if rank == 0:
        n_got = sum(len(v[0]) for v in g.values())
        qa, ka = sum(x[1] for x in roof), max(x[2] for x in roof)
        ach = q * BYTES_PER_QUERY / (kms / 1e3) / 1e9 if kms > 0 else 0.0
        result = {
            "metric": METRIC, "value": round(R / elapsed, 1), "unit": "reads/s", "n_gpus": world, "steps": 1,
            "warmup": 1, "ms_per_step": round(elapsed * 1e3, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": f"{R} x {READ_LEN}bp reads fixed total ("
                                   + ("one 1-3 bp indel + 0-2 substitutions, -n 4 -o 1" if a.config == 3 else
                                      "0-4 substitutions, -n 4 -o 0")
                                   + f") in the reference's {REF_BATCH}-read batches dealt round-robin over {world} "
                                     f"GPU(s), bwa_cal_sa_reg_gap semantics on host arrays (H2D reads, search, D2H "
                                     f"hits, per-read unpacking), the process's first batch with GAPE set (SURVEY Q2), "
                                     f"vs synthetic hg19-sized 2BWT ({T} bp) (BASELINE configs[{a.config - 1}])",
                       "genome_bp": T, "total_reads": R, "batches": len(bounds), "reads_per_batch": REF_BATCH,
                       "parallelism": f"whole batches over {world} rank(s) (hsa_amd/shard.py), index replicated",
                       "backend": dist.get_backend() if world > 1 else None},
            "timing_window": "barrier -> every batch of the rank through hsa_cal_sa_reg_gap_flat (host arrays in and "
                             "out) + the option-state all-reduce -> barrier, max over ranks; the gather after it",
            "roofline": {"bound": "hbm", "kernel": "all search kernels of the calls", "achieved": round(ach, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel_ms_rank0": round(kms, 1), "kernel_ms_max_rank": round(ka, 1),
                         "rank_queries_all_ranks": int(qa)},
            "gather": {"ms": round(t_gather * 1e3, 1), "batches": len(g), "reads": int(n_got),
                       "complete": n_got == R and len(g) == len(bounds)},
            "option_state": {"first_sticky_batch": info.get("first_sticky"), "rerun": info.get("rerun")},
            "per_rank_s": {str(r): round(x[3], 3) for r, x in enumerate(roof)},
            "parity_ranks": {str(r): {"batch_reads_checked": n, "mismatching_reads": b, "first_mismatch": f}
                             for r, n, b, f in pr},
            "parity_against": "oracle (C restatement), the first reads of one steady-state batch per rank"}
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    gi.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--genome", type=int, default=0, help="text length (default: hg19-sized; config 5: 15 Gbp)")
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--cpu-sample", type=int, default=20000, help="reads timed on the CPU restatement")
    ap.add_argument("--parity-sample", type=int, default=-1,
                    help="reads of the timed batch checked against the CPU restatement (-1: all of them; 0: none)")
    ap.add_argument("--config", type=int, default=2, choices=(2, 3, 4, 5),
                    help="BASELINE.json config: 2 = 0-4 substitutions, -n 4 -o 0 (default, the metric's config); "
                         "3 = one 1-3 bp indel + 0-2 substitutions, -n 4 -o 1; "
                         "4 = 150 bp spliced reads, -n 4 -o 1, main path + the splice path's seed searches; "
                         "5 = 250 bp reads, 0-4 substitutions, -n 4 -o 0, 15 Gbp text, 64-bit intervals")
    ap.add_argument("--dropin", type=int, default=1, help="also time the host-array drop-in path (1) or not (0)")
    ap.add_argument("--intervals", type=int, default=0, choices=(0, 32, 64),
                    help="SA interval width of the search (0: 64 for config 5, else 32); 64 on a sub-2^32 text "
                         "and 32 with config 5's reads on one are A/B runs of the two instantiations")
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--pool", type=int, default=0)
    ap.add_argument("--roofline-steps", type=int, default=-1,
                    help="serialized steps after the timed region that the kernel roofline is taken over "
                         "(-1: 20 when --streams > 1, else none: the timed launches themselves)")
    ap.add_argument("--dropin-slots", type=int, default=1,
                    help="also time the drop-in leg with its reads split over this many handles of the index")
    ap.add_argument("--streams", type=int, default=0,
                    help="handles on the index (hsa_index_clone) that consecutive steps alternate over, so step "
                         "s+1's kernels fill the last waves of step s's k_search; handles past the second whose "
                         "search scratch does not fit are dropped (0: 3 for configs 2 and 3, else 2; config 4 "
                         "takes ~115 GB of scratch per handle)")
    ap.add_argument("--ref-sample", type=int, default=-1,
                    help="reads the REFERENCE's own CPU path (oracle/_ref/ref_probe) searches, over --ref-procs "
                         "processes (-1: 8 000 per process for config 2, 2 000 for config 3, 1 000 for config 4; 0: "
                         "skip the reference legs)")
    ap.add_argument("--ref-procs", type=int, default=0,
                    help="reference processes (0: the CPU threads of the job's share, 16 per GPU rank)")
    ap.add_argument("--e2e-reads", type=int, default=1_000_000,
                    help="reads of the drop-in end-to-end leg (oracle/_ref/ref_probe_gpu, 100 000 per call)")
    ap.add_argument("--copies", type=int, default=1,
                    help="also time the steps with the H2D reads and D2H hits inside them (value_with_copies)")
    ap.add_argument("--rank-parity", type=int, default=100_000,
                    help="with N > 1 ranks: reads of each rank's timed batch checked against the restatement")
    ap.add_argument("--total-reads", type=int, default=0,
                    help="fixed-total mode (strong scaling, BASELINE configs[2] as stated: e.g. --config 3 "
                         "--total-reads 10000000): the reads in the reference's 100 000-read batches dealt over the "
                         "ranks, host-array bwa_cal_sa_reg_gap semantics, gather timed apart (fixed_total)")
    a = ap.parse_args()
    if a.streams <= 0:
        # three handles where three handles' scratch fits: config 2 +1.8 % (profiles/r05_streams3_ab.log),
        # config 3 +0.8-1.6 % with its 16 384-entry pools (profiles/r05_pool16k_ab.log)
        a.streams = 3 if a.config in (2, 3) else 2
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))
    if a.total_reads > 0:
        if a.config not in (2, 3):
            sys.exit("--total-reads: configs 2 and 3")
        return fixed_total(a)

    import hsa_amd  # noqa: F401  (libhsa_gpu.so before torch)
    import torch
    import torch.distributed as dist
    from hsa_amd import _lib, synth
    from hsa_amd._lib import DeviceBatch, GapOpt, Regime

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL over xGMI, one GPU per rank.  HSA_BENCH_BACKEND=gloo is a rehearsal of the
    # N-rank path on a box with fewer GPUs: ranks share GPUs round-robin and the
    # collectives go over gloo on host tensors (its timings say nothing about scaling).
    backend = os.environ.get("HSA_BENCH_BACKEND", "nccl")
    comm = None
    if world > 1:
        gpu = local % torch.cuda.device_count() if backend == "gloo" else local
        torch.cuda.set_device(gpu)
        if backend == "gloo":
            dist.init_process_group("gloo")
            comm = torch.device("cpu")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
            comm = torch.device("cuda", gpu)
    device = torch.cuda.current_device()
    _lib.configure(a.waves, a.pool, 0)

    wide = a.intervals == 64 or (a.intervals == 0 and a.config == 5)   # the 64-bit interval instantiation
    T = a.genome or (GENOME5_T if a.config == 5 else GENOME_T)
    RL = {4: 150, 5: 250}.get(a.config, READ_LEN)
    HW = _lib.ALN64_WORDS if wide else 9      # u32 words per hit record
    # the reference's CPU path runs on rank 0 after the gather, one process per thread of
    # the job's CPU share (16 per GPU rank: the whole share of the node at N = 8)
    # (never more processes than the CPUs this process may run on: they inherit its affinity)
    ref_procs = a.ref_procs or min(cpu_info()["threads"] * world, cpu_info()["affinity"])
    if a.ref_sample < 0:
        a.ref_sample = {2: 8_000, 3: 2_000, 4: 1_000}.get(a.config, 0) * ref_procs
    # The contract prices the CPU baseline on rank 0 at N = 1 only; at N > 1 the reference's
    # processes (each loads the ~4 GB index files: 16 per rank would be ~0.5 TB of host memory
    # at N = 8) are not started.  HSA_BENCH_REF_AT_N=1 runs them anyway (rehearsals).
    ref_legs = rank == 0 and a.config in (2, 3, 4) and not wide and a.ref_sample > 0 and T < (1 << 32) and \
        (world == 1 or os.environ.get("HSA_BENCH_REF_AT_N") == "1")
    t0 = time.time()
    if wide:
        gi, res, extra = build_index64(T, GENOME_SEED, device)
    else:
        gi, res, extra = build_index(T, GENOME_SEED, device, with_files=ref_legs or a.config == 4)
        if a.config == 4:       # the splice kernel's SA -> position and motif scans
            attach_splice_arrays(gi, T, extra)
    trie_d, trie_sd, trie_b = gi.trie()
    log(f"[bench] rank {rank}: index ready ({gi.nbytes() / 2**30:.2f} GiB of rank blocks, root tries {trie_d}/{trie_sd} "
        f"levels in {trie_b / 2**20:.0f} MiB) in {time.time() - t0:.1f} s")

    # reads: rank r searches batches r, r+world, ... of one global stream (seed 5)
    t0 = time.time()
    genome = synth.PackedGenome(T, GENOME_SEED)
    recs = synth.record_layout(T, RECORDS)
    nb = a.warmup + a.steps
    nd = min(nb, DISTINCT)
    batches = []
    for j in range(nd):
        gidx = j * world + rank
        if a.config == 2:
            reads, _ = synth.make_reads(genome, recs, a.batch, READ_LEN, 5 * 1_000_000 + gidx, max_mm=4)
        elif a.config == 5:
            reads, _ = synth.make_reads(genome, recs, a.batch, RL, 8 * 1_000_000 + gidx, max_mm=4)
        elif a.config == 4:  # SURVEY §8d config 4 (seed 7): exon A 40-110, GT..AG intron 200-5000
            reads, _ = synth.make_spliced_reads(genome, recs, a.batch, RL, 7 * 1_000_000 + gidx)
        else:   # SURVEY §8d config 3 reads (seed 6): one indel of 1-3 bp + 0-2 substitutions
            reads, _ = synth.make_reads(genome, recs, a.batch, READ_LEN, 6 * 1_000_000 + gidx, indel=True,
                                        max_mm_indel=2)
        batches.append(reads)
    log(f"[bench] rank {rank}: {nd} x {a.batch} reads generated in {time.time() - t0:.1f} s")

    # bwa_cal_sa_reg_gap prologue on the host (bwtaln.c:254-337): -n 4 -o 0|1, fixed length.
    # The timed batches are steady-state batches (not the process's first): GAPE is
    # already cleared in the caller's block, so both option regimes coincide.
    max_gapo = 0 if a.config in (2, 5) else 1
    opt_str = f"-n 4 -o {max_gapo}"
    opt = GapOpt.default()
    opt.max_diff, opt.fnr, opt.max_gapo = 4, -1.0, max_gapo
    opt.mode &= ~0x01
    # aln_score(max_diff+1, max_gapo+1, max_gape+1) of local_opt (bwtaln.c:264-267, bwtgap.c:18)
    n_stacks = (opt.max_diff + 1) * opt.s_mm + (opt.max_gapo + 1) * opt.s_gapo + (opt.max_gape + 1) * opt.s_gape
    rg = Regime(s_mm=opt.s_mm, s_gapo=opt.s_gapo, s_gape=opt.s_gape, mode=0, indel_end_skip=opt.indel_end_skip,
                max_del_occ=opt.max_del_occ, max_entries=opt.max_entries, max_gapo=max_gapo, max_gape=opt.max_gape,
                max_seed_diff=opt.max_seed_diff, max_top2=opt.max_top2, n_stacks=n_stacks, max_diff=opt.max_diff)
    jobs = np.zeros(a.batch, _lib.JOB_DTYPE)
    jobs["off"] = np.arange(a.batch, dtype=np.uint64) * RL
    jobs["len"] = RL
    jobs["max_diff"] = opt.max_diff
    jobs["seed_len"] = opt.seed_len
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).cuda()
    d_codes = [torch.from_numpy(_lib.pad_codes(b.reshape(-1))).cuda() for b in batches]
    hit_cap = a.batch * 8
    outs = []
    for j in range(nd):
        outs.append(dict(n=torch.zeros(a.batch, dtype=torch.int32, device="cuda"),
                         f=torch.zeros(a.batch, dtype=torch.int32, device="cuda"),
                         o=torch.zeros(a.batch, dtype=torch.int64, device="cuda"),
                         h=torch.zeros(hit_cap * HW, dtype=torch.int32, device="cuda"),
                         c=torch.zeros(16, dtype=torch.int64, device="cuda")))
        if a.config == 4:   # the splice path's answers: HSA_SP_RES_WORDS words per read
            outs[-1].update(res=torch.zeros(a.batch * _lib.SP_RES_WORDS, dtype=torch.int32, device="cuda"),
                            sc=torch.zeros(8, dtype=torch.int64, device="cuda"))
    if a.config == 4:
        from hsa_amd import splice
        from hsa_amd._lib import SpliceBatch, anchor_regime, ext_regime, regime_of
        so_opt = splice.seed_options(opt.as_dict())
        srg = regime_of(so_opt, n_stacks, so_opt["max_diff"])
        arg_ = anchor_regime(opt.as_dict(), n_stacks, opt.max_diff)
        erg = ext_regime(opt.as_dict(), n_stacks, opt.max_diff)

    handles = [gi] + [gi.clone() for _ in range(max(1, a.streams) - 1)]

    def launch(j, hi=0):
        j %= nd
        o = outs[j]
        gi = handles[hi]
        b = DeviceBatch(d_jobs=d_jobs.data_ptr(), n_jobs=a.batch, d_codes=d_codes[j].data_ptr(),
                        d_n_aln=o["n"].data_ptr(), d_flags=o["f"].data_ptr(), d_hit_off=o["o"].data_ptr(),
                        d_hits=o["h"].data_ptr(), hit_cap=hit_cap, d_counters=o["c"].data_ptr(),
                        max_len=RL, max_seed=opt.seed_len)
        (gi.search_device64 if wide else gi.search_device)([rg], b)
        if a.config == 4:   # same stream: the splice path of the main pass's fallback reads
            gi.splice_device(srg, arg_, erg, SpliceBatch(
                d_jobs=d_jobs.data_ptr(), n_jobs=a.batch, d_codes=d_codes[j].data_ptr(), d_flags=o["f"].data_ptr(),
                d_n_aln=o["n"].data_ptr(), d_res=o["res"].data_ptr(), d_counters=o["sc"].data_ptr(), max_len=RL))

    # the measured ceiling for this access pattern: random whole 64-B blocks over a
    # table as large as the rank index (before the timed region, same process)
    rand_gbs = _lib.probe_gather(gi.nbytes(), 1, device)
    rand64_gbs = _lib.probe_gather(gi.nbytes(), 4, device)
    coop_gbs = _lib.probe_gather(gi.nbytes(), 2, device)
    log(f"[bench] rank {rank}: random-sector gather probe over {gi.nbytes() / 2**30:.2f} GiB: {rand_gbs:.0f} GB/s "
        f"(16-B loads), {coop_gbs:.0f} GB/s (4 lanes x 16 B per sector), {rand64_gbs:.0f} GB/s (whole sectors per lane)")

    # a handle past the second whose search scratch does not fit (a gapped regime's pool
    # is ~95 GB per handle at config 3) is dropped before the timed region
    for hi in range(len(handles)):              # in order: the first two must fit
        try:
            launch(0, hi)
            torch.cuda.synchronize()
        except _lib.HsaError as ex:
            if hi < 2 or "allocation" not in str(ex):
                raise
            log(f"[bench] rank {rank}: {len(handles) - hi} handle(s) dropped: {ex}")
            for h in handles[hi:]:
                h.close()
            del handles[hi:]
            break
    S = len(handles)
    lib_streams = [torch.cuda.ExternalStream(h.stream_handle()) for h in handles]
    for j in range(max(a.warmup, S)):         # every handle's scratch is allocated before the timed region
        launch(j if j < a.warmup else 0, j % S)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    if os.environ.get("HSA_DIAG_OUT"):
        _lib.check(_lib.lib().hsa_diag_counters((C.c_ulonglong * 32)(), 1))
    t0 = time.perf_counter()
    for s, (hi, _, after) in enumerate(step_plan(a.steps, a.warmup, nd, S)):
        st = lib_streams[hi]
        if after is not None:                 # read set (warmup + s) % nd's outputs: its last writer is done
            st.wait_event(ev[after][1])
        ev[s][0].record(st)
        launch(a.warmup + s, hi)
        ev[s][1].record(st)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kms = [e0.elapsed_time(e1) for e0, e1 in ev]
    # per-kernel device time of every timed step: HIP events the library records on
    # its stream around k_widths and k_search (+ its overflow re-run) of each pass
    n_pt = min(a.steps, PASS_RING)             # the library keeps the newest PASS_RING passes per handle
    per_h = [len(range(h, a.steps, S)) for h in range(S)]
    pt = [handles[h].pass_times(min(per_h[h], PASS_RING)) for h in range(S) if per_h[h]]
    w_ms = np.concatenate([p[0] for p in pt]).astype(float)
    s_ms = np.concatenate([p[1] for p in pt]).astype(float)
    n_pt = len(w_ms)
    splice_ms = float(np.mean(kms[-n_pt:]) - np.mean(w_ms) - np.mean(s_ms)) if a.config == 4 else None
    log(f"[bench] rank {rank}: per-step kernels: k_widths {np.mean(w_ms):.2f} ms, k_search {np.mean(s_ms):.2f} ms"
        + (f", splice path {splice_ms:.2f} ms" if a.config == 4 and S == 1 else ""))
    if os.environ.get("HSA_DIAG_OUT"):
        diag_dump(os.environ["HSA_DIAG_OUT"])
    log(f"[bench] rank {rank}: per-step device ms {[round(x, 2) for x in kms]}, wall {elapsed * 1e3:.1f} ms")
    # With S > 1 handles the timed launches overlap, so their event times are not one
    # launch's device time: the kernel roofline is then taken over R more steps of the
    # same read sets, one after another on one stream, right after the timed region.
    R = (min(a.steps, 20) if S > 1 else 0) if a.roofline_steps < 0 else a.roofline_steps
    ovl_w, ovl_s = w_ms, s_ms
    roof_sets = [(a.warmup + s) % nd for s in range(a.steps)]
    if R:
        torch.cuda.synchronize()
        evr = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(R)]
        for s in range(R):
            evr[s][0].record(lib_streams[0])
            launch(a.warmup + s, 0)
            evr[s][1].record(lib_streams[0])
        torch.cuda.synchronize()
        w_ms, s_ms = (x.astype(float) for x in handles[0].pass_times(min(R, PASS_RING)))
        roof_sets = [(a.warmup + s) % nd for s in range(R)][-len(w_ms):]
        if a.config == 4:       # the splice path of a step alone: the serialized step less its two kernels
            step_ser = [e0.elapsed_time(e1) for e0, e1 in evr][-len(w_ms):]
            splice_ms = float(np.mean(step_ser) - np.mean(w_ms) - np.mean(s_ms))
            log(f"[bench] rank {rank}: splice path of a serialized step: {splice_ms:.2f} ms")
        log(f"[bench] rank {rank}: {R} serialized steps: k_widths {np.mean(w_ms):.2f} ms, k_search "
            f"{np.mean(s_ms):.2f} ms (overlapped in the timed region: {np.mean(ovl_w):.2f} / {np.mean(ovl_s):.2f} ms)")
    # The same K steps with the PCIe copies inside each step (SURVEY §8d's timing window:
    # H2D reads -> width + search kernels -> D2H hits): reads from pinned host memory into
    # the read set's device buffer, the per-read outputs and the batch's hit records back,
    # all on the step's handle stream, so the copies of one step overlap the other
    # handle's kernels.  Reported beside `value`, never as it.
    copies = None
    if a.copies and world == 1 and a.config != 4:
        h_codes = [d_codes[j].cpu().pin_memory() for j in range(nd)]
        nh_set = {j: int(outs[j]["c"][1].item()) for j in range(nd)}       # a read set's hit count: fixed
        h_out = [dict(n=torch.empty(a.batch, dtype=torch.int32).pin_memory(),
                      f=torch.empty(a.batch, dtype=torch.int32).pin_memory(),
                      o=torch.empty(a.batch, dtype=torch.int64).pin_memory(),
                      h=torch.empty(max(nh_set[j], 1) * HW, dtype=torch.int32).pin_memory()) for j in range(nd)]
        torch.cuda.synchronize()
        evc = [torch.cuda.Event() for _ in range(a.steps)]
        t0 = time.perf_counter()
        for s, (hi, j, after) in enumerate(step_plan(a.steps, a.warmup, nd, S)):
            st = lib_streams[hi]
            with torch.cuda.stream(st):
                if after is not None:
                    st.wait_event(evc[after])
                d_codes[j].copy_(h_codes[j], non_blocking=True)
                launch(j, hi)
                o = outs[j]
                for k in ("n", "f", "o"):
                    h_out[j][k].copy_(o[k], non_blocking=True)
                h_out[j]["h"][:nh_set[j] * HW].copy_(o["h"][:nh_set[j] * HW], non_blocking=True)
                evc[s].record(st)
        torch.cuda.synchronize()
        el_c = time.perf_counter() - t0
        bytes_in = sum(d_codes[(a.warmup + s) % nd].numel() for s in range(a.steps))
        bytes_out = sum(a.batch * 16 + nh_set[(a.warmup + s) % nd] * HW * 4 for s in range(a.steps))
        copies = {"value": round(a.batch * a.steps / el_c, 1), "unit": "reads/s",
                  "ms_per_step": round(el_c * 1e3 / a.steps, 3),
                  "h2d_bytes_per_step": bytes_in // a.steps, "d2h_bytes_per_step": bytes_out // a.steps,
                  "what": "the timed steps again with H2D of the reads (pinned) and D2H of n_aln, flags, hit offsets "
                          "and the hit records inside each step, on the step's handle stream (the copies of one "
                          "step overlap the other handle's kernels); SURVEY 8d's timing window"}
        log(f"[bench] rank {rank}: with the copies inside the step: {copies['value']:.0f} reads/s "
            f"({copies['ms_per_step']:.2f} ms per step)")
        del h_codes, h_out
    for h in handles[1:]:       # their search scratch (a gapped pool is tens of GB) goes back before the other legs
        h.close()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=comm)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # counters and outputs of the timed launches (the last launch on each read set)
    used = sorted({(a.warmup + s) % nd for s in range(a.steps)})
    per = {j: sum(1 for s in range(a.steps) if (a.warmup + s) % nd == j) for j in used}
    ctr = np.stack([outs[j]["c"].cpu().numpy() * per[j] for j in used])
    queries = int(ctr[:, 2].sum())             # what the reference algorithm issues (include/hsa_gpu.h)
    q_widths = int(ctr[:, 7].sum())            # ... of it in k_widths (strands the reference searches)
    q_search = queries - q_widths              # ... of it in k_search
    q_widths_issued = q_widths - int(ctr[:, 14].sum()) + int(ctr[:, 13].sum())   # + speculative fwd rows
    unfinished = int(ctr[:, 11].sum())
    if unfinished:
        log(f"[bench] WARNING: {unfinished} reads unfinished (hit buffer too small)")
    seed_queries = 0
    splice = None
    if a.config == 4:   # the splice path: its seed and anchor searches' rank queries (with their widths)
        sctr = np.stack([outs[j]["sc"].cpu().numpy() * per[j] for j in used])
        seed_queries = int(sctr[:, 5].sum())
        queries += seed_queries
        nfb = max(int(sctr[:, 0].sum()), 1)
        res_all = [outs[j]["res"].cpu().numpy().view(np.uint32).reshape(-1, _lib.SP_RES_WORDS) for j in used]
        splice = {"reads": int(sctr[:, 0].sum()), "extensions_per_read": round(int(sctr[:, 1].sum()) / nfb, 2),
                  "extension_pops_per_read": round(int(sctr[:, 2].sum()) / nfb, 1),
                  "sa_lookups_per_read": round(int(sctr[:, 3].sum()) / nfb, 1),
                  "not_answered": int(sctr[:, 4].sum()),
                  "spliced_reads": int(sum(int(((r[:, 0] == 0) & (r[:, 1] > 0)).sum()) * per[j]
                                           for r, j in zip(res_all, used))),
                  "what": "bwt_splice_match of every fallback read on the device (hsa_splice_device: the seed and "
                          "anchor searches, then hsa_splice.hip's kernel: correlation, motif scan, extensions, "
                          "intron-end checks); not_answered = reads the kernel hands to the host's bwt_splice_match "
                          "(outside the timed step)"}
    blocks = int(ctr[:, 3].sum())
    pops = int(ctr[:, 4].sum())
    flags = np.concatenate([np.tile(outs[j]["f"].cpu().numpy(), per[j]) for j in used])
    n_aln = np.concatenate([np.tile(outs[j]["n"].cpu().numpy(), per[j]) for j in used])
    overflow = int(((flags & 2) != 0).sum())
    if overflow:
        log(f"[bench] WARNING: {overflow} reads overflowed the per-lane capacity in the timed launches")
    mapped = int((n_aln > 0).sum())
    fallback = int(((flags & 1) != 0).sum())
    reads_local = a.steps * a.batch

    # final hit-list gather to rank 0 (RCCL over xGMI): every read set the timed steps
    # searched (each is one global batch; a read set searched twice gives the same
    # hits), then the counters.  Every rank also sends a digest of each of its batches,
    # and rank 0 checks the gathered lists against them.
    total_hits_local = int(ctr[:, 1].sum())
    gather = None
    if world > 1:
        from hsa_amd import shard
        mine, digests = {}, {}
        for j in used:
            o = outs[j]
            nh = int(o["c"][1].item())
            n_j, f_j, ho_j = o["n"].cpu().numpy(), o["f"].cpu().numpy().view(np.uint32), o["o"].cpu().numpy()
            h_j = o["h"][:nh * HW].cpu().numpy().view(np.uint32).reshape(-1, HW)
            gidx = j * world + rank                                 # global batch index of read set j
            mine[gidx] = (n_j, f_j, ho_j, h_j)
            digests[gidx] = batch_digest(n_j, f_j, hits_in_read_order(n_j, ho_j, h_j))
        t0 = time.perf_counter()
        g = shard.gather_to_root(mine, dist, comm, per_batch=True)
        t_gather = time.perf_counter() - t0
        all_dig = [None] * world
        dist.all_gather_object(all_dig, digests)
        if rank == 0:
            want = {b: h for d in all_dig for b, h in d.items()}
            bad = sorted(b for b in want if b not in g or batch_digest(g[b][0], g[b][1], g[b][2]) != want[b])
            gather = {"batches": len(g), "reads": int(sum(len(v[0]) for v in g.values())),
                      "hits": int(sum(len(v[2]) for v in g.values())), "ms": round(t_gather * 1e3, 1),
                      "batches_differing_from_rank_digest": bad, "backend": dist.get_backend()}
            log(f"[bench] gathered {gather['batches']} batches / {gather['reads']} reads / {gather['hits']} hits from "
                f"{world} ranks in {gather['ms']} ms; {len(bad)} differ from their rank's digest")
        cnt = torch.tensor([total_hits_local, mapped, fallback], dtype=torch.int64, device=comm)
        dist.all_reduce(cnt)
        mapped_all, fallback_all = int(cnt[1].item()), int(cnt[2].item())
    else:
        mapped_all, fallback_all = mapped, fallback

    # the dominant kernel: k_search, its algorithmic bytes per launch (the reference's
    # rank queries it answers x one 64-byte sector) over its mean launch time from the
    # per-pass HIP events of the launches the kernel times above belong to (the timed
    # ones, or the serialized roofline steps): their read sets' counters.  Every rank
    # measures its own; rank 0 reports them all.
    ms_search, ms_widths = float(np.mean(s_ms)), float(np.mean(w_ms))
    cset = {j: outs[j]["c"].cpu().numpy() for j in set(roof_sets)}
    qs_launch = float(np.mean([cset[j][2] - cset[j][7] for j in roof_sets]))
    qw_launch = float(np.mean([cset[j][7] for j in roof_sets]))
    ach_search = qs_launch * BYTES_PER_QUERY / (ms_search / 1e3) / 1e9
    ach_widths = qw_launch * BYTES_PER_QUERY / (ms_widths / 1e3) / 1e9
    per_rank_roof = [(rank, ms_search, ach_search, rand_gbs)]
    if world > 1:
        per_rank_roof = [None] * world
        dist.all_gather_object(per_rank_roof, (rank, ms_search, ach_search, rand_gbs))

    result = None
    if rank == 0:
        reads_all = reads_local * world
        value = reads_all / elapsed
        mean_kms = float(np.mean(kms))
        q_per_launch = queries / a.steps
        # the whole step in the timed region: its algorithmic bytes over the wall time per step
        ms_step = elapsed * 1e3 / a.steps
        ach_step = q_per_launch * BYTES_PER_QUERY / (ms_step / 1e3) / 1e9
        pk = traffic_per_kernel(a.config)
        result = {
            "metric": METRIC, "value": round(value, 1), "unit": "reads/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64" if wide else "u32", "data": "synthetic",
            "timing_window": ("device-resident reads: barrier -> K steps of widths + search kernels (+ the capacity "
                              "re-runs; config 4: + the splice path) on device batches -> barrier, max over ranks; "
                              "not SURVEY 8d's window (H2D reads -> kernels -> D2H hits), which value_with_copies "
                              "times (N = 1)"),
            "config": {"workload": f"{a.batch // 1000}k x {RL}bp reads per step and GPU, "
                                   + {2: "0-4 substitutions", 3: "one 1-3 bp indel + 0-2 substitutions",
                                      4: "spliced (exon 40-110 bp, GT..AG intron 200-5000 bp), main path + the whole "
                                         "splice path of every fallback read on the GPU (seeds, anchors, correlation, "
                                         "motif scan, extensions, intron-end checks: hsa_splice_device)",
                                      5: "0-4 substitutions, 64-bit SA intervals (hsa_search_device64)"}[a.config]
                                   + f", 50% rc, vs synthetic {'plant-scale' if T >= 1 << 32 else 'hg19-sized'} 2BWT ({T} bp, "
                                   f"{RECORDS} records), {opt_str} (BASELINE configs[{a.config - 1}]); "
                                   f"{a.steps} timed steps",
                       "genome_bp": T, "reads_per_step": a.batch, "read_len": RL, "options": opt_str,
                       "parallelism": f"reads sharded over {world} GPU(s), index replicated",
                       "streams": S},
            "roofline": {"bound": "hbm", "kernel": "k_search", "achieved": round(ach_search, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(ach_search / HBM_PEAK_GBS, 4),
                         "traffic": pk.get("k_search"),
                         "k_search_ms": round(ms_search, 3),
                         "k_search_algorithmic_bytes_per_launch": qs_launch * BYTES_PER_QUERY,
                         "kernel_times_from": (f"{len(s_ms)} serialized launches after the timed region (one stream; "
                                               f"the {S} streams' timed launches overlap: k_widths "
                                               f"{np.mean(ovl_w):.3f} ms, k_search {np.mean(ovl_s):.3f} ms per launch "
                                               "there)") if R else "the timed launches",
                         "k_search_frac_of_random_sector": round(ach_search / rand_gbs, 4),
                         # the same kernel by its counter bytes (the PMC pass's FETCH + WRITE per launch):
                         # Q credits 64 B to every reference query, while the kernel loads fewer
                         # blocks (width trie, one block for both ends of a narrow interval, L2 hits)
                         "k_search_counter_gbs": (round(pk["k_search"] / (ms_search / 1e3) / 1e9, 1)
                                                  if pk.get("k_search") else None),
                         "k_search_counter_frac_of_random_sector": (
                             round(pk["k_search"] / (ms_search / 1e3) / 1e9 / rand_gbs, 4) if pk.get("k_search")
                             else None),
                         "k_search_frac_of_random_sector_coop": round(ach_search / coop_gbs, 4),
                         "k_widths": {"ms": round(ms_widths, 3), "achieved": round(ach_widths, 1),
                                      "frac": round(ach_widths / HBM_PEAK_GBS, 4),
                                      "frac_of_random_sector": round(ach_widths / rand_gbs, 4),
                                      "rank_queries_per_read": round(q_widths / reads_local, 1),
                                      "issued_queries_per_read": round(q_widths_issued / reads_local, 1),
                                      "traffic": (pk.get("k_widths", 0) + pk.get("k_widths_reads", 0)) or None},
                         "step": {"ms": round(ms_step, 3), "event_ms": round(mean_kms, 3),
                                  "achieved": round(ach_step, 1),
                                  "frac": round(ach_step / HBM_PEAK_GBS, 4),
                                  "frac_of_random_sector": round(ach_step / rand_gbs, 4)},
                         "rank_queries_per_read": round(queries / reads_local, 1),
                         "k_search_rank_queries_per_read": round(q_search / reads_local, 1),
                         "sectors_per_query": round(blocks / max(queries, 1), 4),
                         "tries": {"width_depth": trie_d, "search_depth": trie_sd, "bytes": trie_b,
                                   "loads_per_read": round(int(ctr[:, 10].sum()) / reads_local, 1),
                                   "what": "steps answered by one root-trie load instead of a rank pair "
                                           "(hsa_amd/csrc/hsa_trie.h); they still count as the reference's queries"},
                         "bytes_per_query": BYTES_PER_QUERY,
                         "peak_random_sector_measured": round(rand_gbs, 1),
                         "peak_random_sector_measured_coop4x16": round(coop_gbs, 1),
                         "peak_random_sector_measured_64B_loads": round(rand64_gbs, 1),
                         "traffic_source": TRAFFIC_SRCS.get(a.config),
                         "per_rank": {str(r): {"k_search_ms": round(m, 3), "achieved": round(x, 1),
                                               "frac": round(x / HBM_PEAK_GBS, 4),
                                               "frac_of_random_sector": round(x / g, 4)}
                                      for r, m, x, g in per_rank_roof}},
            "mapped_frac": round(mapped_all / reads_all, 4), "fallback_frac": round(fallback_all / reads_all, 4),
            "pops_per_read": round(pops / reads_local, 1),
        }
        if copies is not None:
            result["value_with_copies"] = copies
        if a.config == 4:
            result["seed_rank_queries_per_read"] = round(seed_queries / reads_local, 1)
            result["roofline"]["splice_path_ms"] = round(splice_ms, 3)
            result["splice_path"] = splice
        if gather is not None:
            result["gather"] = gather

    # the drop-in path (rank 0, N=1, configs 2 and 3): the C-ABI bwa_cal_sa_reg_gap
    # (flat form) on HOST arrays, the way a host HSA aln calls it -- reads copied in,
    # hits copied out and unpacked per read -- at the reference's 100 000 reads per
    # call (bwtaln.c:477) and at the whole 1 M-read batch per call
    if rank == 0 and world == 1 and a.config in (2, 3) and a.dropin:
        src = batches[0]
        dres = {}
        for k_slots in sorted({1, a.dropin_slots}):
            others = [gi.clone() for _ in range(k_slots - 1)]   # slots on this GPU: handles of one index
            for per_call in (100_000, a.batch):
                per_call = min(per_call, a.batch)
                o = GapOpt.from_dict(opt.as_dict())

                def call(m, r0):
                    if others:
                        gi.cal_sa_reg_gap_slots(others, np.full(m, RL, np.uint32), src[r0:r0 + m].reshape(-1), o)
                    else:
                        gi.cal_sa_reg_gap(np.full(m, RL, np.uint32), src[r0:r0 + m].reshape(-1), o)
                call(per_call, 0)   # warm
                t0 = time.perf_counter()
                done = 0
                while done < a.batch:
                    m = min(per_call, a.batch - done)
                    call(m, done)
                    done += m
                dt = time.perf_counter() - t0
                key = str(per_call) + (f"_slots{k_slots}" if k_slots > 1 else "")
                dres[key] = round(a.batch / dt, 1)
                log(f"[bench] drop-in path: {a.batch} reads in calls of {per_call} over {k_slots} slot(s): "
                    f"{a.batch / dt:.0f} reads/s")
            for h in others:
                h.close()
        result["dropin"] = {"unit": "reads/s", "reads_per_call": dres,
                            "what": "hsa_cal_sa_reg_gap_flat on host arrays: H2D reads, widths + search + "
                                    "re-runs, D2H hits, per-read unpacking (PCIe and host work included)"}

    # N > 1: every rank checks a sample of its own timed batch against the restatement
    # (host threads of its share), rank 0 reports them all
    if world > 1 and a.rank_parity and a.config != 4:
        ox = (host_oracle_index64 if wide else host_oracle_index)(res, T)
        from oracle_ctypes import default_opt
        od = default_opt()
        od.update(max_diff=4, fnr=-1.0, max_gapo=max_gapo, mode=od["mode"] & ~0x01)
        j0 = a.warmup % nd
        n = min(a.rank_parity, a.batch)
        o = outs[j0]
        t0 = time.perf_counter()
        o_n, o_f, o_h, o_q = oracle_threaded(ox, batches[j0][:n], RL, od, cpu_info()["threads"])
        bad, first = compare_batch(o["n"].cpu().numpy()[:n], o["f"].cpu().numpy().astype(np.uint32)[:n],
                                   o["o"].cpu().numpy(), o["h"].cpu().numpy().view(np.uint32).reshape(-1, HW),
                                   o_n, o_f, o_h)
        log(f"[bench] rank {rank}: parity sample {n} reads, {bad} differ ({time.perf_counter() - t0:.1f} s)")
        pr = [None] * world
        dist.all_gather_object(pr, (rank, n, bad, first))
        if rank == 0:
            result["parity_ranks"] = {str(r): {"reads": nn, "mismatching_reads": b, "first_mismatch": f}
                                      for r, nn, b, f in pr}
            result["parity_ranks_against"] = ("oracle (C restatement" + (", 64-bit)" if wide else ")") +
                                              ": the first reads of each rank's first timed read set; every field of "
                                              "every hit, hit order, fallback flags")
        del ox

    # parity and the CPU baseline (rank 0 at N=1 only): configs 2 and 3 compare the
    # WHOLE timed batch with the C restatement run on the host's cores (that run is
    # the CPU baseline); config 4 checks a sample (its seed calls are driven from
    # Python one by one)
    if rank == 0 and world == 1 and (a.parity_sample or a.cpu_sample):
        t0 = time.time()
        ox = (host_oracle_index64 if wide else host_oracle_index)(res, T)
        log(f"[bench] CPU restatement index built in {time.time() - t0:.1f} s")
        from oracle_ctypes import Opt, default_opt
        od = default_opt()
        od.update(max_diff=4, fnr=-1.0, max_gapo=max_gapo, mode=od["mode"] & ~0x01)
        cpu = cpu_info()
        j0 = a.warmup % nd
        last = outs[j0]
        g_n = last["n"].cpu().numpy()
        g_f = last["f"].cpu().numpy().astype(np.uint32)
        g_o = last["o"].cpu().numpy()
        g_h = last["h"].cpu().numpy().view(np.uint32).reshape(-1, HW)
        if a.config != 4 and a.parity_sample:
            n = a.batch if a.parity_sample < 0 else min(a.parity_sample, a.batch)
            threads = cpu["threads"]
            t0 = time.perf_counter()
            o_n, o_f, o_h, o_q = oracle_threaded(ox, batches[j0][:n], RL, od, threads)
            dt = time.perf_counter() - t0
            bad, first = compare_batch(g_n[:n], g_f[:n], g_o[:n], g_h, o_n, o_f, o_h)
            gq = int(outs[j0]["c"][2].item())
            result["parity_full" if n == a.batch else "parity_sample"] = {
                "reads": n, "mismatching_reads": bad, "first_mismatch": first,
                "fields": f"n_aln, splice-fallback flag, every {'hsa_aln64_t' if wide else 'bwt_aln1_t'} field of "
                          "every hit, hit order",
                "against": "oracle (C restatement" + (", 64-bit intervals: liboracle64.so)" if wide else ")"),
                "rank_queries_gpu": gq if n == a.batch else None, "rank_queries_oracle": int(o_q)}
            log(f"[bench] parity: {n} reads, {bad} differ from the CPU restatement; rank queries GPU "
                f"{gq} vs oracle {int(o_q)} ({threads} threads, {dt:.1f} s)")
            if a.cpu_sample:
                n1 = min(a.cpu_sample, a.batch)
                rs = batches[(a.warmup + 1) % nd][-n1:]
                t1 = time.perf_counter()
                ox.cal_sa_reg_gap(np.full(n1, RL, np.uint32), rs.reshape(-1), Opt.from_dict(od))
                dt1 = time.perf_counter() - t1
                share = (f"{threads} threads: the box's CPU share for one GPU (worker pools are capped at 16 per GPU; "
                         f"{cpu['physical_cores']} physical cores are visible)")
                result["cpu_baseline"] = {
                    "value": round(n / dt, 1), "unit": "reads/s", "cores": threads, "kind": "port",
                    "value_1core": round(n1 / dt1, 1), "cpu_model": cpu["model"],
                    "physical_cores_visible": cpu["physical_cores"], "affinity_cpus": cpu["affinity"],
                    "sample": f"the whole timed batch ({n} reads) on the bwa_cal_sa_reg_gap restatement (gcc -O3), "
                              f"{share}, disjoint chunks, {dt:.1f} s (the parity run above); 1 thread: {n1} reads in "
                              f"{dt1:.1f} s"}
        if a.config == 4 and a.parity_sample:
            n = 4000 if a.parity_sample < 0 else min(a.parity_sample, a.batch)
            r0 = batches[a.warmup % nd][:n]
            o_n, o_f, o_h, _ = ox.cal_sa_reg_gap(np.full(n, RL, np.uint32), r0.reshape(-1), Opt.from_dict(od))
            oo = np.concatenate([[0], np.cumsum(o_n)])
            bad = 0
            for i in range(n):
                if (g_f[i] & 1) != (o_f[i] & 1) or g_n[i] != o_n[i] or \
                        not np.array_equal(g_h[g_o[i]:g_o[i] + g_n[i]], o_h[oo[i]:oo[i + 1]]):
                    bad += 1
            result["parity_sample"] = {"reads": n, "mismatching_reads": bad, "against": "oracle (C restatement)"}
            log(f"[bench] parity sample: {n} reads, {bad} differ from the CPU restatement")
    # the reference's own CPU path, and the drop-in end to end (rank 0, configs 2-4; config
    # 4's end to end runs the whole splice path of its fallback reads)
    # With N ranks it runs after the gather on rank 0, over the CPU share of all N ranks
    # (the other ranks wait on the rendezvous store meanwhile, without spinning a core);
    # the drop-in end to end needs a GPU of its own and runs at N = 1 only.
    if ref_legs:
        procs = ref_procs
        j0 = a.warmup % nd
        if world == 1 and a.e2e_reads > 0:
            # the drop-in end to end is a second process on this GPU: this one's search
            # scratch (tens of GB for the gapped regimes) goes back first
            for h in handles:
                if getattr(h, "h", None):
                    h.release_scratch()
            torch.cuda.empty_cache()
        # -G: the reference starts in the steady state of a process's later batches, the
        # state of the timed batches (GAPE cleared in the caller's block)
        opt_args = ["-n", "4", "-o", str(max_gapo), "-G"]
        try:
            legs = reference_legs(T, res, extra, batches[j0], opt_args, min(a.ref_sample, a.batch), procs,
                                  min(a.e2e_reads, a.batch) if world == 1 else 0)
        except Exception as ex:                       # reported, never fatal: a baseline
            legs = {"error": f"{type(ex).__name__}: {ex}"[:400]}
            log(f"[bench] reference legs failed: {legs['error']}")
        if "reference" in legs:
            port = result.get("cpu_baseline")
            result["cpu_baseline"] = dict(legs["reference"])
            if port:
                result["cpu_baseline"].update(cpu_model=port.get("cpu_model"),
                                              physical_cores_visible=port.get("physical_cores_visible"),
                                              port={k: port.get(k) for k in ("value", "cores", "value_1core", "sample")})
                pc = port.get("physical_cores_visible")
                if pc and world == 1:
                    # BASELINE.md §3 prices the reference on every core of the host; the
                    # box gives one GPU's job 16 CPU processes at most, so the whole-host
                    # figure is the measured per-core rate times the physical cores: an
                    # upper bound (128 processes share the memory system the per-core
                    # rate was measured without)
                    v1 = legs["reference"]["value_1core"]
                    result["cpu_baseline"]["all_physical_cores"] = {
                        "value": round(v1 * pc, 1), "cores": pc, "measured": False,
                        "how": f"value_1core ({v1:.0f} reads/s, median of {procs} concurrent processes) x {pc} "
                               "physical cores; linear scaling assumed, so an upper bound; not run: one GPU's job "
                               "may use 16 CPU processes on the box"}
            if legs.get("dropin_e2e"):
                result["dropin_e2e"] = legs["dropin_e2e"]
            if a.config == 4 and legs.get("ref0"):
                # the timed step's results (main path, then the splice path on the device)
                # against the reference's own bwa_cal_sa_reg_gap on the same reads
                r_n, r_h = legs["ref0"]
                o = outs[j0]
                g_n, g_f, g_o = o["n"].cpu().numpy(), o["f"].cpu().numpy(), o["o"].cpu().numpy()
                g_h = o["h"].cpu().numpy().view(np.uint32).reshape(-1, HW)
                g_r = o["res"].cpu().numpy().view(np.uint32).reshape(-1, _lib.SP_RES_WORDS)
                ro = np.concatenate([[0], np.cumsum(np.maximum(r_n, 0).astype(np.int64))])
                bad, na_, spl = [], 0, 0
                for i in range(len(r_n)):
                    if g_n[i] > 0:
                        got = g_h[g_o[i]:g_o[i] + g_n[i]]
                    elif g_f[i] & 1:
                        if g_r[i, 0] != 0:
                            na_ += 1
                            continue
                        got = g_r[i, 2:2 + 9 * g_r[i, 1]].reshape(-1, 9)
                        spl += g_r[i, 1] > 0
                    else:
                        got = np.zeros((0, 9), np.uint32)
                    if len(got) != max(r_n[i], 0) or not np.array_equal(got, r_h[ro[i]:ro[i + 1]]):
                        bad.append(i)
                result["parity_reference"] = {
                    "reads": len(r_n), "mismatching_reads": len(bad), "first_mismatch": bad[0] if bad else None,
                    "not_answered_on_device": na_, "spliced_reads": int(spl),
                    "against": "the reference's own bwa_cal_sa_reg_gap (oracle/_ref/ref_probe -G, steady-state "
                               "batch) on the first reads of the timed read set: n_aln and every bwt_aln1_t word of "
                               "every hit, main path and splice path"}
                log(f"[bench] the timed step vs the reference: {len(r_n)} reads, {len(bad)} differ ({spl} spliced, "
                    f"{na_} not answered on the device)")

        else:
            result["reference_legs"] = legs
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        store = dist.distributed_c10d._get_default_store()
        if rank == 0:
            store.set("hsa_bench_done", "1")
        else:
            store.wait(["hsa_bench_done"], timedelta(minutes=30))
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
