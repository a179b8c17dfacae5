"""Config 4 at hg19 size (BASELINE configs[3]): 20 000 x 150 bp spliced
reads (exon, GT..AG intron of 200-5000 bp, exon; half reverse-complemented) against the
device-built 3 000 000 005 bp index, through the whole drop-in -- the reference's own
driver with every entry point of ours (oracle/_ref/ref_probe_gpu: bwa_cal_sa_reg_gap, the
splice path on the device, the host's bwt_splice_match for what the kernel hands back) --
against the reference itself (oracle/_ref/ref_probe, compiled from its sources) on the
same index files, in the same batches: n_aln and every bwt_aln1_t word of every hit,
splice-path hits included, in order.

Both runs use batches of N_READS / 16 reads (`-B`; 1 250 by default): the reference runs 16 processes of one
batch each, so a batch's option regimes (the first fallback read switches aux->opt,
bwtaln.c:363) are the same on both sides."""
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = os.path.join(ROOT, "oracle", "_ref")

pytestmark = pytest.mark.gpu

# HSA_C4_READS scales the run (the round-6 check ran 200 000: profiles/r06_config4_200k_dropin.log);
# the reference always runs as 16 processes of one batch each
N_READS = int(os.environ.get("HSA_C4_READS", "20000")) // 16 * 16
CHUNK = N_READS // 16


@pytest.mark.skipif(not (os.path.exists(os.path.join(REF, "ref_probe")) and
                         os.path.exists(os.path.join(REF, "ref_probe_gpu"))),
                    reason="oracle/_ref/ref_probe(_gpu) not built (make -C oracle)")
def test_config4_hg19_dropin_matches_reference():
    import torch

    import bench
    from hsa_amd import synth
    T = bench.GENOME_T
    gi, res, extra = bench.build_index(T, bench.GENOME_SEED, torch.cuda.current_device(), with_files=True)
    gi.close()
    genome = synth.PackedGenome(T, bench.GENOME_SEED)
    recs = synth.record_layout(T, bench.RECORDS)
    reads, _ = synth.make_spliced_reads(genome, recs, N_READS, 150, 7 * 1_000_000 + 91)
    d = tempfile.mkdtemp(prefix="hsa_c4_")
    try:
        prefix = bench.reference_files(d, T, res, extra)
        del res, extra
        torch.cuda.empty_cache()
        opt = ["-n", "4", "-o", "1"]
        jobs = []
        for k in range(N_READS // CHUNK):
            rb = os.path.join(d, f"r{k}.bin")
            bench.write_reads_bin(rb, reads[k * CHUNK:(k + 1) * CHUNK])
            jobs.append(subprocess.Popen([os.path.join(REF, "ref_probe"), "aln", prefix, rb, os.path.join(d, f"o{k}.bin"),
                                          *opt, "-B", str(CHUNK)], stdout=subprocess.PIPE, stderr=subprocess.PIPE))
        rb = os.path.join(d, "all.bin")
        bench.write_reads_bin(rb, reads)
        g = subprocess.run([os.path.join(REF, "ref_probe_gpu"), "aln", prefix, rb, os.path.join(d, "g.bin"), *opt, "-B",
                            str(CHUNK)], capture_output=True, timeout=900, env=dict(os.environ, HSA_VERBOSE="1"))
        assert g.returncode == 0, g.stderr.decode()[-3000:]
        for j in jobs:
            _, e = j.communicate(timeout=900)
            assert j.returncode == 0, e.decode()[-2000:]
        r_n, r_h = [], []
        for k in range(N_READS // CHUNK):
            n, h = bench.read_probe_out(os.path.join(d, f"o{k}.bin"))
            r_n.append(n)
            r_h.append(h)
        r_n, r_h = np.concatenate(r_n), np.concatenate(r_h)
        g_n, g_h = bench.read_probe_out(os.path.join(d, "g.bin"))
    finally:
        shutil.rmtree(d, ignore_errors=True)
    assert len(g_n) == len(r_n) == N_READS
    go = np.concatenate([[0], np.cumsum(np.maximum(g_n, 0).astype(np.int64))])
    ro = np.concatenate([[0], np.cumsum(np.maximum(r_n, 0).astype(np.int64))])
    bad = [i for i in range(N_READS) if g_n[i] != r_n[i] or not np.array_equal(g_h[go[i]:go[i + 1]], r_h[ro[i]:ro[i + 1]])]
    spliced = int(sum(1 for i in range(N_READS) if r_n[i] > 0 and (r_h[ro[i], 5] & 0x3FFFFFFF) == 4))
    log = g.stderr.decode()
    kern = [ln for ln in log.splitlines() if ln.startswith("[hsa] splice kernel:") and "reads," in ln]
    print(f"config 4 at hg19 size: {N_READS} reads, {int((r_n > 0).sum())} mapped, {spliced} with spliced hits; "
          f"{len(bad)} differ; {kern[-1] if kern else 'no splice kernel line'}")
    assert not bad, f"{len(bad)} of {N_READS} reads differ from the reference (first {bad[:5]})"
    assert spliced > N_READS // 4
    assert kern, "the drop-in did not run the splice kernel"
