"""BASELINE config 5 at its stated size: a 15 000 000 003 bp plant-scale text (24
records, the bench's genome), far past the 2^32 characters the reference's 32-bit
bwtint_t can index (2BWT-Interface.h:26).

Both BWTs are built on the device (hsa_build_bwt_device64), the 64-bit index is made
over them (hsa_index_create_device64) and 20 000 x 250 bp reads from the whole text
-- 0-4 substitutions, half reverse-complemented, 1 read in 50 with an N -- are
searched with -n 4 -o 0 by the same instantiation the config-5 bench times (64-bit
intervals, 4-bit pruning rows, hsa_search_device64).  Every hsa_aln64_t field of
every hit, the splice-fallback flags, the rank-query count and the pop count equal
the 64-bit restatement's (liboracle64.so, pinned against the reference's golden
vectors below 2^32 in tests/test_oracle.py); hits with SA bounds past 2^32 occur.
No reference output exists at this size: parity is against the restatement only.

Cost: about 30 s of device build, 40 GB of host memory for the restatement's
index, a few seconds of restatement search."""
import os

import numpy as np
import pytest

from test_gpu_wide import _check_past_2_32

pytestmark = pytest.mark.gpu

T5 = 15_000_000_003      # bench.py GENOME5_T
SEED5 = 1234             # bench.py GENOME_SEED
RECORDS5 = 24            # bench.py RECORDS


@pytest.fixture(scope="module")
def plant_index():
    import ctypes as C

    import torch
    from hsa_amd import synth
    from hsa_amd._lib import GpuIndex, check, lib
    from oracle_ctypes import OracleIndex64
    free, total = torch.cuda.mem_get_info()
    if total < 200 * 2**30:
        pytest.skip(f"config 5 needs an MI355X-sized HBM ({total / 2**30:.0f} GiB visible)")
    nw = (T5 + 15) // 16
    text = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
    check(lib().hsa_synth_genome_device(0, T5, SEED5, text.data_ptr()))
    res = []
    for rev in (0, 1):
        bw = torch.zeros(nw + 8, dtype=torch.int32, device="cuda")
        isa0 = C.c_uint64()
        Cc = np.zeros(5, np.uint64)
        check(lib().hsa_build_bwt_device64(0, T5, text.data_ptr(), rev, bw.data_ptr(), C.byref(isa0), Cc))
        res.append((bw, int(isa0.value), Cc))
    del text
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    assert int(res[0][2][4]) == T5 and int(res[1][2][4]) == T5
    gi = GpuIndex.from_device_codes64(T5, res[0][1], res[0][2], res[0][0].data_ptr(), T5, res[1][1], res[1][2],
                                      res[1][0].data_ptr())
    host = [r[0][:nw].cpu().numpy().view(np.uint32) for r in res]
    meta = [(r[1], r[2]) for r in res]
    del res
    torch.cuda.empty_cache()
    ox = OracleIndex64(T5, *meta[0], host[0], T5, *meta[1], host[1])
    del host
    genome = synth.PackedGenome(T5, SEED5)
    yield gi, ox, genome
    del ox
    gi.close()


@pytest.mark.timeout(900)
def test_config5_full_size_matches_oracle(plant_index, monkeypatch, capfd):
    from hsa_amd import synth
    from oracle_ctypes import default_opt
    monkeypatch.setenv("HSA_VERBOSE", "1")
    monkeypatch.delenv("HSA_WFMT", raising=False)
    gi, ox, genome = plant_index
    recs = synth.record_layout(T5, RECORDS5)
    reads, _ = synth.make_reads(genome, recs, 20_000, 250, 8 * 1_000_000 + 5, max_mm=4)
    reads = reads.copy()
    rng = np.random.default_rng(55)
    for r in range(0, len(reads), 50):
        reads[r, int(rng.integers(0, 250))] = 4
    od = default_opt()
    od.update(max_diff=4, fnr=-1.0, max_gapo=0)
    od["mode"] &= ~0x01
    e_n = _check_past_2_32(gi, ox, reads, od)
    err = capfd.readouterr().err
    assert "4-bit rows" in err, "config 5's 4-bit-row instantiation was not the one that ran"
    assert (e_n > 0).mean() > 0.9
    if os.environ.get("HSA_TEST_LOG"):
        print(f"config 5 full size: {len(reads)} reads, {int((e_n > 0).sum())} with hits")
