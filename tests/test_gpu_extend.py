"""The splice path's seed extensions on the GPU (hsa_extend_batch, hsa_amd/csrc/
hsa_extend.hip): every bwt_extend_backward / bwt_extend_foreward call the compiled
reference made on the drop-in splice read set (tests/golden/extcap_*.npz, recorded by
oracle/ref_extcap.c), run as ONE batch -- return value, max_pos and every bwt_aln1_t
field must equal the reference's.  Calls of different option blocks become regimes of
the same launch."""
import numpy as np
import pytest

from golden_io import EXTCAP_CASES, INDEX, load_extcap

pytestmark = pytest.mark.gpu


def ext_batch(name):
    from hsa_amd._lib import EXT_DTYPE, Regime
    calls = list(load_extcap(name))
    keys, regimes = {}, []
    jobs = np.zeros(len(calls), EXT_DTYPE)
    codes, bids = [], []
    off = 0
    for j, c in enumerate(calls):
        o = c["opt"].view(np.int32)      # gap_opt_t: s_mm s_gapo s_gape mode ies mdo me fnr max_diff gapo gape ...
        key = (tuple(int(x) for x in o[[0, 1, 2, 3, 4, 5, 6, 8, 9, 10]]), c["n_stacks"])
        if key not in keys:
            keys[key] = len(regimes)
            regimes.append(Regime(s_mm=o[0], s_gapo=o[1], s_gape=o[2], mode=o[3], indel_end_skip=o[4],
                                  max_del_occ=o[5], max_entries=o[6], max_gapo=o[9], max_gape=o[10],
                                  max_seed_diff=o[11], max_top2=o[14], n_stacks=c["n_stacks"], max_diff=o[8]))
        jobs[j] = (c["dir"], c["len"], c["max_pos"], keys[key], c["lo"], len(c["seq"]), off, c["aln_in"], 0)
        codes.append(c["seq"])
        bids.append(c["bid"])
        off += len(c["seq"])
    return calls, regimes, jobs, np.concatenate(codes), np.concatenate(bids)


@pytest.mark.parametrize("name", EXTCAP_CASES)
def test_extension_batch_matches_reference(name):
    from hsa_amd import _lib, index_io
    fwd, rev = index_io.read_index(INDEX["tiny"])
    gi = _lib.GpuIndex(fwd, rev, device=0)
    calls, regimes, jobs, codes, bids = ext_batch(name)
    ret, mp, aln = gi.extend(regimes, jobs, codes, bids)
    bad = [j for j, c in enumerate(calls)
           if ret[j] != c["ret"] or mp[j] != c["max_pos_out"] or not np.array_equal(aln[j], c["aln_out"])]
    assert len(calls) > 3000
    assert not bad, (f"{len(bad)} of {len(calls)} extensions differ; first {bad[0]}: "
                     f"{ret[bad[0]], mp[bad[0]], aln[bad[0]]} vs {calls[bad[0]]['ret'], calls[bad[0]]['max_pos_out'], calls[bad[0]]['aln_out']}")


@pytest.mark.parametrize("budget", [3, 40])
def test_sliced_extensions_match_reference(budget):
    """hsa_extend_sliced: the same calls in slices of `budget` pops -- each launch runs
    the unfinished calls from the state their slot kept, new calls start in freed slots
    -- must end with the reference's results."""
    from hsa_amd import _lib, index_io
    fwd, rev = index_io.read_index(INDEX["tiny"])
    gi = _lib.GpuIndex(fwd, rev, device=0)
    calls, regimes, jobs, codes, bids = ext_batch("extcap_n4o1")
    n_slots = 512
    todo = list(range(len(calls)))
    slot_of, resume, free = {}, {}, list(range(n_slots))
    res = {}
    launches = 0
    while todo or slot_of:
        while todo and free:
            j = todo.pop()
            slot_of[j] = free.pop()
            resume[j] = 0
        act = sorted(slot_of)
        ret, mp, aln = gi.extend_sliced(regimes, jobs[act], codes, bids, [slot_of[j] for j in act],
                                        [resume[j] for j in act], n_slots, budget)
        launches += 1
        for x, j in enumerate(act):
            if ret[x] == -999:
                resume[j] = 1
                continue
            res[j] = (int(ret[x]), int(mp[x]), aln[x].copy())
            free.append(slot_of.pop(j))
    bad = [j for j, c in enumerate(calls) if res[j][0] != c["ret"] or res[j][1] != c["max_pos_out"]
           or not np.array_equal(res[j][2], c["aln_out"])]
    assert launches > len(calls) // n_slots + 1          # slices really happened
    assert not bad, f"{len(bad)} of {len(calls)} differ; first {bad[0]}"
