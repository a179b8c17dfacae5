"""Diagnostic: per-read pops of k_search_any vs the oracle on long1500_n8o1."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import hsa_amd  # noqa
import numpy as np
import torch
from golden_io import INDEX, load_case, parse_opts
from hsa_amd import index_io
from hsa_amd._lib import JOB_DTYPE, DeviceBatch, GapOpt, pad_codes, regime_of
from oracle_ctypes import Opt, OracleIndex, default_opt
from test_gpu_parity import gpu_index
os.environ["HSA_FORCE_ANY"] = "1"
g = load_case("long1500_n8o1")
fwd, rev = index_io.read_index(INDEX["tiny"])
ox = OracleIndex(fwd, rev)
ix = gpu_index("tiny")
od = parse_opts(g["args"], default_opt())
od["mode"] &= ~0x01
o = GapOpt.from_dict(od)
n_stacks = (o.max_diff + 1) * o.s_mm + (o.max_gapo + 1) * o.s_gapo + (o.max_gape + 1) * o.s_gape
rg = regime_of(od, n_stacks, o.max_diff)
offs = np.concatenate([[0], np.cumsum(g["lens"].astype(np.int64))])
nd = 0
for r in range(len(g["lens"])):
    sq = g["codes"][offs[r]:offs[r + 1]]
    if int((sq > 3).sum()) > od["max_diff"]:
        continue
    L = len(sq)
    e = ox.cal_sa_reg_gap(np.array([L], np.uint32), sq, Opt.from_dict(od))
    jobs = np.zeros(1, JOB_DTYPE)
    jobs["len"] = L
    jobs["max_diff"] = o.max_diff
    jobs["seed_len"] = o.seed_len if L > o.seed_len else 0x7FFFFFFF
    d_jobs = torch.from_numpy(jobs.view(np.uint8).copy()).cuda()
    d_codes = torch.from_numpy(pad_codes(sq)).cuda()
    t = dict(n=torch.zeros(1, dtype=torch.int32, device="cuda"), f=torch.zeros(1, dtype=torch.int32, device="cuda"),
             o=torch.zeros(1, dtype=torch.int64, device="cuda"), h=torch.zeros(64 * 9, dtype=torch.int32, device="cuda"),
             c=torch.zeros(16, dtype=torch.int64, device="cuda"))
    b = DeviceBatch(d_jobs=d_jobs.data_ptr(), n_jobs=1, d_codes=d_codes.data_ptr(), d_n_aln=t["n"].data_ptr(),
                    d_flags=t["f"].data_ptr(), d_hit_off=t["o"].data_ptr(), d_hits=t["h"].data_ptr(), hit_cap=64,
                    d_counters=t["c"].data_ptr(), max_len=L, max_seed=o.seed_len)
    ix.search_device([rg], b)
    torch.cuda.synchronize()
    c = t["c"].cpu().numpy()
    if int(c[4]) != int(e[3][1]) or int(c[2]) != int(e[3][0]):
        nd += 1
        if nd <= 12:
            print(f"read {r} len {L} nN {int((sq > 3).sum())} n_aln gpu {int(t['n'][0])} oracle {int(e[0][0])} "
                  f"flag {int(t['f'][0])}/{int(e[1][0])} pops gpu {int(c[4])} oracle {int(e[3][1])} Q gpu {int(c[2])} "
                  f"oracle {int(e[3][0])} widthQ {int(c[7])}")
print("differing reads", nd)
