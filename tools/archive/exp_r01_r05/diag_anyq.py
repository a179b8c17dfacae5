"""Diagnostic: rank-query counts of the k_search / k_search_any split on long1500_n8o1."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import hsa_amd  # noqa
import numpy as np
from test_gpu_parity import _device_run
got, (e_n, e_f, e_h, st) = _device_run("long1500_n8o1")
print("mixed: gpu Q", int(got["c"][2]), "pops", int(got["c"][4]), "oracle", int(st[0]), int(st[1]), "c", got["c"].tolist())
os.environ["HSA_FORCE_ANY"] = "1"
got, (e_n, e_f, e_h, st) = _device_run("long1500_n8o1")
print("forced any: gpu Q", int(got["c"][2]), "pops", int(got["c"][4]), "oracle", int(st[0]), int(st[1]), "c", got["c"].tolist())
for case in ("gap100_o2e60", "gap100_o15", "tiny_gap100_n4o1"):
    got, (e_n, e_f, e_h, st) = _device_run(case)
    print(case, "forced any: gpu Q", int(got["c"][2]), "pops", int(got["c"][4]), "oracle", int(st[0]), int(st[1]))
del os.environ["HSA_FORCE_ANY"]
got, (e_n, e_f, e_h, st) = _device_run("tiny_gap100_n4o1")
print("tiny_gap100_n4o1 fast: gpu Q", int(got["c"][2]), "pops", int(got["c"][4]), "oracle", int(st[0]), int(st[1]))
