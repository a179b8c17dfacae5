"""The drop-in host C (bwtaln_gpu.c, bwtgap_gpu.c) and the oracle built with
AddressSanitizer + UndefinedBehaviorSanitizer and run on CPU.  The
core's GPU calls are answered by the restatement (tests/san/san_core.c, test
infrastructure only); the hits of bwa_cal_sa_reg_gap -- batch loop, option-regime
switch, filters, hit copying -- must equal the reference's golden vectors, and the
splice path's bwt_match_gap must answer from the prefetch table (tests/san/san_main.c)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from golden_io import INDEX, load_case, parse_opts, split_hits
from oracle_ctypes import Opt, default_opt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["tests/san/san_main.c", "tests/san/san_core.c", "hsa_amd/csrc/bwtaln_gpu.c", "hsa_amd/csrc/bwtgap_gpu.c",
        "oracle/hsa_oracle.c"]
FLAGS = ["-O1", "-g", "-std=gnu11", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
         "-fno-omit-frame-pointer"]


@pytest.fixture(scope="module")
def san_bin(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    out = str(tmp_path_factory.mktemp("san") / "san_main")
    r = subprocess.run(["gcc", *FLAGS, *[os.path.join(ROOT, s) for s in SRCS], "-lm", "-lpthread", "-o", out],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


@pytest.mark.parametrize("name,slots", [("tiny_gap100_n4o1_b400", 1), ("tiny_edge_n3o1e3L", 1),
                                        ("rep_gap60_default", 2), ("tiny_opts_seed", 1), ("tiny_mm100_n4o0", 3)])
def test_dropin_host_c_under_sanitizers(san_bin, tmp_path, name, slots):
    g = load_case(name)
    n = len(g["lens"])
    (tmp_path / "reads.bin").write_bytes(np.uint32(n).tobytes() + g["lens"].astype(np.uint32).tobytes()
                                         + g["codes"].astype(np.uint8).tobytes())
    (tmp_path / "opt.bin").write_bytes(bytes(Opt.from_dict(parse_opts(g["args"], default_opt()))))
    env = dict(os.environ, HSA_GPU_DEVICES=str(slots),
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([san_bin, INDEX[g["index"]], str(tmp_path / "reads.bin"), str(tmp_path / "opt.bin"),
                        str(g["batch"]), str(tmp_path / "out.bin")], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
    raw = np.frombuffer((tmp_path / "out.bin").read_bytes(), np.uint32)
    got, i = [], 0
    for _ in range(n):
        na = int(raw[i].view(np.int32))
        i += 1
        got.append(raw[i:i + 9 * max(na, 0)].reshape(-1, 9))
        i += 9 * max(na, 0)
    assert i == len(raw)
    exp_splice = (g["flags"] & 1).astype(bool)
    exp = split_hits(g["n_aln"], g["hits"])
    bad = [k for k in range(n) if not exp_splice[k] and not np.array_equal(got[k], exp[k])]
    assert not bad, f"{len(bad)} reads differ; first {bad[0]}: {got[bad[0]]} vs {exp[bad[0]]}"
    if exp_splice.any():
        assert "answered from the prefetch table" in r.stderr
