"""CPU-side checks of the C ABI: the library loads and exports every declared symbol,
and the reference struct layouts match the compiled reference's sizes."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\([^;{]*\)\s*(?:__attribute__\(\(weak\)\))?\s*;", txt)
    return {n for n in names if n not in ("bwt_splice_match", "sizeof")}


def test_library_exports_every_declared_symbol():
    from hsa_amd import _lib
    assert os.path.exists(_lib.LIB_PATH), "build libhsa_gpu.so first (python -c 'import __graft_entry__ as g; g.build()')"
    L = ctypes.CDLL(_lib.LIB_PATH)
    want = declared("hsa_gpu.h") | declared("hsa_bwtaln.h")
    assert want >= {"hsa_search_batch", "bwa_cal_sa_reg_gap", "hsa_index_create"}
    missing = [n for n in sorted(want) if not hasattr(L, n)]
    assert not missing, missing
    assert set(_lib.EXPORTS) >= want


def test_no_gpu_fails_loudly():
    """Without a device the product refuses to run (no CPU fallback)."""
    from hsa_amd import _lib
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    import numpy as np
    from golden_io import INDEX
    from hsa_amd import index_io
    with pytest.raises(_lib.HsaError):
        _lib.GpuIndex(*index_io.read_index(INDEX["tiny"]))


def test_release_scratch_rejects_a_null_handle():
    """hsa_index_release_scratch checks its handle before any HIP call."""
    from hsa_amd import _lib
    L = _lib.lib()
    assert L.hsa_index_release_scratch(None) == -2            # HSA_E_ARG (include/hsa_gpu.h)
    assert b"null" in L.hsa_last_error()


def test_struct_sizes_match_reference():
    probe = os.path.join(ROOT, "oracle", "_ref", "ref_probe")
    if not os.path.exists(probe):
        pytest.skip("compiled reference not present")
    from golden_io import INDEX
    out = subprocess.run([probe, "meta", INDEX["tiny"]], capture_output=True, text=True, check=True).stdout
    m = dict(re.findall(r"(\w+)=(\d+)", out.splitlines()[-1]))
    assert m == {"bwt_aln1_t": "36", "gap_opt_t": "64", "bwa_seq_t": "208", "bwt_aux_t": "96", "BWT": "128",
                 "Idx2BWT": "544", "HSP": "48"}
