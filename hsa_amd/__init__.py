"""hsa_amd -- MI355X-native core for HSA's inexact-alignment path.

The product is libhsa_gpu.so (HIP kernels for gfx950 + the C ABI declared in
include/hsa_gpu.h and the reference-compatible entry points of
include/hsa_bwtaln.h).  This package holds its Python binding (`_lib`), the
index file readers/writers (`index_io`) and the synthetic data generators
(`synth`).  Nothing here computes alignments on the CPU.
"""
import os as _os

from . import index_io, synth  # noqa: F401

# Load the HIP library before anything imports torch (see _lib._check_runtime).
if _os.path.exists(_os.path.join(_os.path.dirname(_os.path.abspath(__file__)),
                                 _os.environ.get("HSA_GPU_LIB", "libhsa_gpu.so"))):
    from . import _lib as _l
    _l.lib()

__all__ = ["index_io", "synth", "lib"]


def lib():
    from . import _lib
    return _lib
