"""hsa_amd -- MI355X-native core for HSA's inexact-alignment path.

The product is libhsa_gpu.so (HIP kernels for gfx950 + the C ABI declared in
include/hsa_gpu.h and the reference-compatible entry points of
include/hsa_bwtaln.h).  This package holds its Python binding (`_lib`), the
index file readers/writers (`index_io`) and the synthetic data generators
(`synth`).  Nothing here computes alignments on the CPU.
"""
from . import index_io, synth  # noqa: F401

__all__ = ["index_io", "synth", "lib"]


def lib():
    from . import _lib
    return _lib
