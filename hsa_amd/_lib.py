"""ctypes binding of libhsa_gpu.so (the MI355X search core and its drop-in C ABI).

The library is built in-tree (hsa_amd/libhsa_gpu.so, `make -C hsa_amd/csrc`).
There is no fallback: if the library or a GPU is missing every call raises.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# HSA_GPU_LIB selects another in-tree build of the same library (A/B experiments).
LIB_PATH = os.path.join(HERE, os.environ.get("HSA_GPU_LIB", "libhsa_gpu.so"))

HSA_F_FALLBACK = 1
HSA_F_OVERFLOW = 2
HSA_RF_NFILTER = 0x10
HSA_RF_POLYAT = 0x20

EXPORTS = [  # every symbol include/hsa_gpu.h and include/hsa_bwtaln.h declare
    "hsa_device_count", "hsa_last_error", "hsa_index_create", "hsa_index_create_device", "hsa_index_free",
    "hsa_index_release_scratch",
    "hsa_index_bytes", "hsa_index_device", "hsa_occ4_batch", "hsa_step_batch", "hsa_width_batch",
    "hsa_search_batch", "hsa_search_device", "hsa_configure", "hsa_free", "hsa_synth_genome_device",
    "hsa_build_bwt_device", "bwa_cal_sa_reg_gap", "hsa_gpu_attach", "hsa_gpu_detach", "hsa_gpu_set_devices",
    "hsa_cal_sa_reg_gap_flat", "hsa_index_stream", "hsa_probe_gather", "hsa_last_pass_ms",
    "hsa_index_set_sa", "hsa_sa_position_batch", "hsa_sa_position_device", "hsa_match_gap_batch",
    "bwt_match_gap", "bwt_match_gap_batch", "hsa_splice_seeds_device", "hsa_pass_times",
    "hsa_cal_sa_reg_gap_multi", "hsa_index_create_device64", "hsa_index_is64", "hsa_occ4_batch64",
    "hsa_search_device64", "hsa_build_bwt_device64", "bwa_cal_pac_pos", "generate_sam_se_core",
    "hsa_build_bwt_index_device", "hsa_extend_batch", "bwt_extend_foreward", "bwt_extend_backward",
    "hsa_width0_batch", "bwt_cal_width", "hsa_extend_sliced", "hsa_index_trie",
    "hsa_index_clone", "hsa_splice_prefetch_batch", "hsa_index_set_text", "hsa_splice_match_batch",
    "hsa_splice_device",
]
SP_RES_WORDS = 20  # hsa_splice_match_batch's per-read answer (include/hsa_gpu.h)
ALN64_WORDS = 14   # hsa_aln64_t (include/hsa_gpu.h)


class HsaError(RuntimeError):
    pass


CODES_PAD = 16   # hsa_search_device reads a read's codes in aligned 16-byte loads


def pad_codes(codes) -> np.ndarray:
    """Read codes followed by the padding the device path may read past the last
    read (include/hsa_gpu.h, hsa_device_batch_t.d_codes)."""
    c = np.ascontiguousarray(codes, np.uint8).reshape(-1)
    return np.concatenate([c, np.zeros(4 * CODES_PAD, np.uint8)])


class GapOpt(C.Structure):
    """gap_opt_t (bwtaln.h:133-143)."""
    _fields_ = [("s_mm", C.c_int), ("s_gapo", C.c_int), ("s_gape", C.c_int), ("mode", C.c_int),
                ("indel_end_skip", C.c_int), ("max_del_occ", C.c_int), ("max_entries", C.c_int),
                ("fnr", C.c_float), ("max_diff", C.c_int), ("max_gapo", C.c_int), ("max_gape", C.c_int),
                ("max_seed_diff", C.c_int), ("seed_len", C.c_int), ("n_threads", C.c_int),
                ("max_top2", C.c_int), ("trim_qual", C.c_int)]

    @classmethod
    def default(cls):
        """gap_init_opt (bwtaln.c:21-44)."""
        return cls(s_mm=3, s_gapo=11, s_gape=4, mode=0x03, indel_end_skip=5, max_del_occ=10,
                   max_entries=2000000, fnr=0.04, max_diff=-1, max_gapo=1, max_gape=6,
                   max_seed_diff=2, seed_len=32, n_threads=1, max_top2=30, trim_qual=0)

    @classmethod
    def from_dict(cls, d):
        o = cls()
        for k, _ in cls._fields_:
            setattr(o, k, d[k])
        return o

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Regime(C.Structure):
    _fields_ = [(k, C.c_int32) for k in ("s_mm", "s_gapo", "s_gape", "mode", "indel_end_skip", "max_del_occ",
                                         "max_entries", "max_gapo", "max_gape", "max_seed_diff", "max_top2",
                                         "n_stacks", "max_diff")]


JOB_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("max_diff", "<i4"), ("seed_len", "<i4"),
                      ("regime", "<i4")])
# hsa_mg_job_t (include/hsa_gpu.h): one direct bwt_match_gap call's widths and strand
MG_DTYPE = np.dtype([("wb_off", "<u8"), ("ws_off", "<u8"), ("strand", "<i4"), ("seed", "<i4")])
SEED_NONE, SEED_OWN, SEED_ALIAS = 0, 1, 2
# hsa_ext_job_t (include/hsa_gpu.h): one seed extension of the splice path
EXT_DTYPE = np.dtype([("dir", "<i4"), ("len", "<i4"), ("max_pos", "<i4"), ("regime", "<i4"), ("lo", "<i4"),
                      ("n", "<i4"), ("off", "<u8"), ("aln", "<u4", (9,)), ("pad", "<u4")])
assert EXT_DTYPE.itemsize == 72


def regime_of(opt: dict, n_stacks: int, max_diff: int) -> "Regime":
    """The fields of one option block bwt_match_gap reads (bwtaln_gpu.c hsa_regime_of)."""
    mode = opt["mode"] & (0x01 | 0x04 | 0x10)
    if opt["max_gapo"] == 0:
        mode &= ~(0x01 | 0x04)
    return Regime(s_mm=opt["s_mm"], s_gapo=opt["s_gapo"], s_gape=opt["s_gape"], mode=mode,
                  indel_end_skip=opt["indel_end_skip"], max_del_occ=opt["max_del_occ"],
                  max_entries=opt["max_entries"], max_gapo=opt["max_gapo"], max_gape=opt["max_gape"],
                  max_seed_diff=opt["max_seed_diff"], max_top2=opt["max_top2"], n_stacks=n_stacks,
                  max_diff=max_diff)


class Stats(C.Structure):
    _fields_ = [("rank_queries", C.c_uint64), ("blocks_loaded", C.c_uint64), ("pops", C.c_uint64),
                ("overflow_reruns", C.c_uint64), ("kernel_ms", C.c_double), ("main_kernel_ms", C.c_double),
                ("main_launches", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class DeviceBatch(C.Structure):
    _fields_ = [("d_jobs", C.c_void_p), ("n_jobs", C.c_int), ("d_codes", C.c_void_p), ("d_n_aln", C.c_void_p),
                ("d_flags", C.c_void_p), ("d_hit_off", C.c_void_p), ("d_hits", C.c_void_p),
                ("hit_cap", C.c_uint64), ("d_counters", C.c_void_p), ("max_len", C.c_int32),
                ("max_seed", C.c_int32)]


class SeedBatch(C.Structure):
    """hsa_seed_batch_t (include/hsa_gpu.h): the splice seeds of a device batch."""
    _fields_ = [("d_jobs", C.c_void_p), ("n_jobs", C.c_int), ("d_codes", C.c_void_p), ("d_flags", C.c_void_p),
                ("d_n_aln", C.c_void_p), ("d_hit_off", C.c_void_p), ("d_hits", C.c_void_p), ("hit_cap", C.c_uint64),
                ("d_counters", C.c_void_p), ("max_len", C.c_int32)]


class SplicePf(C.Structure):
    """hsa_splice_pf_t (include/hsa_gpu.h): the splice prefetch's outputs."""
    _fields_ = [("n", C.c_int), ("max_len", C.c_int), ("row_stride", C.c_int), ("cw_stride", C.c_int),
                ("rows", C.c_void_p), ("call_n", C.c_void_p), ("call_hit", C.c_void_p), ("hits", C.c_void_p),
                ("wafter", C.c_void_p), ("call_sa", C.c_void_p), ("sa", C.c_void_p), ("n_hits", C.c_uint64),
                ("n_sa", C.c_uint64), ("kernel_ms", C.c_double)]


class SpliceBatch(C.Structure):
    """hsa_splice_batch_t (include/hsa_gpu.h): the splice path of a device batch."""
    _fields_ = [("d_jobs", C.c_void_p), ("n_jobs", C.c_int), ("d_codes", C.c_void_p), ("d_flags", C.c_void_p),
                ("d_n_aln", C.c_void_p), ("d_res", C.c_void_p), ("d_counters", C.c_void_p), ("max_len", C.c_int32)]


def ext_regime(local_opt: dict, n_stacks: int, max_diff: int) -> "Regime":
    """The splice path's extension regime (aux_ext: local_opt with max_gape 3,
    bwtgap.c:776-782); GAPE / LOGGAP as the extension reads them, whatever max_gapo."""
    ao = dict(local_opt, max_gape=3)
    r = regime_of(ao, n_stacks, max_diff)
    r.mode = ao["mode"] & (0x01 | 0x04 | 0x10)
    return r


def anchor_regime(local_opt: dict, n_stacks: int, max_diff: int) -> "Regime":
    """The 12-mer anchors' regime (aux_ext's options, bwt_match_gap with width_seed NULL)."""
    return regime_of(dict(local_opt, max_gape=3), n_stacks, max_diff)


class SpliceStats(C.Structure):
    """hsa_splice_stats_t (include/hsa_gpu.h)."""
    _fields_ = [("kernel_ms", C.c_double), ("extensions", C.c_uint64), ("pops", C.c_uint64),
                ("sa_lookups", C.c_uint64), ("not_answered", C.c_uint64)]


_lib = None


def _check_runtime():
    """libhsa_gpu.so is built against /opt/rocm's HIP runtime.  PyTorch-ROCm bundles
    an older HIP/HSA runtime with the same sonames; whichever is loaded first serves
    both.  With torch's loaded first the library sees no device, so the package must
    be imported before torch (hsa_amd/__init__.py loads the library eagerly)."""
    try:
        maps = open("/proc/self/maps").read()
    except OSError:
        return
    hip = {ln.split()[-1] for ln in maps.splitlines() if "libamdhip64" in ln}
    if any("/torch/lib/" in h for h in hip):
        raise HsaError("the HIP runtime bundled with torch was loaded before libhsa_gpu.so: "
                       "import hsa_amd before importing torch")


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HsaError(f"{LIB_PATH} is missing: build it with `make -C hsa_amd/csrc` (no CPU fallback exists)")
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    _check_runtime()
    u32 = np.ctypeslib.ndpointer(np.uint32, flags="C")
    u64 = np.ctypeslib.ndpointer(np.uint64, flags="C")
    i32 = np.ctypeslib.ndpointer(np.int32, flags="C")
    u8 = np.ctypeslib.ndpointer(np.uint8, flags="C")
    vp = C.c_void_p
    L.hsa_device_count.restype = C.c_int
    L.hsa_last_error.restype = C.c_char_p
    L.hsa_index_create.argtypes = [C.c_int, C.c_uint32, C.c_uint32, u32, u32, C.c_uint32, C.c_uint32, u32, u32,
                                   C.POINTER(vp)]
    L.hsa_index_create_device.argtypes = [C.c_int, C.c_uint32, C.c_uint32, u32, vp, C.c_uint32, C.c_uint32, u32, vp,
                                          C.POINTER(vp)]
    L.hsa_index_free.argtypes = [vp]
    L.hsa_index_release_scratch.argtypes = [vp]
    L.hsa_index_bytes.restype = C.c_size_t
    L.hsa_index_bytes.argtypes = [vp]
    L.hsa_index_trie.argtypes = [vp, C.c_void_p, C.c_void_p, C.c_void_p]
    L.hsa_index_clone.argtypes = [vp, C.POINTER(vp)]
    L.hsa_index_stream.restype = vp
    L.hsa_index_stream.argtypes = [vp]
    L.hsa_occ4_batch.argtypes = [vp, C.c_int, C.c_size_t, u32, u32]
    L.hsa_step_batch.argtypes = [vp, C.c_size_t, u32, u32]
    L.hsa_width_batch.argtypes = [vp, C.c_size_t, u64, u32, u8, C.c_size_t, u32]
    if hasattr(L, "hsa_width0_batch"):
        L.hsa_width0_batch.argtypes = [vp, C.c_size_t, u64, u32, u8, C.c_size_t, u32]
    L.hsa_search_batch.restype = C.c_long
    L.hsa_search_batch.argtypes = [vp, C.POINTER(Regime), C.c_int, vp, C.c_int, u8, C.c_size_t, i32, u32, u64,
                                   C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(Stats)]
    L.hsa_search_device.argtypes = [vp, C.POINTER(Regime), C.c_int, C.POINTER(DeviceBatch), vp]
    L.hsa_configure.argtypes = [C.c_int, C.c_int, C.c_int]
    L.hsa_free.argtypes = [vp]
    L.hsa_synth_genome_device.argtypes = [C.c_int, C.c_uint64, C.c_uint64, vp]
    L.hsa_index_set_sa.argtypes = [vp, u32, C.c_uint64, C.c_uint32, u32, C.c_int]
    L.hsa_sa_position_batch.argtypes = [vp, C.c_size_t, u32, u32]
    L.hsa_probe_gather.argtypes = [C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_double)]
    L.hsa_build_bwt_device.argtypes = [C.c_int, C.c_uint64, vp, C.c_int, vp, C.POINTER(C.c_uint32), u32]
    L.hsa_match_gap_batch.restype = C.c_long
    L.hsa_match_gap_batch.argtypes = [vp, C.POINTER(Regime), C.c_int, vp, vp, C.c_int, u8, C.c_size_t, i32, C.c_size_t,
                                      i32, i32, u64, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(Stats)]
    L.hsa_splice_seeds_device.argtypes = [vp, C.POINTER(Regime), C.POINTER(SeedBatch), vp]
    if hasattr(L, "hsa_splice_prefetch_batch"):
        L.hsa_splice_prefetch_batch.argtypes = [vp, C.POINTER(Regime), C.POINTER(Regime), C.c_int, u32, u64, u8,
                                                C.c_size_t, i32, C.POINTER(SplicePf)]
    if hasattr(L, "hsa_splice_device"):
        L.hsa_splice_device.argtypes = [vp, C.POINTER(Regime), C.POINTER(Regime), C.POINTER(Regime),
                                        C.POINTER(SpliceBatch), vp]
    if hasattr(L, "hsa_splice_match_batch"):
        L.hsa_index_set_text.argtypes = [vp, u32, C.c_uint64, C.c_uint32]
        L.hsa_splice_match_batch.argtypes = [vp, C.POINTER(Regime), C.POINTER(Regime), C.POINTER(Regime), C.c_int, u32,
                                             u64, u8, C.c_size_t, i32, C.POINTER(SplicePf), u32,
                                             C.POINTER(SpliceStats)]
    if hasattr(L, "hsa_search_device64"):           # (older A/B builds lack the 64-bit path)
        L.hsa_index_create_device64.argtypes = [C.c_int, C.c_uint64, C.c_uint64, u64, vp, C.c_uint64, C.c_uint64,
                                                u64, vp, C.POINTER(vp)]
        L.hsa_index_is64.argtypes = [vp]
        L.hsa_occ4_batch64.argtypes = [vp, C.c_int, C.c_size_t, u64, u64]
        L.hsa_search_device64.argtypes = [vp, C.POINTER(Regime), C.c_int, C.POINTER(DeviceBatch), vp]
        L.hsa_build_bwt_device64.argtypes = [C.c_int, C.c_uint64, vp, C.c_int, vp, C.POINTER(C.c_uint64), u64]
    if hasattr(L, "hsa_build_bwt_index_device"):
        L.hsa_build_bwt_index_device.argtypes = [C.c_int, C.c_uint64, vp, vp, C.POINTER(C.c_uint64), u64, C.c_uint32,
                                                 vp]
    if hasattr(L, "hsa_extend_batch"):
        L.hsa_extend_batch.argtypes = [vp, C.POINTER(Regime), C.c_int, vp, C.c_int, u8, i32, C.c_size_t, i32, i32,
                                       u32]
    if hasattr(L, "hsa_extend_sliced"):
        L.hsa_extend_sliced.argtypes = [vp, C.POINTER(Regime), C.c_int, vp, i32, u8, C.c_int, u8, i32, C.c_size_t,
                                        C.c_int, C.c_uint32, i32, i32, u32]
    f32 = np.ctypeslib.ndpointer(np.float32, flags="C")
    L.hsa_pass_times.argtypes = [vp, C.c_int, f32, f32]
    if hasattr(L, "hsa_cal_sa_reg_gap_multi"):      # (older A/B builds lack it)
        L.hsa_cal_sa_reg_gap_multi.restype = C.c_long
        L.hsa_cal_sa_reg_gap_multi.argtypes = [C.POINTER(vp), C.c_int, C.POINTER(GapOpt), C.c_int, u32, u64, u8,
                                               C.c_size_t, i32, u32, u64, C.POINTER(C.POINTER(C.c_uint32)), i32,
                                               C.POINTER(Stats)]
    L.hsa_cal_sa_reg_gap_flat.restype = C.c_long
    L.hsa_cal_sa_reg_gap_flat.argtypes = [vp, C.POINTER(GapOpt), C.c_int, u32, u64, u8, C.c_size_t, i32, u32, u64,
                                          C.POINTER(C.POINTER(C.c_uint32)), i32, C.POINTER(Stats)]
    _lib = L
    return L


def check(rc):
    if rc < 0:
        raise HsaError(f"libhsa_gpu error {rc}: {lib().hsa_last_error().decode()}")
    return rc


def device_count() -> int:
    return lib().hsa_device_count()


def probe_gather(table_bytes: int, per_sector: int = 1, device: int = 0) -> float:
    """Measured random 64-byte-sector gather rate in GB/s (hsa_probe_gather)."""
    g = C.c_double()
    check(lib().hsa_probe_gather(device, table_bytes, per_sector, C.byref(g)))
    return g.value


def configure(waves_per_cu=0, pool_entries=0, hit_cap=0):
    check(lib().hsa_configure(waves_per_cu, pool_entries, hit_cap))


def _take_hits(hp, n):
    if n == 0:
        lib().hsa_free(hp)
        return np.zeros((0, 9), np.uint32)
    arr = np.ctypeslib.as_array(hp, shape=(n * 9,)).reshape(n, 9).copy()
    lib().hsa_free(hp)
    return arr


class GpuIndex:
    """The bidirectional index resident in HBM as rank blocks (one device)."""

    def __init__(self, fwd, rev, device: int = 0):
        self.T = fwd.T
        self.fwd_meta = fwd
        h = C.c_void_p()
        check(lib().hsa_index_create(device, fwd.T, fwd.isa0, np.ascontiguousarray(fwd.C, np.uint32),
                                     np.ascontiguousarray(fwd.code, np.uint32), rev.T, rev.isa0,
                                     np.ascontiguousarray(rev.C, np.uint32),
                                     np.ascontiguousarray(rev.code, np.uint32), C.byref(h)))
        self.h = h

    @classmethod
    def from_device_codes(cls, T, isa0, Cf, d_code, rT, risa0, Cr, d_rcode, device=0):
        self = cls.__new__(cls)
        self.T = T
        h = C.c_void_p()
        check(lib().hsa_index_create_device(device, T, isa0, np.ascontiguousarray(Cf, np.uint32), d_code, rT, risa0,
                                            np.ascontiguousarray(Cr, np.uint32), d_rcode, C.byref(h)))
        self.h = h
        return self

    @classmethod
    def from_device_codes64(cls, T, isa0, Cf, d_code, rT, risa0, Cr, d_rcode, device=0):
        """A 64-bit interval index (hsa_index_create_device64): any text length; under
        2^32 characters the 32-bit entry points serve it too."""
        self = cls.__new__(cls)
        self.T = T
        h = C.c_void_p()
        check(lib().hsa_index_create_device64(device, T, isa0, np.ascontiguousarray(Cf, np.uint64), d_code, rT, risa0,
                                              np.ascontiguousarray(Cr, np.uint64), d_rcode, C.byref(h)))
        self.h = h
        return self

    def is64(self) -> bool:
        return bool(lib().hsa_index_is64(self.h))

    def occ4_64(self, d, pos):
        pos = np.ascontiguousarray(pos, np.uint64)
        out = np.zeros((len(pos), 4), np.uint64)
        check(lib().hsa_occ4_batch64(self.h, d, len(pos), pos, out))
        return out

    def search_device64(self, regimes, batch: "DeviceBatch"):
        """hsa_search_device64: d_hits holds hsa_aln64_t records (14 u32)."""
        rg = (Regime * len(regimes))(*regimes)
        check(lib().hsa_search_device64(self.h, rg, len(regimes), C.byref(batch), None))

    def clone(self) -> "GpuIndex":
        """A second handle on this resident index (hsa_index_clone): the rank blocks,
        tries and SA are shared, the stream and search scratch are its own, so passes on
        the two handles run concurrently.  Closing this index closes its clones first."""
        h = C.c_void_p()
        check(lib().hsa_index_clone(self.h, C.byref(h)))
        c = GpuIndex.__new__(GpuIndex)
        c.T, c.h, c._parent = self.T, h, self
        if hasattr(self, "fwd_meta"):
            c.fwd_meta = self.fwd_meta
        if not hasattr(self, "_clones"):
            self._clones = weakref.WeakSet()
        self._clones.add(c)
        return c

    def release_scratch(self):
        """hsa_index_release_scratch: the handle's search and splice working buffers go back
        (the next call allocates them again)."""
        if getattr(self, "h", None):
            check(lib().hsa_index_release_scratch(self.h))

    def close(self):
        for c in list(getattr(self, "_clones", ())):
            c.close()
        if getattr(self, "h", None):
            lib().hsa_index_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stream_handle(self) -> int:
        return int(lib().hsa_index_stream(self.h))

    def search_device(self, regimes, batch: "DeviceBatch"):
        rg = (Regime * len(regimes))(*regimes)
        check(lib().hsa_search_device(self.h, rg, len(regimes), C.byref(batch), None))

    def splice_seeds_device(self, seed_regime, batch: "SeedBatch"):
        """The six splice seed searches of every fallback read of a device batch
        (hsa_splice_seeds_device); records 6 r + i on the device."""
        check(lib().hsa_splice_seeds_device(self.h, C.byref(seed_regime), C.byref(batch), None))

    def splice_prefetch(self, seed_regime, anchor_regime, lens, codes, anchor_max_diff):
        """hsa_splice_prefetch_batch over host reads: numpy copies of its outputs
        (rows (n, 6, row_stride, 2), call_n (n, 8), call_hit, hits (m, 9), wafter
        (n, 8, cw_stride, 2), call_sa, sa (k, 4))."""
        lens = np.ascontiguousarray(lens, np.uint32)
        codes = np.ascontiguousarray(codes, np.uint8)
        offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64)
        amd = np.ascontiguousarray(anchor_max_diff, np.int32)
        o = SplicePf()
        check(lib().hsa_splice_prefetch_batch(self.h, C.byref(seed_regime), C.byref(anchor_regime), len(lens), lens,
                                              offs, codes, len(codes), amd, C.byref(o)))
        n, rs, cws = o.n, o.row_stride, o.cw_stride

        def arr(ptr, ct, count):
            if not ptr or count == 0:
                return np.zeros(0, ct)
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(ct))), (count,)).copy()
        return dict(rows=arr(o.rows, np.int32, n * 6 * rs * 2).reshape(n, 6, rs, 2),
                    call_n=arr(o.call_n, np.int32, n * 8).reshape(n, 8),
                    call_hit=arr(o.call_hit, np.uint64, n * 8).reshape(n, 8),
                    hits=arr(o.hits, np.uint32, int(o.n_hits) * 9).reshape(-1, 9),
                    wafter=arr(o.wafter, np.int32, n * 8 * cws * 2).reshape(n, 8, cws, 2),
                    call_sa=arr(o.call_sa, np.uint64, n * 8).reshape(n, 8) if o.call_sa else None,
                    sa=arr(o.sa, np.uint32, int(o.n_sa) * 4).reshape(-1, 4), kernel_ms=o.kernel_ms)

    def set_text(self, packed_words, dna_len):
        """Upload the packed reference as the HSP holds it (16 codes per u32, the first in
        the high bits; hsa_index_set_text) for the splice kernel."""
        w = np.ascontiguousarray(packed_words, np.uint32)
        check(lib().hsa_index_set_text(self.h, w, len(w), int(dna_len)))

    def splice_device(self, seed_regime, anchor_regime, ext_regime, batch: "SpliceBatch"):
        """bwt_splice_match of every fallback read of a device batch, on the device
        (hsa_splice_device): HSA_SP_RES_WORDS words per job at batch.d_res."""
        check(lib().hsa_splice_device(self.h, C.byref(seed_regime), C.byref(anchor_regime), C.byref(ext_regime),
                                      C.byref(batch), None))

    def splice_match(self, seed_regime, anchor_regime, ext_regime, lens, codes, max_diff):
        """hsa_splice_match_batch: bwt_splice_match of each read on the device.  Returns
        (res (n, SP_RES_WORDS) uint32: status, n_aln, res_aln[0], res_aln[1]; stats)."""
        lens = np.ascontiguousarray(lens, np.uint32)
        codes = np.ascontiguousarray(codes, np.uint8)
        offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64)
        amd = np.ascontiguousarray(max_diff, np.int32)
        res = np.zeros((len(lens), SP_RES_WORDS), np.uint32)
        o, st = SplicePf(), SpliceStats()
        check(lib().hsa_splice_match_batch(self.h, C.byref(seed_regime), C.byref(anchor_regime), C.byref(ext_regime),
                                           len(lens), lens, offs, codes, len(codes), amd, C.byref(o), res,
                                           C.byref(st)))
        return res, {k: getattr(st, k) for k, _ in SpliceStats._fields_}

    def set_sa(self, sa, blocks):
        """Upload the sampled SA (index_io.SaFile) and the block table (rows of
        chrID, blockStart, blockEnd, ori) for SA -> position (hsa_index_set_sa)."""
        vals = np.ascontiguousarray(sa.values, np.uint32)
        blk = np.ascontiguousarray(blocks, np.uint32).reshape(-1)
        if blk.size == 0:
            blk = np.zeros(4, np.uint32)
        check(lib().hsa_index_set_sa(self.h, vals, len(vals), sa.interval, blk, len(blocks)))

    def sa_positions(self, idx):
        """(SA value, chrID, 1-based position, packed position) per SA index."""
        idx = np.ascontiguousarray(idx, np.uint32)
        out = np.zeros((len(idx), 4), np.uint32)
        check(lib().hsa_sa_position_batch(self.h, len(idx), idx, out))
        return out

    def last_pass_ms(self):
        """(k_widths ms, k_search ms) of the last device pass on this index."""
        w, q = C.c_float(), C.c_float()
        check(lib().hsa_last_pass_ms(self.h, C.byref(w), C.byref(q)))
        return w.value, q.value

    def pass_times(self, n):
        """(k_widths ms, k_search ms) arrays of the last n hsa_search_device passes."""
        w = np.zeros(n, np.float32)
        s = np.zeros(n, np.float32)
        check(lib().hsa_pass_times(self.h, n, w, s))
        return w, s

    def nbytes(self) -> int:
        return int(lib().hsa_index_bytes(self.h))

    def trie(self):
        """(width-trie depth, search-trie depth, bytes) of the index's root tries."""
        d, sd, b = C.c_uint32(), C.c_uint32(), C.c_size_t()
        check(lib().hsa_index_trie(self.h, C.byref(d), C.byref(sd), C.byref(b)))
        return int(d.value), int(sd.value), int(b.value)

    def occ4(self, d, pos):
        pos = np.ascontiguousarray(pos, np.uint32)
        out = np.zeros((len(pos), 4), np.uint32)
        check(lib().hsa_occ4_batch(self.h, d, len(pos), pos, out))
        return out

    def step_all(self, klrr):
        klrr = np.ascontiguousarray(klrr, np.uint32).reshape(-1, 4)
        out = np.zeros((len(klrr), 16), np.uint32)
        check(lib().hsa_step_batch(self.h, len(klrr), klrr, out))
        return out.reshape(-1, 4, 4)   # [n][k, l, rk, rl][c]

    def widths(self, lens, codes, type=1):
        """bwt_cal_width of each sequence (type 1: hsa_width_batch, 0: hsa_width0_batch):
        2 * (len + 1) words each, packed."""
        lens = np.ascontiguousarray(lens, np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64)
        tot = int(np.sum(2 * (lens.astype(np.int64) + 1)))
        out = np.zeros(tot, np.uint32)
        codes = np.ascontiguousarray(codes, np.uint8)
        fn = lib().hsa_width_batch if type == 1 else lib().hsa_width0_batch
        check(fn(self.h, len(lens), offs, lens, codes, len(codes), out))
        return out

    def search(self, regimes, jobs, codes):
        """Raw search over a job table (JOB_DTYPE)."""
        jobs = np.ascontiguousarray(jobs, JOB_DTYPE)
        n = len(jobs)
        rg = (Regime * len(regimes))(*regimes)
        n_aln = np.zeros(n, np.int32)
        flags = np.zeros(n, np.uint32)
        hoff = np.zeros(n, np.uint64)
        hp = C.POINTER(C.c_uint32)()
        st = Stats()
        codes = np.ascontiguousarray(codes, np.uint8)
        tot = check(lib().hsa_search_batch(self.h, rg, len(regimes), jobs.ctypes.data, n, codes, len(codes), n_aln,
                                           flags, hoff, C.byref(hp), C.byref(st)))
        return n_aln, flags, hoff, _take_hits(hp, tot), st.as_dict()

    def extend(self, regimes, jobs, codes, bids):
        """hsa_extend_batch: jobs (EXT_DTYPE), the windows' codes / bids; returns
        (ret, max_pos, aln (n, 9))."""
        n = len(jobs)
        rg = (Regime * len(regimes))(*regimes)
        ret = np.zeros(n, np.int32)
        mp = np.zeros(n, np.int32)
        aln = np.zeros((n, 9), np.uint32)
        codes = np.ascontiguousarray(codes, np.uint8)
        bids = np.ascontiguousarray(bids, np.int32)
        check(lib().hsa_extend_batch(self.h, rg, len(regimes), np.ascontiguousarray(jobs).ctypes.data, n,
                                     codes if len(codes) else np.zeros(1, np.uint8),
                                     bids if len(bids) else np.zeros(1, np.int32), len(codes), ret, mp, aln))
        return ret, mp, aln

    def extend_sliced(self, regimes, jobs, codes, bids, slots, resume, n_slots, budget):
        """One hsa_extend_sliced launch: returns (ret, max_pos, aln (n, 9))."""
        n = len(jobs)
        rg = (Regime * len(regimes))(*regimes)
        ret = np.zeros(n, np.int32)
        mp = np.zeros(n, np.int32)
        aln = np.zeros((n, 9), np.uint32)
        codes = np.ascontiguousarray(codes, np.uint8)
        bids = np.ascontiguousarray(bids, np.int32)
        check(lib().hsa_extend_sliced(self.h, rg, len(regimes), np.ascontiguousarray(jobs).ctypes.data,
                                      np.ascontiguousarray(slots, np.int32), np.ascontiguousarray(resume, np.uint8), n,
                                      codes if len(codes) else np.zeros(1, np.uint8),
                                      bids if len(bids) else np.zeros(1, np.int32), len(codes), int(n_slots),
                                      int(budget), ret, mp, aln))
        return ret, mp, aln

    def match_gap(self, regimes, jobs, mg, codes, widths):
        """hsa_match_gap_batch: direct bwt_match_gap calls with caller widths.
        widths (P, 2) int32 pairs; returns (n_aln, hit_off, hits, widths after, stats)."""
        jobs = np.ascontiguousarray(jobs, JOB_DTYPE)
        mg = np.ascontiguousarray(mg, MG_DTYPE)
        n = len(jobs)
        rg = (Regime * len(regimes))(*regimes)
        w = np.ascontiguousarray(widths, np.int32).reshape(-1)
        wout = w.copy()
        n_aln = np.zeros(n, np.int32)
        hoff = np.zeros(n, np.uint64)
        hp = C.POINTER(C.c_uint32)()
        st = Stats()
        codes = np.ascontiguousarray(codes, np.uint8)
        tot = check(lib().hsa_match_gap_batch(self.h, rg, len(regimes), jobs.ctypes.data, mg.ctypes.data, n, codes,
                                              len(codes), w, len(w) // 2, wout, n_aln, hoff, C.byref(hp),
                                              C.byref(st)))
        return n_aln, hoff, _take_hits(hp, tot), wout.reshape(-1, 2), st.as_dict()

    def cal_sa_reg_gap(self, lens, codes, opt: GapOpt):
        """bwa_cal_sa_reg_gap semantics over one batch (mutates opt like the reference)."""
        lens = np.ascontiguousarray(lens, np.uint32)
        n = len(lens)
        offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64) if n else \
            np.zeros(0, np.uint64)
        codes = np.ascontiguousarray(codes, np.uint8)
        n_aln = np.zeros(n, np.int32)
        flags = np.zeros(n, np.uint32)
        hoff = np.zeros(n, np.uint64)
        sp = np.zeros(2 * n + 2, np.int32)
        hp = C.POINTER(C.c_uint32)()
        st = Stats()
        tot = check(lib().hsa_cal_sa_reg_gap_flat(self.h, C.byref(opt), n, lens, offs, codes, len(codes), n_aln,
                                                  flags, hoff, C.byref(hp), sp, C.byref(st)))
        hits = _take_hits(hp, tot)
        return n_aln, flags, hoff, hits, st.as_dict()

    def cal_sa_reg_gap_slots(self, others, lens, codes, opt: GapOpt):
        """cal_sa_reg_gap split over this index and `others` (device slots holding the
        same BWT: hsa_cal_sa_reg_gap_multi)."""
        ixs = [self] + list(others)
        arr = (C.c_void_p * len(ixs))(*[i.h for i in ixs])
        lens = np.ascontiguousarray(lens, np.uint32)
        n = len(lens)
        offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64) if n else \
            np.zeros(0, np.uint64)
        codes = np.ascontiguousarray(codes, np.uint8)
        n_aln = np.zeros(n, np.int32)
        flags = np.zeros(n, np.uint32)
        hoff = np.zeros(n, np.uint64)
        sp = np.zeros(2 * n + 2, np.int32)
        hp = C.POINTER(C.c_uint32)()
        st = Stats()
        tot = check(lib().hsa_cal_sa_reg_gap_multi(arr, len(ixs), C.byref(opt), n, lens, offs, codes, len(codes), n_aln,
                                                   flags, hoff, C.byref(hp), sp, C.byref(st)))
        return n_aln, flags, hoff, _take_hits(hp, tot), st.as_dict()

    def run_batches(self, lens, codes, opt_dict, batch, others=()):
        """bwa_aln_core's batch loop (bwtaln.c:477-506); hits regrouped in read order.
        With `others`, each batch is split over the device slots self + others."""
        opt = GapOpt.from_dict(opt_dict)
        lens = np.asarray(lens, np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
        na_all, fl_all, per_read, stats = [], [], [], []
        for b0 in range(0, len(lens), batch):
            b1 = min(b0 + batch, len(lens))
            if others:
                na, fl, ho, hits, st = self.cal_sa_reg_gap_slots(others, lens[b0:b1], codes[offs[b0]:offs[b1]], opt)
            else:
                na, fl, ho, hits, st = self.cal_sa_reg_gap(lens[b0:b1], codes[offs[b0]:offs[b1]], opt)
            for j in range(b1 - b0):
                per_read.append(hits[int(ho[j]):int(ho[j]) + max(int(na[j]), 0)])
            na_all.append(na)
            fl_all.append(fl)
            stats.append(st)
        n_aln = np.concatenate(na_all) if na_all else np.zeros(0, np.int32)
        flags = np.concatenate(fl_all) if fl_all else np.zeros(0, np.uint32)
        return n_aln, flags, per_read, stats
