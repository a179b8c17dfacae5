"""ctypes binding of oracle/liboracle.so -- the CPU restatement (test infrastructure).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "liboracle.so")
LIB64 = os.path.join(ROOT, "oracle", "liboracle64.so")   # the same restatement, 64-bit intervals

OPT_FIELDS = [("s_mm", C.c_int), ("s_gapo", C.c_int), ("s_gape", C.c_int), ("mode", C.c_int),
              ("indel_end_skip", C.c_int), ("max_del_occ", C.c_int), ("max_entries", C.c_int),
              ("fnr", C.c_float), ("max_diff", C.c_int), ("max_gapo", C.c_int), ("max_gape", C.c_int),
              ("max_seed_diff", C.c_int), ("seed_len", C.c_int), ("n_threads", C.c_int),
              ("max_top2", C.c_int), ("trim_qual", C.c_int)]


class Opt(C.Structure):
    _fields_ = OPT_FIELDS

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in OPT_FIELDS}

    @classmethod
    def from_dict(cls, d):
        o = cls()
        for k, _ in OPT_FIELDS:
            setattr(o, k, d[k])
        return o


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"], check=True,
                           capture_output=True)
        L = C.CDLL(LIB)
        u32p = np.ctypeslib.ndpointer(np.uint32, flags="C")
        L.or_index_create.restype = C.c_void_p
        L.or_index_create.argtypes = [C.c_uint32, C.c_uint32, u32p, u32p, C.c_uint32, C.c_uint32, u32p, u32p]
        L.or_index_free.argtypes = [C.c_void_p]
        L.or_occ4.argtypes = [C.c_void_p, C.c_int, C.c_uint32, u32p]
        L.or_step_all.argtypes = [C.c_void_p] + [C.c_uint32] * 4 + [u32p] * 4
        L.or_cal_width.argtypes = [C.c_void_p, C.c_int, np.ctypeslib.ndpointer(np.uint8, flags="C"), u32p]
        L.or_cal_width0.argtypes = [C.c_void_p, C.c_int, np.ctypeslib.ndpointer(np.uint8, flags="C"), u32p]
        L.or_init_opt.argtypes = [C.POINTER(Opt)]
        L.or_cal_maxdiff.argtypes = [C.c_int, C.c_double, C.c_double]
        L.or_cal_sa_reg_gap.restype = C.c_long
        L.or_cal_sa_reg_gap.argtypes = [C.c_void_p, C.c_int, u32p, np.ctypeslib.ndpointer(np.uint8, flags="C"),
                                        C.POINTER(Opt), np.ctypeslib.ndpointer(np.int32, flags="C"), u32p,
                                        C.POINTER(C.POINTER(C.c_uint32)), np.ctypeslib.ndpointer(np.uint64, flags="C")]
        L.or_free.argtypes = [C.c_void_p]
        i32p = np.ctypeslib.ndpointer(np.int32, flags="C")
        L.or_match_gap.restype = C.c_int
        L.or_match_gap.argtypes = [C.c_void_p, C.POINTER(Opt), C.c_int, np.ctypeslib.ndpointer(np.uint8, flags="C"),
                                   C.c_int, C.c_int, i32p, C.c_int, C.c_void_p, C.POINTER(C.POINTER(C.c_uint32))]
        L.or_sa_value.restype = C.c_uint32
        L.or_sa_value.argtypes = [C.c_void_p, u32p, C.c_uint32, C.c_uint32]
        L.or_sa_position.argtypes = [C.c_void_p, u32p, C.c_uint32, u32p, C.c_int, C.c_uint32,
                                     C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.or_extend.restype = C.c_int
        L.or_extend.argtypes = [C.c_void_p, C.POINTER(Opt), C.c_int, C.c_int, C.c_int,
                                np.ctypeslib.ndpointer(np.uint8, flags="C"), i32p, C.c_int, C.c_int, u32p,
                                C.POINTER(C.c_int)]
        _lib = L
    return _lib


_lib64 = None


def lib64():
    global _lib64
    if _lib64 is None:
        if not os.path.exists(LIB64):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle64.so"], check=True,
                           capture_output=True)
        L = C.CDLL(LIB64)
        u32p = np.ctypeslib.ndpointer(np.uint32, flags="C")
        u64p = np.ctypeslib.ndpointer(np.uint64, flags="C")
        L.or64_index_create.restype = C.c_void_p
        L.or64_index_create.argtypes = [C.c_uint64, C.c_uint64, u64p, u32p, C.c_uint64, C.c_uint64, u64p, u32p]
        L.or64_index_free.argtypes = [C.c_void_p]
        L.or64_occ4.argtypes = [C.c_void_p, C.c_int, C.c_uint64, u64p]
        L.or64_step_all.argtypes = [C.c_void_p] + [C.c_uint64] * 4 + [u64p] * 4
        L.or64_cal_width.argtypes = [C.c_void_p, C.c_int, np.ctypeslib.ndpointer(np.uint8, flags="C"), u64p]
        L.or64_cal_sa_reg_gap.restype = C.c_long
        L.or64_cal_sa_reg_gap.argtypes = [C.c_void_p, C.c_int, u32p, np.ctypeslib.ndpointer(np.uint8, flags="C"),
                                          C.POINTER(Opt), np.ctypeslib.ndpointer(np.int32, flags="C"), u32p,
                                          C.POINTER(C.POINTER(C.c_uint32)), np.ctypeslib.ndpointer(np.uint64, flags="C")]
        L.or64_free.argtypes = [C.c_void_p]
        _lib64 = L
    return _lib64


def msb_to_lsb(code, T):
    """.bwt words (char j at bits 31-2j..30-2j) -> LSB-first words (char j at bits
    2j..2j+1), the trailing codes past T cleared."""
    x = np.ascontiguousarray(code, np.uint32).copy()
    x = (x >> 16) | (x << 16)
    x = ((x & 0xFF00FF00) >> 8) | ((x & 0x00FF00FF) << 8)
    x = ((x & 0xF0F0F0F0) >> 4) | ((x & 0x0F0F0F0F) << 4)
    x = ((x & 0xCCCCCCCC) >> 2) | ((x & 0x33333333) << 2)
    x = x.astype(np.uint32)
    if T % 16:
        x[-1] &= np.uint32((1 << (2 * (T % 16))) - 1)
    return x


def default_opt():
    o = Opt()
    lib().or_init_opt(C.byref(o))
    return o.as_dict()


class OracleIndex:
    def __init__(self, fwd, rev):
        self.fwd, self.rev = fwd, rev
        self.h = lib().or_index_create(fwd.T, fwd.isa0, fwd.C, fwd.code, rev.T, rev.isa0, rev.C, rev.code)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_index_free(self.h)
            self.h = None

    def occ4(self, d, i):
        o = np.zeros(4, np.uint32)
        lib().or_occ4(self.h, d, i, o)
        return o

    def step_all(self, k, l, rk, rl):
        out = [np.zeros(4, np.uint32) for _ in range(4)]
        lib().or_step_all(self.h, k, l, rk, rl, *out)
        return out

    def sa_positions(self, sa, blocks, idx):
        """BWTSaValue + BWTRetrievePositionFromSAIndex per SA index: (sa, seq_id, ori_pos,
        occ_pos), seq_id / ori_pos = 0xFFFFFFFF when no block holds the position."""
        vals = np.ascontiguousarray(sa.values, np.uint32)
        blk = np.ascontiguousarray(blocks, np.uint32).reshape(-1)
        out = np.zeros((len(idx), 4), np.uint32)
        sid, ori, occ = C.c_uint32(), C.c_uint32(), C.c_uint32()
        for j, i in enumerate(np.asarray(idx, np.uint64)):
            sid.value = ori.value = 0xFFFFFFFF
            lib().or_sa_position(self.h, vals, sa.interval, blk, len(blk) // 4, int(i), C.byref(sid), C.byref(ori),
                                 C.byref(occ))
            out[j] = (occ.value, sid.value, ori.value, occ.value)
        return out

    def cal_width(self, seq):
        seq = np.ascontiguousarray(seq, np.uint8)
        w = np.zeros(2 * (len(seq) + 1), np.uint32)
        lib().or_cal_width(self.h, len(seq), seq, w)
        return w.reshape(-1, 2)

    def cal_width0(self, seq):
        """bwt_cal_width type 0; entry 0 (never written by the reference) is 0."""
        seq = np.ascontiguousarray(seq, np.uint8)
        w = np.zeros(2 * (len(seq) + 1), np.uint32)
        lib().or_cal_width0(self.h, len(seq), seq, w)
        return w.reshape(-1, 2)

    def match_gap(self, opt: Opt, n_stacks, seq, strand, width, seed, width_seed=None):
        """bwt_match_gap with caller widths (or_match_gap): width (len+1, 2) int32 is
        copied, returns (hits (n, 9), width after gap_shadow)."""
        seq = np.ascontiguousarray(seq, np.uint8)
        w = np.ascontiguousarray(width, np.int32).copy()
        ws = np.ascontiguousarray(width_seed, np.int32) if seed == 1 else None
        hp = C.POINTER(C.c_uint32)()
        n = lib().or_match_gap(self.h, C.byref(opt), int(n_stacks), seq, len(seq), int(strand), w, int(seed),
                               ws.ctypes.data if ws is not None else None, C.byref(hp))
        hits = np.ctypeslib.as_array(hp, shape=(max(n, 1) * 9,))[:n * 9].reshape(n, 9).copy()
        lib().or_free(hp)
        return hits, w

    def extend(self, opt: Opt, n_stacks, is_backward, length, seq, bid, lo, aln, max_pos):
        """bwt_extend_backward / bwt_extend_foreward (or_extend) on a window of the read:
        returns (ret, max_pos, aln after (9,) uint32)."""
        a = np.ascontiguousarray(aln, np.uint32).copy()
        mp = C.c_int(int(max_pos))
        seq = np.ascontiguousarray(seq, np.uint8)
        bid = np.ascontiguousarray(bid, np.int32)
        ret = lib().or_extend(self.h, C.byref(opt), int(n_stacks), int(is_backward), int(length),
                              seq if len(seq) else np.zeros(1, np.uint8), bid if len(bid) else np.zeros(1, np.int32),
                              int(lo), len(seq), a, C.byref(mp))
        return ret, mp.value, a

    def cal_sa_reg_gap(self, lens, codes, opt: Opt):
        """One batch; returns (n_aln, flags, hits(H,9), stats[queries, pops]); mutates opt."""
        n = len(lens)
        n_aln = np.zeros(n, np.int32)
        flags = np.zeros(n, np.uint32)
        stats = np.zeros(2, np.uint64)
        hp = C.POINTER(C.c_uint32)()
        tot = lib().or_cal_sa_reg_gap(self.h, n, np.ascontiguousarray(lens, np.uint32),
                                       np.ascontiguousarray(codes, np.uint8), C.byref(opt),
                                       n_aln, flags, C.byref(hp), stats)
        hits = np.ctypeslib.as_array(hp, shape=(max(tot, 1) * 9,))[:tot * 9].reshape(tot, 9).copy()
        lib().or_free(hp)
        return n_aln, flags, hits, stats

    def run_batches(self, lens, codes, opt_dict, batch):
        """bwa_aln_core's batch loop (bwtaln.c:477-506) over all reads."""
        opt = Opt.from_dict(opt_dict)
        offs = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
        outs = []
        for b0 in range(0, len(lens), batch):
            b1 = min(b0 + batch, len(lens))
            outs.append(self.cal_sa_reg_gap(lens[b0:b1], codes[offs[b0]:offs[b1]], opt))
        n_aln = np.concatenate([o[0] for o in outs])
        flags = np.concatenate([o[1] for o in outs])
        hits = np.concatenate([o[2] for o in outs]) if outs else np.zeros((0, 9), np.uint32)
        stats = sum(o[3] for o in outs)
        return n_aln, flags, hits, stats


class OracleIndex64:
    """liboracle64.so: the restatement with 64-bit intervals over LSB-first codes."""

    HW = 14

    def __init__(self, T, isa0, Cf, code_lsb, rT, risa0, Cr, rcode_lsb):
        self.T = int(T)
        self.h = lib64().or64_index_create(int(T), int(isa0), np.ascontiguousarray(Cf, np.uint64),
                                           np.ascontiguousarray(code_lsb, np.uint32), int(rT), int(risa0),
                                           np.ascontiguousarray(Cr, np.uint64), np.ascontiguousarray(rcode_lsb, np.uint32))

    @classmethod
    def from_index(cls, fwd, rev):
        """From index_io BWT objects (.bwt MSB-first words)."""
        return cls(fwd.T, fwd.isa0, np.asarray(fwd.C, np.uint64), msb_to_lsb(fwd.code, fwd.T), rev.T, rev.isa0,
                   np.asarray(rev.C, np.uint64), msb_to_lsb(rev.code, rev.T))

    def __del__(self):
        if getattr(self, "h", None):
            lib64().or64_index_free(self.h)
            self.h = None

    def occ4(self, d, i):
        o = np.zeros(4, np.uint64)
        lib64().or64_occ4(self.h, d, int(i), o)
        return o

    def step_all(self, k, l, rk, rl):
        out = [np.zeros(4, np.uint64) for _ in range(4)]
        lib64().or64_step_all(self.h, int(k), int(l), int(rk), int(rl), *out)
        return out

    def cal_width(self, seq):
        seq = np.ascontiguousarray(seq, np.uint8)
        w = np.zeros(2 * (len(seq) + 1), np.uint64)
        lib64().or64_cal_width(self.h, len(seq), seq, w)
        return w.reshape(-1, 2)

    def extend(self, opt: Opt, n_stacks, is_backward, length, seq, bid, lo, aln, max_pos):
        """bwt_extend_backward / bwt_extend_foreward (or_extend) on a window of the read:
        returns (ret, max_pos, aln after (9,) uint32)."""
        a = np.ascontiguousarray(aln, np.uint32).copy()
        mp = C.c_int(int(max_pos))
        seq = np.ascontiguousarray(seq, np.uint8)
        bid = np.ascontiguousarray(bid, np.int32)
        ret = lib().or_extend(self.h, C.byref(opt), int(n_stacks), int(is_backward), int(length),
                              seq if len(seq) else np.zeros(1, np.uint8), bid if len(bid) else np.zeros(1, np.int32),
                              int(lo), len(seq), a, C.byref(mp))
        return ret, mp.value, a

    def cal_sa_reg_gap(self, lens, codes, opt: Opt):
        """One batch; returns (n_aln, flags, hits(H,14), stats[queries, pops]); mutates opt."""
        n = len(lens)
        n_aln = np.zeros(n, np.int32)
        flags = np.zeros(n, np.uint32)
        stats = np.zeros(2, np.uint64)
        hp = C.POINTER(C.c_uint32)()
        tot = lib64().or64_cal_sa_reg_gap(self.h, n, np.ascontiguousarray(lens, np.uint32),
                                           np.ascontiguousarray(codes, np.uint8), C.byref(opt),
                                           n_aln, flags, C.byref(hp), stats)
        hits = np.ctypeslib.as_array(hp, shape=(max(tot, 1) * 14,))[:tot * 14].reshape(tot, 14).copy()
        lib64().or64_free(hp)
        return n_aln, flags, hits, stats


def aln64_to_aln32(h64):
    """hsa_aln64_t rows (14 u32) -> bwt_aln1_t rows (9 u32) when every interval bound
    fits 32 bits (sub-2^32 parity between the two instantiations)."""
    h64 = np.asarray(h64, np.uint32).reshape(-1, 14)
    assert not h64[:, [3, 5, 7, 9]].any(), "interval bound >= 2^32"
    out = np.zeros((len(h64), 9), np.uint32)
    out[:, 0] = h64[:, 0]
    out[:, 1:5] = h64[:, [2, 4, 6, 8]]
    out[:, 5] = h64[:, 1]
    out[:, 6] = h64[:, 10]
    out[:, 7] = h64[:, 11]
    out[:, 8] = h64[:, 12]
    return out
