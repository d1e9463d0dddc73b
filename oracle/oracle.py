"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU restatement
(oracle/liboracle.so).  Importable only from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; never from the product path."""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


class OracleParams(C.Structure):
    _fields_ = [("k", C.c_uint32), ("psa_min", C.c_uint32), ("stretch_constant", C.c_double),
                ("stretch_factor", C.c_double), ("stretch_cap", C.c_double), ("window_size", C.c_uint32),
                ("forward", C.c_int), ("max_match", C.c_int), ("max_count", C.c_int32),
                ("mers_matching", C.c_double), ("bases_matching", C.c_double), ("unitigs_k", C.c_uint32),
                ("unitig_lengths", C.POINTER(C.c_int32)), ("n_unitigs", C.c_size_t), ("legacy_no_filter", C.c_int),
                ("legacy_int_abs", C.c_int), ("fine_k", C.c_uint32)]


class OracleRecord(C.Structure):
    _fields_ = [("rs", C.c_int32), ("re", C.c_int32), ("qs", C.c_int32), ("qe", C.c_int32), ("nb_mers", C.c_int32),
                ("pb_cons", C.c_uint32), ("sr_cons", C.c_uint32), ("pb_cover", C.c_uint32), ("sr_cover", C.c_uint32),
                ("rl", C.c_uint64), ("ql", C.c_uint64), ("rn", C.c_int32), ("sr_index", C.c_uint32),
                ("use_bwd_name", C.c_int32), ("stretch", C.c_double), ("offset", C.c_double), ("avg_err", C.c_double),
                ("n_info", C.c_uint32), ("kmers_info", C.POINTER(C.c_int32)), ("bases_info", C.POINTER(C.c_int32)),
                ("emit", C.c_uint32)]


class OracleReadResult(C.Structure):
    _fields_ = [("n", C.c_size_t), ("recs", C.POINTER(OracleRecord))]


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(os.path.join(_HERE, "liboracle.so"))
        vp = C.c_void_p
        L.oracle_params_default.argtypes = [C.POINTER(OracleParams)]
        L.oracle_index_build_fasta.argtypes = [C.POINTER(C.c_char_p), C.c_size_t, C.c_uint32, C.c_int]
        L.oracle_index_build_fasta.restype = vp
        L.oracle_index_build_mem.argtypes = [C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.POINTER(C.c_uint64),
                                             C.c_size_t, C.c_uint32, C.c_int]
        L.oracle_index_build_mem.restype = vp
        L.oracle_index_free.argtypes = [vp]
        L.oracle_index_nb_sr.argtypes = [vp]
        L.oracle_index_nb_sr.restype = C.c_size_t
        L.oracle_index_sr_name.argtypes = [vp, C.c_size_t, C.c_int]
        L.oracle_index_sr_name.restype = C.c_char_p
        L.oracle_index_lookup.argtypes = [vp, C.c_uint64, C.POINTER(C.c_uint64), C.c_uint64]
        L.oracle_index_lookup.restype = C.c_uint64
        L.oracle_align_read.argtypes = [vp, C.POINTER(OracleParams), C.c_char_p, C.c_size_t,
                                        C.POINTER(OracleReadResult)]
        L.oracle_read_result_free.argtypes = [C.POINTER(OracleReadResult)]
        L.oracle_align_format.argtypes = [vp, C.POINTER(OracleParams), C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                          C.POINTER(C.c_uint64), C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.POINTER(C.c_size_t)]
        L.oracle_align_format.restype = C.c_void_p
        L.oracle_align_format_ex.argtypes = L.oracle_align_format.argtypes + [C.POINTER(C.c_void_p),
                                                                               C.POINTER(C.c_size_t)]
        L.oracle_align_format_ex.restype = C.c_void_p
        L.oracle_index_build_fine.argtypes = [vp, C.c_uint32, C.c_int]
        L.oracle_index_lookup_fine.argtypes = [vp, C.c_uint64, C.POINTER(C.c_uint64), C.c_uint64]
        L.oracle_index_lookup_fine.restype = C.c_uint64
        L.oracle_align_timed.argtypes = [vp, C.POINTER(OracleParams), C.POINTER(C.c_char_p), C.POINTER(C.c_uint64),
                                         C.c_size_t, C.c_int, C.POINTER(C.c_uint64)]
        L.oracle_align_timed.restype = C.c_double
        L.oracle_lis.argtypes = [C.POINTER(C.c_int32), C.c_uint32, C.c_uint32, C.c_int, C.c_double, C.c_double,
                                 C.c_double, C.c_int, C.c_double, C.POINTER(C.c_uint32)]
        L.oracle_lis.restype = C.c_uint32
        L.oracle_lsq.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_size_t, C.POINTER(C.c_double)]
        L.oracle_kmers_info.argtypes = [C.c_char_p, C.POINTER(C.c_int32), C.c_size_t, C.c_uint32, C.c_uint32,
                                        C.POINTER(C.c_int32), C.c_size_t, C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32), C.c_uint32]
        L.oracle_kmers_info.restype = C.c_uint32
        L.oracle_coords_info.argtypes = [C.c_char_p, C.c_uint32,
                                         C.POINTER(C.c_int32), C.c_uint32, C.POINTER(C.c_uint32), C.c_uint32,
                                         C.POINTER(C.c_int32), C.c_uint32, C.POINTER(C.c_uint32), C.c_uint32,
                                         C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(C.c_int32), C.c_size_t,
                                         C.c_int, C.POINTER(OracleRecord)]
        L.oracle_sr_name_reverse.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
        L.oracle_encode_line.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_uint8)]
        L.oracle_encode_line.restype = None
        L.oracle_is_ssr.argtypes = [C.c_uint64, C.c_uint32]
        L.free = C.CDLL(None).free
        _lib = L
    return _lib


def _cstrs(items):
    arr = (C.c_char_p * max(1, len(items)))()
    for i, s in enumerate(items):
        arr[i] = s if isinstance(s, bytes) else s.encode()
    return arr


def params(k=17, stretch_factor=1.3, stretch_constant=10, stretch_cap=10000.0, window_size=1, forward=False,
           max_match=False, max_count=5000, mers_matching=0.0, bases_matching=17.0, unitigs_k=0,
           unitig_lengths=None, legacy_no_filter=False, psa_min=13, fine_k=0, legacy_int_abs=False):
    p = OracleParams()
    lib().oracle_params_default(C.byref(p))
    p.k = k; p.psa_min = psa_min; p.stretch_constant = stretch_constant; p.stretch_factor = stretch_factor
    p.stretch_cap = stretch_cap; p.window_size = window_size; p.forward = int(bool(forward))
    p.max_match = int(bool(max_match)); p.max_count = max_count; p.mers_matching = mers_matching
    p.bases_matching = bases_matching; p.unitigs_k = unitigs_k; p.legacy_no_filter = int(bool(legacy_no_filter))
    p.fine_k = fine_k
    p.legacy_int_abs = int(bool(legacy_int_abs))
    keep = None
    if unitig_lengths is not None:
        keep = np.ascontiguousarray(unitig_lengths, dtype=np.int32)
        p.unitig_lengths = keep.ctypes.data_as(C.POINTER(C.c_int32))
        p.n_unitigs = len(keep)
    p._keep = keep
    return p


class OracleIndex:
    def __init__(self, h, k):
        self.h, self.k = h, k

    @classmethod
    def from_fasta(cls, paths, k, threads=8):
        return cls(lib().oracle_index_build_fasta(_cstrs(paths), len(paths), k, threads), k)

    @classmethod
    def from_records(cls, names, seqs, k, threads=8):
        bs = [s if isinstance(s, bytes) else s.encode() for s in seqs]
        lens = (C.c_uint64 * max(1, len(bs)))(*[len(b) for b in bs])
        return cls(lib().oracle_index_build_mem(_cstrs(names), _cstrs(bs), lens, len(bs), k, threads), k)

    def lookup(self, code, cap=1 << 16):
        out = (C.c_uint64 * cap)()
        n = lib().oracle_index_lookup(self.h, code, out, cap)
        return n, [out[i] for i in range(min(n, cap))]

    def build_fine(self, fine_k, threads=8):
        if lib().oracle_index_build_fine(self.h, fine_k, threads) != 0:
            raise ValueError(f"fine_k={fine_k} outside [1, k={self.k}]")
        return self

    def lookup_fine(self, code, cap=1 << 16):
        out = (C.c_uint64 * cap)()
        n = lib().oracle_index_lookup_fine(self.h, code, out, cap)
        return n, [out[i] for i in range(min(n, cap))]

    def sr_name(self, i, bwd=False):
        return lib().oracle_index_sr_name(self.h, i, int(bwd)).decode()

    def align_format(self, p, names, seqs, threads=1, compact=True, header=False, zero_match=False, details=False):
        """coords text; with details=True a (coords, details) pair."""
        bs = [s if isinstance(s, bytes) else s.encode() for s in seqs]
        lens = (C.c_uint64 * max(1, len(bs)))(*[len(b) for b in bs])
        n, dn, dt = C.c_size_t(), C.c_size_t(), C.c_void_p()
        t = lib().oracle_align_format_ex(self.h, C.byref(p), _cstrs(names), _cstrs(bs), lens, len(bs), threads,
                                         int(compact), int(header), int(zero_match), C.byref(n),
                                         C.byref(dt) if details else None, C.byref(dn))
        try:
            text = C.string_at(t, n.value).decode()
            if details:
                return text, C.string_at(dt.value, dn.value).decode() if dn.value else ""
            return text
        finally:
            lib().free(C.c_void_p(t))
            if dt.value:
                lib().free(dt)

    def align_timed(self, p, seqs, threads=1):
        bs = [s if isinstance(s, bytes) else s.encode() for s in seqs]
        lens = (C.c_uint64 * max(1, len(bs)))(*[len(b) for b in bs])
        nrec = C.c_uint64()
        sec = lib().oracle_align_timed(self.h, C.byref(p), _cstrs(bs), lens, len(bs), threads, C.byref(nrec))
        return sec, nrec.value

    def close(self):
        if self.h:
            lib().oracle_index_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def lis(X, window=1, a=1.3, b=10.0, cap=10000.0, mer_all=False, seq_all=False, seq_a=None):
    X = np.ascontiguousarray(np.asarray(X, dtype=np.int32).reshape(-1, 2))
    n = len(X)
    out = (C.c_uint32 * max(1, n))()
    L = lib().oracle_lis(X.ctypes.data_as(C.POINTER(C.c_int32)), n, window, int(mer_all), a, b, cap,
                         int(seq_all), a if seq_a is None else seq_a, out)
    return [out[i] for i in range(L)]
