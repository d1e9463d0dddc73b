"""ctypes binding of tools/libpbsynth.so (deterministic synthetic workload,
SURVEY.md §8d)."""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


class SynthConfig(C.Structure):
    _fields_ = [("genome_len", C.c_uint64), ("seed", C.c_uint64), ("n_sr", C.c_uint64), ("n_pb", C.c_uint64),
                ("pb_len_mean", C.c_double), ("pb_len_sigma", C.c_double), ("pb_len_min", C.c_uint32),
                ("pb_len_max", C.c_uint32), ("err_ins", C.c_double), ("err_del", C.c_double),
                ("err_sub", C.c_double), ("n_run_rate", C.c_double), ("unitig_k", C.c_uint32),
                ("unitig_mean", C.c_double), ("unitig_min", C.c_uint32), ("sr_max_unitigs", C.c_uint32),
                ("repeat_frac", C.c_double), ("pb_index_base", C.c_uint64)]


class SynthSeqs(C.Structure):
    _fields_ = [("n", C.c_uint64), ("seq", C.c_void_p), ("off", C.POINTER(C.c_uint64)), ("names", C.c_void_p),
                ("name_off", C.POINTER(C.c_uint64))]


PRESETS = {
    # BASELINE.json configs[0]: 100 x 10 kb PB vs 1k SRs, k=17
    "C1": dict(genome_len=1_000_000, n_sr=1000, n_pb=100, pb_len_mean=10000, pb_len_sigma=0.0),
    # configs[1]: E. coli-scale, 50k PB (mean 12 kb) vs 200k SRs, k=17
    "C2": dict(genome_len=4_600_000, n_sr=200_000, n_pb=50_000, pb_len_mean=12000, pb_len_sigma=0.5),
    # configs[2]: yeast-scale, 300k PB vs 1M SRs, k=21
    "C3": dict(genome_len=12_000_000, n_sr=1_000_000, n_pb=300_000, pb_len_mean=12000, pb_len_sigma=0.5),
    # configs[3] (property tests only; the oracle cannot hold its index): chr1-scale, 10M SRs over a
    # 250 Mbp genome with 2% 5-50-copy repeats, PB reads of 15 kb N50 (lognormal mean 12.5 kb, sigma 0.6)
    "C4": dict(genome_len=250_000_000, n_sr=10_000_000, n_pb=2_000_000, pb_len_mean=12500, pb_len_sigma=0.6,
               repeat_frac=0.02),
    # configs[4] (one MI355X, index sharded; property tests only): whole-human scale, 50M SRs (~62 Gbp
    # of text) over a 3.1 Gbp genome with the C4 repeat model, PB reads of 15 kb N50
    "C5": dict(genome_len=3_100_000_000, n_sr=50_000_000, n_pb=20_000_000, pb_len_mean=12500, pb_len_sigma=0.6,
               repeat_frac=0.02),
    # C4's repeat model (2% of the genome in 5-50-copy repeats, PB reads of 15 kb N50) at a size the
    # CPU oracle holds: a 16 Mbp genome at C4's ~50x super-read coverage (800k SRs, ~1 Gbp of text)
    "C4r": dict(genome_len=16_000_000, n_sr=800_000, n_pb=1000, pb_len_mean=12500, pb_len_sigma=0.6,
                repeat_frac=0.02),
    "tiny": dict(genome_len=20_000, n_sr=60, n_pb=8, pb_len_mean=2000, pb_len_sigma=0.0),
    "small": dict(genome_len=200_000, n_sr=1500, n_pb=40, pb_len_mean=6000, pb_len_sigma=0.4),
}


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(os.path.join(_HERE, "libpbsynth.so"))
        L.pbsynth_default.argtypes = [C.POINTER(SynthConfig)]
        L.pbsynth_default.restype = None
        L.pbsynth_make.argtypes = [C.POINTER(SynthConfig), C.c_int, C.POINTER(SynthSeqs), C.POINTER(SynthSeqs),
                                   C.POINTER(C.POINTER(C.c_int32)), C.POINTER(C.c_uint64)]
        L.pbsynth_free.argtypes = [C.POINTER(SynthSeqs)]
        L.pbsynth_free.restype = None
        L.pbsynth_free_ul.argtypes = [C.POINTER(C.c_int32)]
        L.pbsynth_free_ul.restype = None
        L.pbsynth_write_fasta.argtypes = [C.POINTER(SynthSeqs), C.c_char_p, C.c_int]
        L.pbsynth_write_ul.argtypes = [C.POINTER(C.c_int32), C.c_uint64, C.c_char_p]
        _lib = L
    return _lib


class Dataset:
    """Generated workload kept in C buffers; exposes numpy views."""

    def __init__(self, preset="C1", seed=42, threads=8, **over):
        cfg = SynthConfig()
        lib().pbsynth_default(C.byref(cfg))
        for k, v in {**PRESETS[preset], **over}.items():
            setattr(cfg, k, v)
        cfg.seed = seed
        self.cfg = cfg
        self.sr, self.pb = SynthSeqs(), SynthSeqs()
        ul = C.POINTER(C.c_int32)()
        nul = C.c_uint64()
        if lib().pbsynth_make(C.byref(cfg), threads, C.byref(self.sr), C.byref(self.pb), C.byref(ul), C.byref(nul)):
            raise RuntimeError("pbsynth_make failed")
        self._ul = ul
        self.unitig_lengths = np.ctypeslib.as_array(ul, shape=(nul.value,)).copy() if nul.value else np.zeros(0, np.int32)

    @staticmethod
    def _blob(s):
        n = s.n
        off = np.ctypeslib.as_array(s.off, shape=(n + 1,))
        return (C.c_char * int(off[n])).from_address(s.seq), off

    def sr_pointers(self):
        """(names, seqs, lens) as ctypes arrays pointing into the generator's buffers
        (no Python copies: C4 holds 10 Gbp of super-reads)"""
        s = self.sr
        n = s.n
        off = np.ctypeslib.as_array(s.off, shape=(n + 1,))
        noff = np.ctypeslib.as_array(s.name_off, shape=(n,))
        seqp = (off[:-1] + np.uint64(s.seq)).astype(np.uint64)
        namep = (noff + np.uint64(s.names)).astype(np.uint64)
        lens = np.diff(off).astype(np.uint64)
        self._keep_ptrs = (seqp, namep, lens)
        P = C.POINTER(C.c_char_p)
        return (namep.ctypes.data_as(P), seqp.ctypes.data_as(P), lens.ctypes.data_as(C.POINTER(C.c_uint64)), n)

    def pb_blob(self):
        """(bytes-like buffer, offsets) of the concatenated PB reads"""
        return self._blob(self.pb)

    def pb_seqs(self):
        buf, off = self._blob(self.pb)
        raw = bytes(buf)
        return [raw[off[i]:off[i + 1]] for i in range(self.pb.n)]

    def sr_seqs(self):
        buf, off = self._blob(self.sr)
        raw = bytes(buf)
        return [raw[off[i]:off[i + 1]] for i in range(self.sr.n)]

    def _names(self, s):
        out = []
        for i in range(s.n):
            out.append(C.string_at(s.names + int(s.name_off[i])))
        return out

    def sr_names(self):
        return self._names(self.sr)

    def pb_names(self):
        return self._names(self.pb)

    def write(self, d, sr_line=70):
        os.makedirs(d, exist_ok=True)
        lib().pbsynth_write_fasta(C.byref(self.sr), os.path.join(d, "sr.fa").encode(), sr_line)
        lib().pbsynth_write_fasta(C.byref(self.pb), os.path.join(d, "pb.fa").encode(), 0)
        lib().pbsynth_write_ul(self._ul, len(self.unitig_lengths), os.path.join(d, "ul.txt").encode())

    def close(self):
        if self._ul:
            lib().pbsynth_free(C.byref(self.sr))
            lib().pbsynth_free(C.byref(self.pb))
            lib().pbsynth_free_ul(self._ul)
            self._ul = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
