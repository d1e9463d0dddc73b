"""ctypes binding of the pbgpu C ABI (include/pbgpu.h).

Plumbing for tests and bench.py only: the product is libpbgpu.so (HIP kernels
+ C ABI) and the C++ CLI pacbio_amd/bin/jf_aligner.  The classes mirror the
reference objects they replace:

  Index    <- superread_parse() / sequence_psa   (superread_parser.hpp:53-224)
  Aligner  <- coarse_aligner + ::thread          (coarse_aligner.hpp:38-150)
  Coords   <- coords_info_type of a whole batch  (pb_aligner.hpp:103-177)

There is no CPU fallback: if libpbgpu.so is missing or no GPU is usable the
calls raise.
"""
import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PBGPU_LIB") or os.path.join(_HERE, "libpbgpu.so")  # PBGPU_LIB: profiling builds only

PBGPU_OK = 0
STATUS = {0: "OK", 1: "INVALID", 2: "IO", 3: "NOMEM", 4: "DEVICE", 5: "UNSUPPORTED", 6: "INTERNAL"}

# every symbol include/pbgpu.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "pbgpu_abi_version", "pbgpu_last_error", "pbgpu_device_count", "pbgpu_device_synchronize",
    "pbgpu_measure_gather", "pbgpu_measure_gather_shape", "pbgpu_measure_group_shape", "pbgpu_check_reciprocal",
    "pbgpu_index_build_fasta", "pbgpu_index_build", "pbgpu_index_free", "pbgpu_index_get_info",
    "pbgpu_index_sr_name", "pbgpu_index_sr_len",
    "pbgpu_align_params_default", "pbgpu_aligner_create", "pbgpu_aligner_free",
    "pbgpu_align_batch", "pbgpu_coords_free",
    "pbgpu_reads_upload", "pbgpu_reads_free", "pbgpu_align_resident", "pbgpu_download",
    "pbgpu_aligner_get_stats", "pbgpu_aligner_reset_stats", "pbgpu_aligner_set_hit_budget",
    "pbgpu_format_coords", "pbgpu_free_text",
    "pbgpu_aligner_set_details", "pbgpu_download_details", "pbgpu_details_free", "pbgpu_format_details",
    "pbgpu_shard_counts", "pbgpu_shard_counts_download", "pbgpu_shard_counts_upload", "pbgpu_rccl_unique_id",
    "pbgpu_rccl_comm_create", "pbgpu_rccl_comm_free", "pbgpu_shard_counts_allreduce", "pbgpu_align_resident_shard",
    "pbgpu_coords_merge", "pbgpu_rccl_comm_last_bytes",
    "pbgpu_format_device", "pbgpu_text_download", "pbgpu_host_alloc", "pbgpu_host_free", "pbgpu_format_double",
    "pbgpu_index_replicate", "pbgpu_run", "pbgpu_runner_create", "pbgpu_runner_run", "pbgpu_runner_free",
    "pbgpu_index_save", "pbgpu_index_load", "pbgpu_aligner_set_graph",
]


class PbgpuError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"pbgpu {STATUS.get(status, status)}: {msg}")
        self.status = status


class IndexParams(C.Structure):
    _fields_ = [("k", C.c_uint32), ("psa_min", C.c_uint32), ("device", C.c_int32), ("threads", C.c_int32),
                ("fine_k", C.c_uint32), ("shard", C.c_uint32), ("n_shards", C.c_uint32)]


class IndexInfo(C.Structure):
    _fields_ = [("n_sr", C.c_uint64), ("text_len", C.c_uint64), ("n_kmers", C.c_uint64),
                ("n_occurrences", C.c_uint64), ("table_buckets", C.c_uint64), ("device_bytes", C.c_uint64),
                ("build_seconds", C.c_double), ("sr_begin", C.c_uint64), ("sr_end", C.c_uint64),
                ("filter_bytes", C.c_uint64)]


class AlignParams(C.Structure):
    _fields_ = [("k", C.c_uint32), ("stretch_factor", C.c_double), ("stretch_constant", C.c_double),
                ("stretch_cap", C.c_double), ("window_size", C.c_uint32), ("forward", C.c_int32),
                ("max_match", C.c_int32), ("max_count", C.c_int32), ("mers_matching", C.c_double),
                ("bases_matching", C.c_double), ("unitigs_k", C.c_uint32),
                ("unitig_lengths", C.POINTER(C.c_int32)), ("n_unitigs", C.c_uint64), ("fine_k", C.c_uint32)]


class ReadBatch(C.Structure):
    _fields_ = [("n_reads", C.c_uint64), ("seq", C.c_void_p), ("offsets", C.POINTER(C.c_uint64)),
                ("names", C.c_void_p), ("name_offsets", C.POINTER(C.c_uint64))]


class RunParams(C.Structure):
    _fields_ = [("pb_paths", C.POINTER(C.c_char_p)), ("n_pb_paths", C.c_size_t), ("coords_path", C.c_char_p),
                ("details_path", C.c_char_p), ("compact", C.c_int32), ("header", C.c_int32),
                ("zero_match", C.c_int32), ("aligners_per_device", C.c_uint32), ("batch_bases", C.c_uint64),
                ("host_threads", C.c_int32), ("records_fn", C.c_void_p), ("records_user", C.c_void_p),
                ("n_parts", C.c_uint32), ("graph", C.c_void_p)]


class RunStats(C.Structure):
    _fields_ = [("wall_seconds", C.c_double)] + \
               [(n, C.c_uint64) for n in ("n_batches", "n_reads", "n_bases", "n_records", "coords_bytes",
                                          "details_bytes")] + \
               [(n, C.c_double) for n in ("read_seconds", "upload_seconds", "align_seconds", "format_seconds",
                                          "d2h_seconds", "write_seconds", "writer_idle_seconds", "open_seconds",
                                          "close_seconds")] + \
               [(n, C.c_uint64) for n in ("n_device_allocs", "n_device_allocs_late", "n_pinned_allocs",
                                          "n_pinned_allocs_late", "device_alloc_bytes")] + \
               [("alloc_seconds", C.c_double), ("device_peak_bytes", C.c_uint64), ("graph_host_reads", C.c_uint64)]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


RECORD_DTYPE = np.dtype([
    ("rs", "<i4"), ("re", "<i4"), ("qs", "<i4"), ("qe", "<i4"), ("nb_mers", "<i4"),
    ("pb_cons", "<u4"), ("sr_cons", "<u4"), ("pb_cover", "<u4"), ("sr_cover", "<u4"),
    ("ql", "<u4"), ("sr_index", "<u4"), ("read", "<u4"), ("emit", "<u4"), ("flags", "<u4"),
    ("n_info", "<u4"), ("reserved", "<u4"), ("info_offset", "<u8"),
    ("stretch", "<f8"), ("offset", "<f8"), ("avg_err", "<f8")])
assert RECORD_DTYPE.itemsize == 96


class CoordsBatch(C.Structure):
    _fields_ = [("n_reads", C.c_uint64), ("n_records", C.c_uint64), ("read_offsets", C.POINTER(C.c_uint64)),
                ("records", C.c_void_p), ("n_info", C.c_uint64), ("kmers_info", C.POINTER(C.c_int32)),
                ("bases_info", C.POINTER(C.c_int32)), ("graph", C.c_void_p), ("mega_offsets", C.c_void_p),
                ("mega", C.c_void_p), ("mega_units", C.c_void_p), ("mega_host", C.c_void_p)]


# pbgpu_graph_node (create_mega_reads' overlap graph, pbgpu_aligner_set_graph)
GRAPH_NODE_DTYPE = np.dtype([("lpath", "<i4"), ("lstart", "<i4"), ("lprev", "<i4"), ("lunitigs", "<i4"),
                             ("root", "<u4"), ("flags", "<u4")])
assert GRAPH_NODE_DTYPE.itemsize == 24
GRAPH_START, GRAPH_END, GRAPH_HOST = 1, 2, 0x80000000
# pbgpu_mega_read (pbgpu_graph_params.mega_reads)
MEGA_DTYPE = np.dtype([("imp_s", "<f8"), ("imp_e", "<f8"), ("density", "<f8"), ("rs", "<i4"), ("re", "<i4"),
                       ("qs", "<i4"), ("lpath", "<i4"), ("sr_len", "<i4"), ("start_unitig", "<i4"),
                       ("nb_unitigs", "<i4"), ("n_units", "<u4"), ("qend", "<u8"), ("unit_offset", "<u8")])
assert MEGA_DTYPE.itemsize == 72


class GraphParams(C.Structure):
    _fields_ = [("overlap_play", C.c_double), ("nb_errors", C.c_double), ("k_len", C.c_uint32),
                ("maximize_bases", C.c_int32), ("n_sr", C.c_uint64), ("name_offsets", C.POINTER(C.c_uint64)),
                ("name_units", C.POINTER(C.c_uint32)), ("unitig_lengths", C.POINTER(C.c_int32)),
                ("n_unitigs", C.c_uint64), ("mega_reads", C.c_int32), ("tiling", C.c_int32), ("trim", C.c_int32),
                ("min_density", C.c_double), ("min_len", C.c_double)]


class DetailsBatch(C.Structure):
    _fields_ = [("n_reads", C.c_uint64), ("n_lists", C.c_uint64), ("n_hits", C.c_uint64),
                ("read_offsets", C.POINTER(C.c_uint64)), ("list_sr", C.POINTER(C.c_uint32)),
                ("hit_offsets", C.POINTER(C.c_uint64)), ("n_fwd", C.POINTER(C.c_uint32)),
                ("hits", C.POINTER(C.c_int32)), ("in_lis", C.POINTER(C.c_uint8))]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("n_batches", "n_reads", "n_bases", "n_kmers", "n_probes", "n_kept",
                                          "n_hits", "n_chains", "n_lis_tests", "n_records")] + \
               [(n, C.c_double) for n in ("ms_seed", "ms_group", "ms_lis", "ms_fit", "ms_records")] + \
               [("kernel_ms", C.c_double * 8), ("kernel_launches", C.c_uint64 * 8)] + \
               [(n, C.c_uint64) for n in ("g0_kept", "g0_hits", "g0_chains", "l0_hits", "l0_strands",
                                          "n_fine_hits", "n_fine_windows")] + [("ms_fine", C.c_double)] + \
               [(n, C.c_uint64) for n in ("fit_chains", "fit_points", "n_filter", "l0_points")] + \
               [("ms_graph", C.c_double), ("graph_records", C.c_uint64), ("graph_ovf_nodes", C.c_uint64),
                                                                    ("ms_host_order", C.c_double),
                                                                    ("graph_host_reads", C.c_uint64),
                                                                    ("group_refines", C.c_uint64),
                                                                    ("group_hbm_reads", C.c_uint64),
                                                                    ("group_overflow_items", C.c_uint64),
                                                                    ("group_bucketed_reads", C.c_uint64)]

    def as_dict(self):
        d = {n: getattr(self, n) for n, _ in self._fields_ if not n.startswith("kernel_")}
        d["kernel_ms"] = {k: self.kernel_ms[i] for k, i in KERNELS.items()}
        d["kernel_launches"] = {k: self.kernel_launches[i] for k, i in KERNELS.items()}
        return d


# pbgpu.h PBGPU_KERNEL_*: kernels timed individually
KERNELS = {"k_seed": 0, "k_group": 1, "k_lis": 2, "k_coords": 3, "k_rec_sort": 4}


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m pacbio_amd.build`")
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.pbgpu_abi_version.restype = C.c_int
        L.pbgpu_last_error.restype = C.c_char_p
        L.pbgpu_device_count.restype = C.c_int
        L.pbgpu_device_synchronize.argtypes = [C.c_int]
        L.pbgpu_measure_gather.argtypes = [C.c_int, C.c_uint64, C.POINTER(C.c_double)]
        L.pbgpu_measure_gather_shape.argtypes = [C.c_int, C.c_uint64, C.c_uint32, C.POINTER(C.c_double)]
        L.pbgpu_measure_group_shape.argtypes = [C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_double),
                                                C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        if hasattr(L, "pbgpu_check_reciprocal"):  # (absent from older experiment builds)
            L.pbgpu_check_reciprocal.argtypes = [C.c_int, C.c_uint32, C.POINTER(C.c_uint64)]
        L.pbgpu_index_build_fasta.argtypes = [C.POINTER(C.c_char_p), C.c_size_t, C.POINTER(IndexParams), C.POINTER(vp)]
        L.pbgpu_index_build.argtypes = [C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.POINTER(C.c_uint64),
                                        C.c_size_t, C.POINTER(IndexParams), C.POINTER(vp)]
        L.pbgpu_index_free.argtypes = [vp]
        L.pbgpu_index_get_info.argtypes = [vp, C.POINTER(IndexInfo)]
        L.pbgpu_index_sr_name.argtypes = [vp, C.c_uint32, C.c_int]
        L.pbgpu_index_sr_name.restype = C.c_char_p
        L.pbgpu_index_sr_len.argtypes = [vp, C.c_uint32]
        L.pbgpu_index_sr_len.restype = C.c_uint32
        L.pbgpu_align_params_default.argtypes = [C.POINTER(AlignParams)]
        L.pbgpu_align_params_default.restype = None
        L.pbgpu_aligner_create.argtypes = [vp, C.POINTER(AlignParams), C.POINTER(vp)]
        L.pbgpu_aligner_free.argtypes = [vp]
        L.pbgpu_align_batch.argtypes = [vp, C.POINTER(ReadBatch), C.POINTER(C.POINTER(CoordsBatch))]
        L.pbgpu_coords_free.argtypes = [C.POINTER(CoordsBatch)]
        L.pbgpu_reads_upload.argtypes = [vp, C.POINTER(ReadBatch), C.POINTER(vp)]
        L.pbgpu_reads_free.argtypes = [vp]
        L.pbgpu_align_resident.argtypes = [vp, vp]
        L.pbgpu_download.argtypes = [vp, C.POINTER(C.POINTER(CoordsBatch))]
        L.pbgpu_aligner_get_stats.argtypes = [vp, C.POINTER(Stats)]
        L.pbgpu_aligner_reset_stats.argtypes = [vp]
        L.pbgpu_aligner_set_hit_budget.argtypes = [vp, C.c_uint64]
        L.pbgpu_format_coords.argtypes = [vp, C.POINTER(CoordsBatch), C.POINTER(C.c_char_p), C.POINTER(C.c_uint64),
                                          C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p),
                                          C.POINTER(C.c_uint64)]
        L.pbgpu_aligner_set_details.argtypes = [vp, C.c_int]
        L.pbgpu_download_details.argtypes = [vp, C.POINTER(C.POINTER(DetailsBatch))]
        L.pbgpu_details_free.argtypes = [C.POINTER(DetailsBatch)]
        L.pbgpu_format_details.argtypes = [vp, C.POINTER(DetailsBatch), C.POINTER(C.c_char_p), C.c_int,
                                           C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]
        L.pbgpu_shard_counts.argtypes = [vp, vp]
        L.pbgpu_shard_counts_download.argtypes = [vp, C.c_void_p, C.c_uint64]
        L.pbgpu_shard_counts_upload.argtypes = [vp, C.c_void_p, C.c_uint64]
        L.pbgpu_rccl_unique_id.argtypes = [C.c_void_p]
        L.pbgpu_rccl_comm_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.POINTER(vp)]
        L.pbgpu_rccl_comm_free.argtypes = [vp]
        L.pbgpu_rccl_comm_last_bytes.argtypes = [vp]
        L.pbgpu_rccl_comm_last_bytes.restype = C.c_uint64
        L.pbgpu_shard_counts_allreduce.argtypes = [vp, vp]
        L.pbgpu_align_resident_shard.argtypes = [vp, vp]
        L.pbgpu_coords_merge.argtypes = [C.POINTER(C.POINTER(CoordsBatch)), C.c_uint64,
                                         C.POINTER(C.POINTER(CoordsBatch))]
        L.pbgpu_free_text.argtypes = [C.c_void_p]
        L.pbgpu_free_text.restype = None
        L.pbgpu_format_device.argtypes = [vp, vp, C.c_int, C.c_int, C.POINTER(C.c_uint64)]
        L.pbgpu_text_download.argtypes = [vp, C.c_void_p, C.c_uint64]
        L.pbgpu_host_alloc.argtypes = [C.c_uint64, C.POINTER(C.c_void_p)]
        L.pbgpu_host_free.argtypes = [C.c_void_p]
        L.pbgpu_format_double.argtypes = [C.c_double, C.c_char_p]
        L.pbgpu_format_double.restype = C.c_int
        L.pbgpu_index_replicate.argtypes = [vp, C.c_int, C.POINTER(vp)]
        L.pbgpu_index_save.argtypes = [vp, C.c_char_p, C.c_char_p]
        L.pbgpu_index_load.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.POINTER(vp)]
        L.pbgpu_run.argtypes = [C.POINTER(vp), C.c_size_t, C.POINTER(AlignParams), C.POINTER(RunParams),
                                C.POINTER(RunStats)]
        L.pbgpu_runner_create.argtypes = [C.POINTER(vp), C.c_size_t, C.POINTER(AlignParams), C.POINTER(RunParams),
                                          C.POINTER(vp)]
        L.pbgpu_runner_run.argtypes = [vp, C.POINTER(RunParams), C.POINTER(RunStats)]
        L.pbgpu_runner_free.argtypes = [vp]
        _lib = L
    return _lib


def _check(st):
    if st != PBGPU_OK:
        raise PbgpuError(st, lib().pbgpu_last_error().decode(errors="replace"))


def device_synchronize(device=0):
    _check(lib().pbgpu_device_synchronize(device))


def measure_gather(device=0, buffer_bytes=64 << 30, unit_bytes=64):
    """GB/s of uniformly random 64-B sector loads (B_rand), or of random 512-B runs
    read as 64 consecutive 8-B words (unit_bytes=512), over a buffer of buffer_bytes."""
    g = C.c_double()
    _check(lib().pbgpu_measure_gather_shape(device, buffer_bytes, unit_bytes, C.byref(g)))
    return g.value


def measure_group_shape(device=0, buffer_bytes=64 << 30, mode=2):
    """k_group's occurrence-read shape (pbgpu_measure_group_shape): mode 0 = pass 0's 4-B ids,
    1 = pass 1's 8-B words, 2 = both passes over the same runs.  Returns a dict: sector-byte
    rate (GB/s) and, per launch, the 64-B sectors / 128-B lines spanned and the algorithmic
    bytes (the known counts FETCH_SIZE is read against)."""
    g, s64, l128, alg = C.c_double(), C.c_uint64(), C.c_uint64(), C.c_uint64()
    _check(lib().pbgpu_measure_group_shape(device, buffer_bytes, mode, C.byref(g), C.byref(s64), C.byref(l128),
                                           C.byref(alg)))
    return {"mode": mode, "sector_gbs": g.value, "sectors64_per_launch": s64.value,
            "lines128_per_launch": l128.value, "alg_bytes_per_launch": alg.value}


def check_reciprocal(device=0, n_max=1 << 24):
    """Mismatches of the fit's device reciprocal against __ddiv_rn(1.0, n), n in [1, n_max]."""
    m = C.c_uint64()
    _check(lib().pbgpu_check_reciprocal(device, n_max, C.byref(m)))
    return m.value


def _cstrs(items):
    arr = (C.c_char_p * max(1, len(items)))()
    for i, s in enumerate(items):
        arr[i] = s if isinstance(s, bytes) else s.encode()
    return arr


def _addr(blob):
    """address of a bytes object or a ctypes buffer (kept alive by the caller)"""
    if isinstance(blob, (bytes, bytearray)):
        return C.cast(C.c_char_p(bytes(blob)), C.c_void_p).value if isinstance(blob, bytearray) else \
            C.cast(C.c_char_p(blob), C.c_void_p).value
    return C.addressof(blob)


def _pack_reads(seqs):
    """list of str/bytes -> (blob bytes, offsets uint64)"""
    bs = [s if isinstance(s, bytes) else s.encode() for s in seqs]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    np.cumsum([len(b) for b in bs], out=off[1:])
    return b"".join(bs), off


class Index:
    def __init__(self, handle):
        self.h = handle

    @classmethod
    def from_fasta(cls, paths, k, psa_min=13, device=0, threads=0, fine_k=0, shard=0, n_shards=1):
        p = IndexParams(k, psa_min, device, threads, fine_k, shard, n_shards)
        h = C.c_void_p()
        _check(lib().pbgpu_index_build_fasta(_cstrs(paths), len(paths), C.byref(p), C.byref(h)))
        return cls(h)

    @classmethod
    def from_records(cls, names, seqs, k, psa_min=13, device=0, threads=0, fine_k=0, shard=0, n_shards=1):
        p = IndexParams(k, psa_min, device, threads, fine_k, shard, n_shards)
        bs = [s if isinstance(s, bytes) else s.encode() for s in seqs]
        lens = (C.c_uint64 * max(1, len(bs)))(*[len(b) for b in bs])
        h = C.c_void_p()
        _check(lib().pbgpu_index_build(_cstrs(names), _cstrs(bs), lens, len(bs), C.byref(p), C.byref(h)))
        return cls(h)

    @classmethod
    def from_pointers(cls, names, seqs, lens, n, k, psa_min=13, device=0, threads=0, fine_k=0, shard=0, n_shards=1):
        """pbgpu_index_build on caller-owned C arrays (names / seqs: char* arrays, lens: uint64)"""
        p = IndexParams(k, psa_min, device, threads, fine_k, shard, n_shards)
        h = C.c_void_p()
        _check(lib().pbgpu_index_build(names, seqs, lens, n, C.byref(p), C.byref(h)))
        return cls(h)

    def replicate(self, device):
        """pbgpu_index_replicate: the same index on another device (or a second copy on this one)"""
        h = C.c_void_p()
        _check(lib().pbgpu_index_replicate(self.h, device, C.byref(h)))
        return Index(h)

    def save(self, path, tag=""):
        """pbgpu_index_save: the whole index (host and device arrays) to `path`"""
        _check(lib().pbgpu_index_save(self.h, os.fsencode(path), tag.encode()))

    @classmethod
    def load(cls, path, device=0, tag=""):
        """pbgpu_index_load: an index saved by save(), rebuilt on `device` (PBGPU_ERR_IO if
        the file is missing, truncated or saved with another tag)"""
        h = C.c_void_p()
        _check(lib().pbgpu_index_load(os.fsencode(path), device, tag.encode(), C.byref(h)))
        return cls(h)

    def info(self):
        i = IndexInfo()
        _check(lib().pbgpu_index_get_info(self.h, C.byref(i)))
        return {n: getattr(i, n) for n, _ in i._fields_}

    def sr_name(self, i, bwd=False):
        r = lib().pbgpu_index_sr_name(self.h, i, 1 if bwd else 0)
        return None if r is None else r.decode()

    def close(self):
        if self.h:
            lib().pbgpu_index_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def align_params(k=17, stretch_factor=1.3, stretch_constant=10, stretch_cap=10000.0, window_size=1,
                 forward=False, max_match=False, max_count=5000, mers_matching=0.0, bases_matching=17.0,
                 unitigs_k=0, unitig_lengths=None, fine_k=0):
    p = AlignParams()
    lib().pbgpu_align_params_default(C.byref(p))
    p.k = k; p.stretch_factor = stretch_factor; p.stretch_constant = stretch_constant
    p.stretch_cap = stretch_cap; p.window_size = window_size; p.forward = int(bool(forward))
    p.max_match = int(bool(max_match)); p.max_count = max_count; p.mers_matching = mers_matching
    p.bases_matching = bases_matching; p.unitigs_k = unitigs_k; p.fine_k = fine_k
    keep = None
    if unitig_lengths is not None:
        keep = np.ascontiguousarray(unitig_lengths, dtype=np.int32)
        p.unitig_lengths = keep.ctypes.data_as(C.POINTER(C.c_int32))
        p.n_unitigs = len(keep)
    return p, keep


class Coords:
    """Host copy of one batch of records (owns the C allocation)."""

    def __init__(self, ptr):
        self.ptr = ptr
        c = ptr.contents
        n, nr = c.n_reads, c.n_records
        self.n_reads, self.n_records = n, nr
        self.read_offsets = np.ctypeslib.as_array(c.read_offsets, shape=(n + 1,)).copy() if n + 1 else np.zeros(1, np.uint64)
        if nr:
            buf = (C.c_char * (nr * RECORD_DTYPE.itemsize)).from_address(c.records)
            self.records = np.frombuffer(buf, dtype=RECORD_DTYPE).copy()
        else:
            self.records = np.zeros(0, dtype=RECORD_DTYPE)
        self.mega = None  # (offsets per read, MEGA_DTYPE records, units, host flags) with the device mega-reads
        if c.mega_offsets:
            moff = np.ctypeslib.as_array(C.cast(c.mega_offsets, C.POINTER(C.c_uint64)), shape=(n + 1,)).copy()
            nm = int(moff[-1])
            recs = np.zeros(0, MEGA_DTYPE)
            if nm:
                mbuf = (C.c_char * (nm * MEGA_DTYPE.itemsize)).from_address(c.mega)
                recs = np.frombuffer(mbuf, dtype=MEGA_DTYPE).copy()
            nu = int((recs["unit_offset"] + recs["n_units"]).max()) if nm else 0
            units = (np.ctypeslib.as_array(C.cast(c.mega_units, C.POINTER(C.c_uint32)), shape=(nu,)).copy()
                     if nu else np.zeros(0, np.uint32))
            host = np.ctypeslib.as_array(C.cast(c.mega_host, C.POINTER(C.c_uint8)), shape=(n,)).copy() if n else \
                np.zeros(0, np.uint8)
            self.mega = (moff, recs, units, host)
        self.graph = None  # pbgpu_graph_node per record (GRAPH_NODE_DTYPE) when the aligner's graph is on
        if c.graph and nr:
            gbuf = (C.c_char * (nr * GRAPH_NODE_DTYPE.itemsize)).from_address(c.graph)
            self.graph = np.frombuffer(gbuf, dtype=GRAPH_NODE_DTYPE).copy()
        if c.n_info:
            self.kmers_info = np.ctypeslib.as_array(c.kmers_info, shape=(c.n_info,)).copy()
            self.bases_info = np.ctypeslib.as_array(c.bases_info, shape=(c.n_info,)).copy()
        else:
            self.kmers_info = np.zeros(0, np.int32)
            self.bases_info = np.zeros(0, np.int32)

    def format(self, index, headers, lens, compact=True, header=False, zero_match=False, threads=0):
        t = C.c_void_p()
        tl = C.c_uint64()
        lens_a = (C.c_uint64 * max(1, len(lens)))(*[int(x) for x in lens])
        _check(lib().pbgpu_format_coords(index.h, self.ptr, _cstrs(headers), lens_a, int(compact), int(header),
                                         int(zero_match), threads, C.byref(t), C.byref(tl)))
        try:
            return C.string_at(t, tl.value).decode()
        finally:
            lib().pbgpu_free_text(t)

    def close(self):
        if self.ptr:
            lib().pbgpu_coords_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Aligner:
    def __init__(self, index, **kw):
        self.index = index
        self.params, self._ul = align_params(**kw)
        h = C.c_void_p()
        _check(lib().pbgpu_aligner_create(index.h, C.byref(self.params), C.byref(h)))
        self.h = h

    def align(self, seqs):
        blob, off = _pack_reads(seqs)
        b = ReadBatch(len(seqs), _addr(blob), off.ctypes.data_as(C.POINTER(C.c_uint64)), None, None)
        out = C.POINTER(CoordsBatch)()
        _check(lib().pbgpu_align_batch(self.h, C.byref(b), C.byref(out)))
        return Coords(out)

    def upload(self, seqs=None, blob=None, offsets=None, names=None):
        """names: read names (header up to the first whitespace) for format_device"""
        if seqs is not None:
            blob, offsets = _pack_reads(seqs)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        b = ReadBatch(len(offsets) - 1, _addr(blob), offsets.ctypes.data_as(C.POINTER(C.c_uint64)), None, None)
        if names is not None:
            nblob, noff = _pack_reads(names)
            b.names = _addr(nblob)
            b.name_offsets = noff.ctypes.data_as(C.POINTER(C.c_uint64))
        r = C.c_void_p()
        _check(lib().pbgpu_reads_upload(self.h, C.byref(b), C.byref(r)))
        return ResidentReads(r)

    def format_device(self, reads, compact=True, zero_match=False):
        """pbgpu_format_device + pbgpu_text_download: the last alignment's coords text,
        formatted on the device"""
        n = C.c_uint64()
        _check(lib().pbgpu_format_device(self.h, reads.h, int(compact), int(zero_match), C.byref(n)))
        buf = C.create_string_buffer(n.value + 1)
        _check(lib().pbgpu_text_download(self.h, buf, n.value))
        return buf.raw[:n.value].decode()

    def align_resident(self, reads):
        _check(lib().pbgpu_align_resident(self.h, reads.h))

    def download(self):
        out = C.POINTER(CoordsBatch)()
        _check(lib().pbgpu_download(self.h, C.byref(out)))
        return Coords(out)

    def stats(self):
        s = Stats()
        _check(lib().pbgpu_aligner_get_stats(self.h, C.byref(s)))
        return s.as_dict()

    def reset_stats(self):
        _check(lib().pbgpu_aligner_reset_stats(self.h))

    def set_graph(self, names, unitig_lengths, k_len, overlap_play=1.3, nb_errors=3.0, maximize_bases=False,
                  mega_reads=False, tiling="greedy", trim=False, min_density=0.029, min_len=100.0):
        """pbgpu_aligner_set_graph: create_mega_reads' overlap graph after every alignment
        (and with mega_reads the components, tiling and printed paths too).
        names: per super-read of the index its unitig list (id << 1 | R); None turns it off."""
        if names is None:
            _check(lib().pbgpu_aligner_set_graph(self.h, None))
            return
        off = np.zeros(len(names) + 1, np.uint64)
        off[1:] = np.cumsum([len(u) for u in names])
        units = np.ascontiguousarray(np.concatenate([np.asarray(u, np.uint32) for u in names]) if int(off[-1])
                                     else np.zeros(1, np.uint32), dtype=np.uint32)
        ul = np.ascontiguousarray(unitig_lengths, dtype=np.int32)
        self._graph_keep = (off, units, ul)
        til = {"none": 0, "greedy": 1, "maximal": 2, "weighted": 3}[tiling]
        g = GraphParams(float(overlap_play), float(nb_errors), int(k_len), int(bool(maximize_bases)), len(names),
                        off.ctypes.data_as(C.POINTER(C.c_uint64)), units.ctypes.data_as(C.POINTER(C.c_uint32)),
                        ul.ctypes.data_as(C.POINTER(C.c_int32)), len(ul), int(bool(mega_reads)), til, int(bool(trim)),
                        float(min_density), float(min_len))
        _check(lib().pbgpu_aligner_set_graph(self.h, C.byref(g)))


    def shard_counts(self, reads):
        """Sharded index, step 1: this shard's saturated k-mer counts of the batch
        into the aligner's count buffer."""
        _check(lib().pbgpu_shard_counts(self.h, reads.h))

    def counts_download(self, n_bases):
        out = np.empty(n_bases, dtype=np.uint32)
        _check(lib().pbgpu_shard_counts_download(self.h, out.ctypes.data, n_bases))
        return out

    def counts_upload(self, counts):
        c = np.ascontiguousarray(counts, dtype=np.uint32)
        _check(lib().pbgpu_shard_counts_upload(self.h, c.ctypes.data, len(c)))

    def counts_allreduce(self, comm):
        """Step 2 over RCCL: sum the count buffers of all ranks in place."""
        _check(lib().pbgpu_shard_counts_allreduce(self.h, comm.h))

    def align_resident_shard(self, reads):
        """Sharded index, step 3: the rest of the path with the summed counts."""
        _check(lib().pbgpu_align_resident_shard(self.h, reads.h))

    def set_details(self, on=True):
        _check(lib().pbgpu_aligner_set_details(self.h, int(bool(on))))

    def download_details(self):
        out = C.POINTER(DetailsBatch)()
        _check(lib().pbgpu_download_details(self.h, C.byref(out)))
        return Details(out)

    def set_hit_budget(self, hits):
        _check(lib().pbgpu_aligner_set_hit_budget(self.h, C.c_uint64(int(hits))))

    def close(self):
        if self.h:
            lib().pbgpu_aligner_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def stream_cuts(offsets, S):
    """Read-range boundaries [c0=0, c1, ..., cS=n] cutting a batch into S contiguous
    ranges of about equal bases (non-decreasing; an empty range gets no aligner)."""
    off = np.asarray(offsets, dtype=np.uint64)
    n = len(off) - 1
    cuts = [0] + [int(np.searchsorted(off, off[-1] * np.uint64(i) // np.uint64(S), side="left"))
                  for i in range(1, S)] + [n]
    for i in range(1, len(cuts)):
        cuts[i] = min(max(cuts[i], cuts[i - 1]), n)
    return cuts


class StreamAligner:
    """One batch spread over S aligners (own HIP stream and buffers each) that
    share one index, each driven by its own host thread.  A single aligner
    leaves the GPU idle while its host waits on the sub-batch sizing copies
    and in each kernel's tail; a second stream fills those gaps (C2: 122.4 ->
    113.3 ms a step at S=2, 118.2 at S=3; tools/exp_streams.py).

    Reads are cut into S contiguous ranges of about equal bases, so the
    parts' records, concatenated, are the batch's records in read order:
    `format` output is byte-identical to one aligner's."""

    def __init__(self, index, streams=2, **kw):
        if streams < 1:
            raise ValueError("streams must be >= 1")
        self.index = index
        self.aligners = [Aligner(index, **kw) for _ in range(streams)]

    def upload(self, seqs=None, blob=None, offsets=None):
        if seqs is not None:
            blob, offsets = _pack_reads(seqs)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(off) - 1
        S = len(self.aligners)
        cuts = stream_cuts(off, S)
        raw = memoryview(blob if isinstance(blob, (bytes, bytearray)) else bytes(blob))
        parts = []
        for j, (lo, hi) in enumerate(zip(cuts[:-1], cuts[1:])):
            if hi > lo:
                sub_off = off[lo:hi + 1] - off[lo]
                parts.append((j, lo, hi, self.aligners[j].upload(blob=bytes(raw[int(off[lo]):int(off[hi])]),
                                                                 offsets=sub_off)))
        return parts

    def align_resident(self, parts):
        errs = []

        def run(al, r):
            try:
                al.align_resident(r)
            except Exception as e:  # re-raised on the caller's thread
                errs.append(e)
        th = [threading.Thread(target=run, args=(self.aligners[j], r)) for j, _, _, r in parts]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]

    def download(self, parts):
        return [(lo, hi, self.aligners[j].download()) for j, lo, hi, _ in parts]

    def free(self, parts):
        for _, _, _, r in parts:
            r.close()

    def format(self, coords_parts, headers, lens, **kw):
        return "".join(c.format(self.index, headers[lo:hi], lens[lo:hi], **kw) for lo, hi, c in coords_parts)

    def stats(self):
        """Counters and kernel times summed over the aligners (kernel_ms / kernel_launches
        stay a per-launch mean when divided)."""
        out = None
        for al in self.aligners:
            s = al.stats()
            if out is None:
                out = s
                continue
            for k, v in s.items():
                if isinstance(v, dict):
                    for kk, vv in v.items():
                        out[k][kk] += vv
                else:
                    out[k] += v
        return out

    def reset_stats(self):
        for al in self.aligners:
            al.reset_stats()

    def set_hit_budget(self, hits):
        for al in self.aligners:
            al.set_hit_budget(hits)

    def close(self):
        for al in self.aligners:
            al.close()


def _run_params(pb_paths, coords_path, details_path=None, compact=True, header=True, zero_match=False,
                aligners_per_device=2, batch_bases=0, host_threads=0, n_parts=0):
    paths = _cstrs([p if isinstance(p, bytes) else str(p).encode() for p in pb_paths])
    rp = RunParams(paths, len(pb_paths), coords_path.encode() if coords_path else None,
                   details_path.encode() if details_path else None, int(compact), int(header), int(zero_match),
                   aligners_per_device, int(batch_bases), host_threads, None, None, int(n_parts))
    return rp, paths


def _index_handles(indexes):
    if isinstance(indexes, Index):
        indexes = [indexes]
    return (C.c_void_p * len(indexes))(*[ix.h.value if isinstance(ix.h, C.c_void_p) else ix.h for ix in indexes])


_RUN_KEYS = ("details_path", "compact", "header", "zero_match", "aligners_per_device", "batch_bases", "host_threads",
             "n_parts")


def run(indexes, pb_paths, coords_path, **kw):
    """pbgpu_run: PacBio files -> coords file, on every listed index (one per device, repeats allowed).
    Returns the run's stage statistics."""
    rkw = {k: kw.pop(k) for k in list(kw) if k in _RUN_KEYS}
    p, keep = align_params(**kw)
    rp, paths = _run_params(pb_paths, coords_path, **rkw)
    st = RunStats()
    hs = _index_handles(indexes)
    _check(lib().pbgpu_run(hs, len(hs), C.byref(p), C.byref(rp), C.byref(st)))
    del keep
    return st.as_dict()


class Runner:
    """pbgpu_runner: the driver's aligners and pinned buffers kept across runs."""

    def __init__(self, indexes, aligners_per_device=2, batch_bases=0, details=False, n_parts=0, **align_kw):
        self._p, self._keep = align_params(**align_kw)
        self.details = details
        rp, _ = _run_params([], None, details_path="-" if details else None, aligners_per_device=aligners_per_device,
                            batch_bases=batch_bases, n_parts=n_parts)
        hs = _index_handles(indexes)
        h = C.c_void_p()
        _check(lib().pbgpu_runner_create(hs, len(hs), C.byref(self._p), C.byref(rp), C.byref(h)))
        self.h = h

    def run(self, pb_paths, coords_path, details_path=None, compact=True, header=True, zero_match=False,
            host_threads=0):
        rp, paths = _run_params(pb_paths, coords_path, details_path, compact, header, zero_match, 0, 0, host_threads)
        st = RunStats()
        _check(lib().pbgpu_runner_run(self.h, C.byref(rp), C.byref(st)))
        return st.as_dict()

    def close(self):
        if self.h:
            lib().pbgpu_runner_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rccl_unique_id():
    buf = (C.c_uint8 * 128)()
    _check(lib().pbgpu_rccl_unique_id(buf))
    return bytes(buf)


class RcclComm:
    """An RCCL communicator (one per rank) for the sharded-index count exchange."""

    def __init__(self, device, n_ranks, rank, uid):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        h = C.c_void_p()
        _check(lib().pbgpu_rccl_comm_create(device, n_ranks, rank, buf, C.byref(h)))
        self.h = h

    def last_bytes(self):
        """payload of the last count all-reduce on this rank (2 B a read base when packed)"""
        return lib().pbgpu_rccl_comm_last_bytes(self.h)

    def close(self):
        if self.h:
            lib().pbgpu_rccl_comm_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def merge_coords(parts):
    """pbgpu_coords_merge: the shards' batches of one read batch, merged per read."""
    arr = (C.POINTER(CoordsBatch) * len(parts))(*[p.ptr for p in parts])
    out = C.POINTER(CoordsBatch)()
    _check(lib().pbgpu_coords_merge(arr, len(parts), C.byref(out)))
    return Coords(out)


class Details:
    """--details lists of the last alignment (owns the C allocation)."""

    def __init__(self, ptr):
        self.ptr = ptr

    def format(self, index, headers, threads=0):
        t = C.c_void_p()
        tl = C.c_uint64()
        _check(lib().pbgpu_format_details(index.h, self.ptr, _cstrs(headers), threads, C.byref(t), C.byref(tl)))
        try:
            return C.string_at(t, tl.value).decode()
        finally:
            lib().pbgpu_free_text(t)

    def close(self):
        if self.ptr:
            lib().pbgpu_details_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ResidentReads:
    def __init__(self, h):
        self.h = h

    def close(self):
        if self.h:
            lib().pbgpu_reads_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def parse_unitigs(name):
    """super_read_name::parse (super_read_name.cc:74-90) for the synthetic names: 12F_13R -> [24, 27]"""
    out = []
    for tok in name.split("_"):
        digits = tok.rstrip("FR")
        if not digits.isdigit():
            return []
        out.append(int(digits) << 1 | (tok.endswith("R")))
    return out
