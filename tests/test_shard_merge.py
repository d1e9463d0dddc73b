"""Host side of the index-sharded mode, no GPU needed:
pbgpu_coords_merge merges the shards' per-read record runs in the order of the
whole index, (rs, re, ql) (jf_aligner.cc:148-154) then (sr_index, emit), and
carries each record's kmers_info along."""
import ctypes as C

import numpy as np

from pacbio_amd import pbgpu


def _batch(per_read, keep):
    """per_read: list (one per read) of lists of (rs, re, ql, sr, emit, info) -> CoordsBatch"""
    recs, off, km, kb = [], [0], [], []
    for rl in per_read:
        for (rs, re, ql, sr, emit, info) in sorted(rl):
            r = np.zeros(1, pbgpu.RECORD_DTYPE)[0]
            r["rs"], r["re"], r["ql"], r["sr_index"], r["emit"] = rs, re, ql, sr, emit
            r["info_offset"], r["n_info"] = len(km), len(info)
            km += [m for m, _ in info]
            kb += [b for _, b in info]
            recs.append(r)
        off.append(len(recs))
    rec_a = np.array(recs, dtype=pbgpu.RECORD_DTYPE) if recs else np.zeros(0, pbgpu.RECORD_DTYPE)
    off_a = np.array(off, np.uint64)
    km_a, kb_a = np.array(km or [0], np.int32), np.array(kb or [0], np.int32)
    keep += [rec_a, off_a, km_a, kb_a]
    return pbgpu.CoordsBatch(len(per_read), len(recs), off_a.ctypes.data_as(C.POINTER(C.c_uint64)),
                             rec_a.ctypes.data, len(km), km_a.ctypes.data_as(C.POINTER(C.c_int32)),
                             kb_a.ctypes.data_as(C.POINTER(C.c_int32)))


def test_merge_orders_records_like_the_whole_index():
    keep = []
    a = _batch([[(5, 90, 300, 1, 0, [(1, 17)]), (5, 90, 300, 7, 0, [])], [], [(2, 50, 100, 3, 1, [(4, 40), (2, 20)])]],
               keep)
    b = _batch([[(5, 90, 300, 4, 0, [(9, 99)]), (1, 10, 300, 9, 0, [])], [(7, 70, 10, 12, 0, [])], []], keep)
    parts = (C.POINTER(pbgpu.CoordsBatch) * 2)(C.pointer(a), C.pointer(b))
    out = C.POINTER(pbgpu.CoordsBatch)()
    pbgpu._check(pbgpu.lib().pbgpu_coords_merge(parts, 2, C.byref(out)))
    co = pbgpu.Coords(out)
    assert list(co.read_offsets) == [0, 4, 5, 6]
    key = [(int(r["rs"]), int(r["re"]), int(r["ql"]), int(r["sr_index"])) for r in co.records]
    assert key == [(1, 10, 300, 9), (5, 90, 300, 1), (5, 90, 300, 4), (5, 90, 300, 7), (7, 70, 10, 12), (2, 50, 100, 3)]
    info = [[(int(co.kmers_info[r["info_offset"] + t]), int(co.bases_info[r["info_offset"] + t]))
             for t in range(r["n_info"])] for r in co.records]
    assert info == [[], [(1, 17)], [(9, 99)], [], [], [(4, 40), (2, 20)]]
    co.close()


def test_merge_rejects_mismatched_batches():
    keep = []
    a = _batch([[]], keep)
    b = _batch([[], []], keep)
    parts = (C.POINTER(pbgpu.CoordsBatch) * 2)(C.pointer(a), C.pointer(b))
    out = C.POINTER(pbgpu.CoordsBatch)()
    assert pbgpu.lib().pbgpu_coords_merge(parts, 2, C.byref(out)) == 1  # PBGPU_ERR_INVALID
